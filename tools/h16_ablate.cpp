// Timing harness for wv_bf_h16_kernel variants (tools/h16_ablate.sh): the
// whole exact pipeline through the C ABI (wv_search_batch_device with kernel
// timing) on a uniform [0,1) corpus; each variant binary links its own
// wv_h16.o built with ablation defines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/wvgpu.h"

// debug builds (-DWV_BF_DBG_ITERS) export wave-level counts: tiles, extraction rounds
extern "C" void wv_dbg_read(unsigned long long* out) __attribute__((weak));

int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
    const int nq = argc > 2 ? atoi(argv[2]) : 10000;
    const int D = argc > 3 ? atoi(argv[3]) : 128;
    const char* name = argc > 4 ? argv[4] : "h16";
    std::vector<float> hx(N * D), hq((size_t)nq * D);
    uint64_t st = 88172645463325252ull;
    auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (float)(st >> 40) * (1.0f / 16777216.0f); };
    for (auto& v : hx) v = rnd();
    for (auto& v : hq) v = rnd();
    wv_config cfg;
    wv_config_default(&cfg);
    wv_index* ix = nullptr;
    if (wv_index_create(D, WV_L2_SQUARED, &cfg, N, &ix)) { printf("create: %s\n", wv_last_error()); return 1; }
    if (wv_index_upload_vectors(ix, hx.data(), N, 0)) { printf("upload: %s\n", wv_last_error()); return 1; }
    const int ld = wv_index_query_ld(ix);
    std::vector<float> hqp((size_t)nq * ld, 0.f);
    for (int i = 0; i < nq; ++i)
        for (int k = 0; k < D; ++k) hqp[(size_t)i * ld + k] = hq[(size_t)i * D + k];
    float* dq; uint64_t* di; float* dd; int32_t* dn;
    hipMalloc(&dq, hqp.size() * 4); hipMalloc(&di, (size_t)nq * 10 * 8); hipMalloc(&dd, (size_t)nq * 10 * 4);
    hipMalloc(&dn, (size_t)nq * 4);
    hipMemcpy(dq, hqp.data(), hqp.size() * 4, hipMemcpyHostToDevice);
    wv_index_set_timing(ix, 1);
    hipStream_t s; hipStreamCreate(&s);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) wv_search_batch_device(ix, dq, nq, 10, 0, nullptr, 0, 0, WV_MODE_EXACT, di, dd, dn, s);
    hipStreamSynchronize(s);
    float km = 0, kf = 0, ks = 0, wall = 0;
    const int it = 5;
    for (int r = 0; r < it; ++r) {
        hipEventRecord(a, s);
        if (wv_search_batch_device(ix, dq, nq, 10, 0, nullptr, 0, 0, WV_MODE_EXACT, di, dd, dn, s)) {
            printf("search: %s\n", wv_last_error()); return 1;
        }
        hipEventRecord(b, s);
        hipStreamSynchronize(s);
        float m, f, h, sd, w;
        wv_last_kernel_times(ix, &m, &f, &h);
        wv_last_seed_time(ix, &sd);
        hipEventElapsedTime(&w, a, b);
        km += m; kf += f; ks += sd; wall += w;
    }
    // one more batch with the fallback on: WV_ABLATE_NO_FALLBACK skips (and
    // does not count) the uncertified queries
    unsetenv("WV_ABLATE_NO_FALLBACK");
    wv_search_batch_device(ix, dq, nq, 10, 0, nullptr, 0, 0, WV_MODE_EXACT, di, dd, dn, s);
    hipStreamSynchronize(s);
    uint64_t de, ex, fb;
    wv_last_batch_stats(ix, &de, &ex, &fb);
    std::vector<uint64_t> ids(10);
    hipMemcpy(ids.data(), di, 80, hipMemcpyDeviceToHost);
    printf("%-16s N=%llu nq=%d D=%d  main %.3f ms  seed %.3f ms  finalize %.3f ms  batch %.3f ms  (%.0f TF main) fb=%llu ids0=%llu,%llu\n",
           name, (unsigned long long)N, nq, D, km / it, ks / it, kf / it, wall / it,
           2.0 * D * N * nq / (km / it * 1e-3) / 1e12, (unsigned long long)fb, (unsigned long long)ids[0],
           (unsigned long long)ids[1]);
    if (wv_dbg_read) {
        // (summed over the 2 warm-up + `it` timed batches + the fallback-counting one)
        unsigned long long c[4] = {0, 0, 0, 0};
        wv_dbg_read(c);
        const double nb = 3.0 + it;
        printf("%-16s per batch: wave-tiles %.0f  extraction calls %.0f  wave rounds %.0f  lane rounds %.0f  "
               "(calls per wave-tile %.3f, lanes per round %.2f)\n", name, c[0] / nb, c[3] / nb, c[1] / nb, c[2] / nb,
               c[0] ? (double)c[3] / (double)c[0] : 0.0, c[1] ? (double)c[2] / (double)c[1] : 0.0);
    }
    wv_index_destroy(ix);
    return 0;
}
