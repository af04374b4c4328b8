// HNSW latency harness (tools/hnsw_latency.sh): the C1 graph shape (1M x 128
// SIFT-shaped rows, M=64, efConstruction=128, GPU-built) searched at ef=64 with
// device-resident batches of 1 .. 10000 queries through wv_search_batch_device.
// Prints per batch size the launch-to-completion time, expansions per query and
// time per expansion; a -DWV_HNSW_STAMPS build of wv_hnsw.o also reports the
// expansion loop's per-phase share (wv_hnsw_stamps_read).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/wvgpu.h"

extern "C" void wv_hnsw_stamps_read(unsigned long long* out, int reset) __attribute__((weak));

static uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static float uni(uint64_t s, uint64_t i) { return (float)((mix(s * 0x100000001B3ull + i) >> 40) + 0.5) / 16777216.0f; }
static float gau(uint64_t s, uint64_t i) {
    const float u1 = uni(s, 2 * i), u2 = uni(s, 2 * i + 1);
    return std::sqrt(-2.f * std::log(u1)) * std::cos(6.2831853f * u2);
}

// SIFT-shaped rows (bench.py counter_sift's recipe: 1024 centres, 24-d latent
// spread, isotropic noise, rounded and clipped at 0)
static void sift_rows(uint64_t seed, uint64_t n, int D, std::vector<float>& out) {
    const int C = 1024, L = 24;
    static std::vector<float> centres, basis;
    if (centres.empty()) {
        centres.resize((size_t)C * D);
        basis.resize((size_t)D * L);
        for (size_t i = 0; i < centres.size(); ++i) centres[i] = 60.f * uni(77, i);
        for (size_t i = 0; i < basis.size(); ++i) basis[i] = gau(78, i);
    }
    out.resize(n * D);
#pragma omp parallel for
    for (int64_t r = 0; r < (int64_t)n; ++r) {
        const int c = (int)(uni(seed + 2000, r) * C) % C;
        float z[24];
        for (int l = 0; l < L; ++l) z[l] = gau(seed + 3000, (uint64_t)r * L + l);
        for (int d = 0; d < D; ++d) {
            float s = 0.f;
            for (int l = 0; l < L; ++l) s += z[l] * basis[(size_t)d * L + l];
            const float x = centres[(size_t)c * D + d] + 12.f * s + 3.f * gau(seed + 4000, (uint64_t)r * D + d);
            out[(size_t)r * D + d] = std::max(0.f, std::rint(x));
        }
    }
}

int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
    const int D = argc > 2 ? atoi(argv[2]) : 128;
    const char* name = argc > 3 ? argv[3] : "hnsw";
    const int ef = 64, k = 10;
    std::vector<float> hx, hq;
    sift_rows(1, N, D, hx);
    sift_rows(2, 10000, D, hq);
    wv_config cfg;
    wv_config_default(&cfg);
    cfg.max_connections = 64;
    cfg.ef = ef;
    wv_index* ix = nullptr;
    if (wv_index_create(D, WV_L2_SQUARED, &cfg, N, &ix)) { printf("create: %s\n", wv_last_error()); return 1; }
    if (wv_index_upload_vectors(ix, hx.data(), N, 0)) { printf("upload: %s\n", wv_last_error()); return 1; }
    const auto b0 = std::chrono::steady_clock::now();
    if (wv_index_build_graph(ix, 128, 1, 64)) { printf("build: %s\n", wv_last_error()); return 1; }
    printf("%s: graph built in %.1f s\n", name,
           std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count());
    fflush(stdout);
    const int ld = wv_index_query_ld(ix);
    const int NQ = 10000;
    std::vector<float> hqp((size_t)NQ * ld, 0.f);
    for (int i = 0; i < NQ; ++i)
        for (int d = 0; d < D; ++d) hqp[(size_t)i * ld + d] = hq[(size_t)i * D + d];
    float* dq; uint64_t* di; float* dd; int32_t* dn;
    hipMalloc(&dq, hqp.size() * 4); hipMalloc(&di, (size_t)NQ * k * 8); hipMalloc(&dd, (size_t)NQ * k * 4);
    hipMalloc(&dn, (size_t)NQ * 4);
    hipMemcpy(dq, hqp.data(), hqp.size() * 4, hipMemcpyHostToDevice);
    wv_index_set_timing(ix, 1);
    hipStream_t s; hipStreamCreate(&s);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) wv_search_batch_device(ix, dq, NQ, k, ef, nullptr, 0, 0, WV_MODE_HNSW, di, dd, dn, s);
    hipStreamSynchronize(s);
    const int sizes[] = {1, 8, 32, 64, 256, 1024, 4096, 10000};
    for (int nq : sizes) {
        const int it = nq <= 64 ? 40 : 10;
        unsigned long long st[16] = {};
        if (wv_hnsw_stamps_read) wv_hnsw_stamps_read(st, 1);
        std::vector<float> wall, kern;
        uint64_t de = 0, ex = 0, fb = 0, de_sum = 0, ex_sum = 0;
        for (int r = 0; r < it; ++r) {
            // a different slice of the queries each time (no cache reuse)
            const int q0 = (int)(((uint64_t)r * 7919 * nq) % (uint64_t)(NQ - nq + 1));
            hipEventRecord(a, s);
            if (wv_search_batch_device(ix, dq + (size_t)q0 * ld, nq, k, ef, nullptr, 0, 0, WV_MODE_HNSW, di, dd, dn, s)) {
                printf("search: %s\n", wv_last_error()); return 1;
            }
            hipEventRecord(b, s);
            hipStreamSynchronize(s);
            float w, m, f, h;
            hipEventElapsedTime(&w, a, b);
            wv_last_kernel_times(ix, &m, &f, &h);
            wall.push_back(w);
            kern.push_back(h);
            wv_last_batch_stats(ix, &de, &ex, &fb);
            de_sum += de;
            ex_sum += ex;
        }
        std::sort(wall.begin(), wall.end());
        std::sort(kern.begin(), kern.end());
        const double exq = (double)ex_sum / ((double)it * nq), deq = (double)de_sum / ((double)it * nq);
        const double km = kern[it / 2];
        printf("%-8s nq=%5d  batch p50 %.3f ms  hnsw kernel p50 %.3f ms  exp/q %.1f  dist/q %.0f  us/exp %.2f  "
               "QPS %.0f\n", name, nq, wall[it / 2], km, exq, deq, km * 1e3 / exq, nq / (wall[it / 2] * 1e-3));
        if (wv_hnsw_stamps_read) {
            wv_hnsw_stamps_read(st, 0);
            const double tot = (double)st[5];
            const double clk = st[6] ? (double)st[5] / ((double)st[6] * 10.0) : 0.0;   // cycles per ns (100 MHz ticks)
            printf("%-8s   stamps: pop %.1f%%  ids+level %.1f%%  visited %.1f%%  dist %.1f%%  merge %.1f%%  "
                   "(cycles/exp %.0f, clock %.2f GHz, wall/query %.1f us, exp/q %.1f)\n", name,
                   100 * st[0] / tot, 100 * st[1] / tot, 100 * st[2] / tot, 100 * st[3] / tot, 100 * st[4] / tot,
                   tot / (double)std::max<unsigned long long>(st[7], 1), clk,
                   st[8] ? (double)st[6] * 0.01 / (double)st[8] : 0.0, st[8] ? (double)st[7] / st[8] : 0.0);
        }
        fflush(stdout);
    }
    wv_index_destroy(ix);
    return 0;
}
