// Standalone timing harness for wv_bf_mfma_kernel variants (tools/bf_ablate.sh).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include "../weaviate_amd/csrc/wv_params.h"
#ifdef WV_BF_DBG_ITERS
extern "C" void wv_dbg_read(unsigned long long*);
#endif
extern "C" hipError_t wv_launch_bf_mfma(const wv::BfParams* p, hipStream_t s);
int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
    const int nq = argc > 2 ? atoi(argv[2]) : 10000, D = 128;
    std::vector<float> hx(N * D), hq((size_t)nq * D), hn(N);
    srand(1);
    for (auto& v : hx) v = rand() / (float)RAND_MAX;
    for (auto& v : hq) v = -2.f * rand() / (float)RAND_MAX;  // pre-scaled B operand (-2q)
    for (uint64_t i = 0; i < N; ++i) { float s = 0; for (int k = 0; k < D; ++k) s += hx[i * D + k] * hx[i * D + k]; hn[i] = s; }
    float *X, *Q, *xn, *od; uint32_t* oi;
    const bool split = getenv("SPLIT") && atoi(getenv("SPLIT"));
    const int bq = split ? (getenv("BQ") ? atoi(getenv("BQ")) : 192) : 128;
    const int prod = bq == 192 ? 8 : 4;
    const uint64_t Np = (N + 127) / 128 * 128; const size_t nqp = (nq + bq - 1) / bq * bq;
    hipMalloc(&X, Np * D * 4); hipMalloc(&Q, nqp * D * 4); hipMalloc(&xn, Np * 4);
    hipMemset(X, 0, Np * D * 4); hipMemset(Q, 0, nqp * D * 4); hipMemset(xn, 0, Np * 4);
    if (split) {   // native bf16 hi/lo images (wv_split_rows_kernel layout)
        auto bf = [](float v) { uint32_t b; memcpy(&b, &v, 4); return (uint16_t)((b + 0x7FFFu + ((b >> 16) & 1u)) >> 16); };
        auto img = [&](std::vector<float>& m, size_t rows) {
            std::vector<float> o((rows + bq - 1) / bq * bq * D, 0.f);
            uint16_t* h = reinterpret_cast<uint16_t*>(o.data());
            for (size_t r = 0; r < rows; ++r)
                for (int k = 0; k < D; ++k) {
                    const float v = m[r * D + k];
                    const uint16_t hi = bf(v);
                    uint32_t hb = (uint32_t)hi << 16; float hf; memcpy(&hf, &hb, 4);
                    const uint64_t o = wv::split_hi_index(r, k, D / 32);
                    h[o] = hi;
                    h[o + 512] = bf(v - hf);
                }
            m.swap(o);
        };
        img(hx, N); img(hq, nq);
    }
    hipMemcpy(X, hx.data(), (split ? Np : N) * D * 4, hipMemcpyHostToDevice);
    hipMemcpy(Q, hq.data(), (split ? nqp : (size_t)nq) * D * 4, hipMemcpyHostToDevice);
    hipMemcpy(xn, hn.data(), N * 4, hipMemcpyHostToDevice);
    wv::BfParams p{};
    const int nqb = (nq + bq - 1) / bq;
    const int target = getenv("BLOCKS") ? atoi(getenv("BLOCKS")) : (bq == 128 ? 512 : 256);
    const wv::BfSchedule sch = wv::bf_schedule(nq, N, target, bq);
    const int ns = sch.n_slots;
    hipMalloc(&od, (size_t)nq * ns * prod * wv::BF_KP * 4); hipMalloc(&oi, (size_t)nq * ns * prod * wv::BF_KP * 4);
    p.X = X; p.Q = Q; p.xnorm = xn; p.N = N; p.nq = nq; p.D = D; p.ldx = D; p.ldq = D; p.metric = 0;
    p.n_qblocks = nqb; p.n_slots = ns; p.ntiles = sch.ntiles; p.units_per_block = sch.units_per_block; p.out_d = od; p.out_id = oi;
    p.split = split; p.bq = bq; p.prod = prod; p.locality = getenv("LOC") ? atoi(getenv("LOC")) : 3;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    wv_launch_bf_mfma(&p, 0); hipDeviceSynchronize();
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
        hipEventRecord(a, 0); wv_launch_bf_mfma(&p, 0); hipEventRecord(b, 0); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    printf("%s blocks=%d N=%llu nq=%d: %.3f ms  %.1f TF/s  (%.1f%% of 157.3) split=%d\n", argc > 3 ? argv[3] : "variant", sch.n_blocks,
           (unsigned long long)N, nq, best, 2.0 * D * N * nq / best / 1e9, 100 * 2.0 * D * N * nq / best / 1e9 / 157.3, (int)split);
#ifdef WV_BF_DBG_ITERS
    unsigned long long c[2]; wv_dbg_read(c);
    printf("  wave-tiles %llu, extract iterations %llu (%.3f per wave-tile)\n", c[0], c[1], (double)c[1] / c[0]);
#endif
    return 0;
}
