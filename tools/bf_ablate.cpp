// Standalone timing harness for wv_bf_mfma_kernel variants (tools/bf_ablate.sh).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../weaviate_amd/csrc/wv_params.h"
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
    const uint64_t Np = (N + 127) / 128 * 128; const size_t nqp = (nq + 127) / 128 * 128;
    hipMalloc(&X, Np * D * 4); hipMalloc(&Q, nqp * D * 4); hipMalloc(&xn, Np * 4);
    hipMemset(X, 0, Np * D * 4); hipMemset(Q, 0, nqp * D * 4); hipMemset(xn, 0, Np * 4);
    hipMemcpy(X, hx.data(), N * D * 4, hipMemcpyHostToDevice);
    hipMemcpy(Q, hq.data(), (size_t)nq * D * 4, hipMemcpyHostToDevice);
    hipMemcpy(xn, hn.data(), N * 4, hipMemcpyHostToDevice);
    wv::BfParams p{};
    const int nqb = (nq + 127) / 128;
    const int target = getenv("BLOCKS") ? atoi(getenv("BLOCKS")) : 512;
    const wv::BfSchedule sch = wv::bf_schedule(nq, N, target);
    const int ns = sch.n_slots;
    hipMalloc(&od, (size_t)nq * ns * 4 * wv::BF_KP * 4); hipMalloc(&oi, (size_t)nq * ns * 4 * wv::BF_KP * 4);
    p.X = X; p.Q = Q; p.xnorm = xn; p.N = N; p.nq = nq; p.D = D; p.ldx = D; p.ldq = D; p.metric = 0;
    p.n_qblocks = nqb; p.n_slots = ns; p.ntiles = sch.ntiles; p.units_per_block = sch.units_per_block; p.out_d = od; p.out_id = oi;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    wv_launch_bf_mfma(&p, 0); hipDeviceSynchronize();
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
        hipEventRecord(a, 0); wv_launch_bf_mfma(&p, 0); hipEventRecord(b, 0); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    printf("%s blocks=%d N=%llu nq=%d: %.3f ms  %.1f TF/s  (%.1f%% of 157.3)\n", argc > 3 ? argv[3] : "variant", sch.n_blocks,
           (unsigned long long)N, nq, best, 2.0 * D * N * nq / best / 1e9, 100 * 2.0 * D * N * nq / best / 1e9 / 157.3);
    return 0;
}
