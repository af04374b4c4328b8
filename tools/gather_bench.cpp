// Random row gather ceiling: the HBM rate a kernel reaches when every access
// is one whole row of R bytes at a random index -- the access pattern of the
// HNSW search's distance evaluations (wv_hnsw.hip), which the bench's HNSW
// roofline prices against the 8 TB/s streaming peak.  Rows of 384 B (C5's 96-d
// fp32) and 512 B (C1's 128-d) over corpora of 1M and 12.5M rows; each group
// of R/16 lanes loads one row as float4s, the indices are uniform random
// (host LCG), and the sum of each row's first element is written so the loads
// stay live.  Usage: gather_bench [n_gathers]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void gather(const float4* __restrict__ X, const uint32_t* __restrict__ idx,
                                              uint64_t n_gathers, int row_f4, float* out) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t per_block_rows = 256 / row_f4;   // rows a block loads per step (lanes past it idle)
    const uint64_t r0 = (uint64_t)blockIdx.x * per_block_rows;
    const uint64_t stride = (uint64_t)gridDim.x * per_block_rows;
    const int lr = threadIdx.x / row_f4, lc = threadIdx.x % row_f4;
    float acc = 0.f;
    if (lr < (int)per_block_rows)
        for (uint64_t r = r0 + lr; r < n_gathers; r += stride) {
            const float4 v = X[(uint64_t)idx[r] * row_f4 + lc];
            acc += v.x + v.y + v.z + v.w;
        }
    out[t] = acc;
}

int main(int argc, char** argv) {
    const uint64_t n_gathers = argc > 1 ? strtoull(argv[1], nullptr, 10) : 40000000ull;
    const uint64_t sizes[2] = {1000000ull, 12500000ull};
    const int row_bytes[2] = {384, 512};
    std::vector<uint32_t> h(n_gathers);
    const int nb = 256 * 64;
    float* out;
    uint32_t* idx;
    hipMalloc(&out, (size_t)nb * 256 * 4);
    hipMalloc(&idx, n_gathers * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (uint64_t n : sizes) {
        uint64_t s = 0x9E3779B97F4A7C15ull ^ n;
        for (uint64_t i = 0; i < n_gathers; ++i) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            h[i] = (uint32_t)((s >> 33) % n);
        }
        hipMemcpy(idx, h.data(), n_gathers * 4, hipMemcpyHostToDevice);
        for (int rb : row_bytes) {
            float4* X;
            if (hipMalloc(&X, n * rb) != hipSuccess) return 1;
            hipMemset(X, 0, n * rb);
            const int row_f4 = rb / 16;
            hipLaunchKernelGGL(gather, dim3(nb), dim3(256), 0, 0, X, idx, n_gathers / 4, row_f4, out);   // warm
            hipEventRecord(e0);
            hipLaunchKernelGGL(gather, dim3(nb), dim3(256), 0, 0, X, idx, n_gathers, row_f4, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("{\"rows\": %llu, \"row_bytes\": %d, \"gathers\": %llu, \"ms\": %.3f, \"GBs\": %.1f}\n",
                   (unsigned long long)n, rb, (unsigned long long)n_gathers, ms, (double)n_gathers * rb / (ms * 1e-3) / 1e9);
            hipFree(X);
        }
    }
    hipFree(idx);
    hipFree(out);
    return 0;
}
