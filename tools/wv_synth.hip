// wv_synth.hip -- counter-based synthetic corpora generated on the device
// (measurement infrastructure for bench.py: configs[3]'s 10M x 768 and
// configs[4]'s 100M x 96 corpora take minutes to generate with numpy on the
// host and must be copied over PCIe afterwards; here they are written in
// HBM where the index reads them).  Not part of the product library.
//
// Every value depends only on (seed, row, column), as bench.py's numpy
// generators, so any rank can generate exactly its own rows:
//   kind 0  U[0,1)            bit-identical to bench.counter_uniform
//   kind 1  N(0,1)/sqrt(dim)  Box-Muller over the same two counter streams as
//                             bench.counter_gauss (device log/cos: not
//                             guaranteed bit-identical to numpy's)
//   kind 2  SIFT-shaped       bench.counter_sift's construction (1024 centres,
//                             24-d latent, noise, rounded, clipped at 0)
// The bench downloads the rows it hands to the CPU restatement, so parity
// never depends on host and device generators agreeing.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t cmix(uint64_t seed, uint64_t idx) {
    uint64_t x = idx * 0x9E3779B97F4A7C15ull + seed * 0xD1B54A32D192ED03ull;
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
// counter_uniform(seed, row, col) of a dim-wide matrix
__device__ __forceinline__ float cuni(uint64_t seed, uint64_t row, int col, int dim) {
    return (float)(cmix(seed, row * (uint64_t)dim + (uint64_t)col) >> 40) * (1.0f / 16777216.0f);
}
// counter_gauss(seed, row, col) * sqrt(dim) (the unit normal)
__device__ __forceinline__ float cgauss_unit(uint64_t seed, uint64_t row, int col, int dim) {
    const double u1 = (double)cuni(seed, row, col, dim), u2 = (double)cuni(seed + 1000, row, col, dim);
    return (float)(sqrt(-2.0 * log(u1 + 2.9802322387695312e-08)) * cos(6.283185307179586 * u2));
}

__global__ void k_uniform(uint64_t seed, uint64_t row0, uint64_t n, int dim, float* out, int ld) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * (uint64_t)dim) return;
    const uint64_t r = i / (uint64_t)dim;
    const int c = (int)(i - r * (uint64_t)dim);
    out[r * (uint64_t)ld + c] = cuni(seed, row0 + r, c, dim);
}

__global__ void k_gauss(uint64_t seed, uint64_t row0, uint64_t n, int dim, float* out, int ld) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * (uint64_t)dim) return;
    const uint64_t r = i / (uint64_t)dim;
    const int c = (int)(i - r * (uint64_t)dim);
    out[r * (uint64_t)ld + c] = cgauss_unit(seed, row0 + r, c, dim) / sqrtf((float)dim);
}

constexpr int SIFT_C = 1024, SIFT_L = 24, SIFT_DMAX = 128;

// centres [C][dim] and basis [dim][L] (bench.counter_sift's constants)
__global__ void k_sift_tables(int dim, float* centres, float* basis) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < SIFT_C * dim) centres[i] = cuni(77, i / dim, i % dim, dim) * 60.0f;
    if (i < dim * SIFT_L) basis[i] = cgauss_unit(78, i / SIFT_L, i % SIFT_L, SIFT_L);   // counter_gauss * sqrt(L)
}

// 64 rows per block, one per thread, staged in LDS and written row-major
__global__ __launch_bounds__(64) void k_sift(uint64_t seed, uint64_t row0, uint64_t n, int dim, float* out, int ld,
                                             const float* __restrict__ centres, const float* __restrict__ basis) {
    __shared__ float tile[64][SIFT_DMAX + 1];
    const uint64_t r = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (r < n) {
        const uint64_t row = row0 + r;
        const int cid = (int)(cuni(seed + 2000, row, 0, 1) * (float)SIFT_C);
        float z[SIFT_L];
#pragma unroll
        for (int l = 0; l < SIFT_L; ++l) z[l] = cgauss_unit(seed + 3000, row, l, SIFT_L);
        const float* cen = centres + (size_t)cid * dim;
        for (int c = 0; c < dim; ++c) {
            float zb = 0.f;
#pragma unroll
            for (int l = 0; l < SIFT_L; ++l) zb = fmaf(z[l], basis[c * SIFT_L + l], zb);
            const float e = cgauss_unit(seed + 4000, row, c, dim);
            const float x = cen[c] + zb * 12.0f + e * 3.0f;
            tile[threadIdx.x][c] = fmaxf(rintf(x), 0.f);
        }
    }
    __syncthreads();
    const uint64_t nr = n - (uint64_t)blockIdx.x * 64 < 64 ? n - (uint64_t)blockIdx.x * 64 : 64;
    for (int i = threadIdx.x; i < (int)nr * dim; i += 64) {
        const int rr = i / dim, c = i - rr * dim;
        out[((uint64_t)blockIdx.x * 64 + rr) * (uint64_t)ld + c] = tile[rr][c];
    }
}

}  // namespace

extern "C" {

// rows [row0, row0 + n) of the kind's dim-wide matrix into out (row stride
// ld floats; columns dim .. ld - 1 untouched), on stream; 0 or a HIP error
int wvs_fill(int kind, uint64_t seed, uint64_t row0, uint64_t n, int dim, float* out, int ld, void* stream) {
    if (n == 0) return 0;
    if (dim <= 0 || ld < dim || !out) return (int)hipErrorInvalidValue;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t total = n * (uint64_t)dim;
    const unsigned blocks = (unsigned)((total + 255) / 256);
    if (kind == 0) {
        hipLaunchKernelGGL(k_uniform, dim3(blocks), dim3(256), 0, s, seed, row0, n, dim, out, ld);
    } else if (kind == 1) {
        hipLaunchKernelGGL(k_gauss, dim3(blocks), dim3(256), 0, s, seed, row0, n, dim, out, ld);
    } else if (kind == 2) {
        if (dim > SIFT_DMAX) return (int)hipErrorInvalidValue;
        float* tables = nullptr;
        hipError_t e = hipMallocAsync((void**)&tables, sizeof(float) * (SIFT_C * dim + dim * SIFT_L), s);
        if (e != hipSuccess) return (int)e;
        const int nt = SIFT_C * dim;
        hipLaunchKernelGGL(k_sift_tables, dim3((nt + 255) / 256), dim3(256), 0, s, dim, tables, tables + SIFT_C * dim);
        for (uint64_t r0 = 0; r0 < n; r0 += 64ull << 20) {   // (grid of < 2^31 blocks per launch)
            const uint64_t m = n - r0 < (64ull << 20) ? n - r0 : (64ull << 20);
            hipLaunchKernelGGL(k_sift, dim3((unsigned)((m + 63) / 64)), dim3(64), 0, s, seed, row0 + r0, m, dim,
                               out + r0 * (uint64_t)ld, ld, tables, tables + SIFT_C * dim);
        }
        e = hipFreeAsync(tables, s);
        if (e != hipSuccess) return (int)e;
    } else {
        return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

}  // extern "C"
