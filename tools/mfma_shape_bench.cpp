// Bare f16 MFMA loop: v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 at
// the same output tile per wave (64 x 64) and two waves per SIMD, operands in
// registers (random f16 bits), to see which shape sustains more FLOP/s under
// the clock the chip holds (MI355X_MICROARCH.md 'DVFS give-back' item 7).
// Usage: mfma_shape_bench [iters]; prints TF/s per shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ half8 rnd8(uint32_t s) {
    half8 h;
    for (int i = 0; i < 8; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = (_Float16)((float)(s >> 9) * (1.0f / 8388608.0f) * 2.0f - 1.0f);
    }
    return h;
}

// 64 x 64 per wave, K = 128 per "tile": 32x32x16 -> 2 x 2 accumulators x 8 k-steps
__global__ __launch_bounds__(512, 1) void k32(int iters, float* out) {
    const uint32_t seed = blockIdx.x * 512 + threadIdx.x;
    half8 a[2][8], b[2][8];
    for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 8; ++k) { a[i][k] = rnd8(seed * 31 + i * 8 + k); b[i][k] = rnd8(seed * 17 + i * 8 + k + 99); }
    floatx16 c00 = {}, c01 = {}, c10 = {}, c11 = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            c00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][k], b[0][k], c00, 0, 0, 0);
            c01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][k], b[1][k], c01, 0, 0, 0);
            c10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1][k], b[0][k], c10, 0, 0, 0);
            c11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1][k], b[1][k], c11, 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c00[r] + c01[r] + c10[r] + c11[r];
    out[seed] = s;
}

// 64 x 64 per wave, K = 128: 16x16x32 -> 4 x 4 accumulators x 4 k-steps
__global__ __launch_bounds__(512, 1) void k16(int iters, float* out) {
    const uint32_t seed = blockIdx.x * 512 + threadIdx.x;
    half8 a[4][4], b[4][4];
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k) { a[i][k] = rnd8(seed * 31 + i * 4 + k); b[i][k] = rnd8(seed * 17 + i * 4 + k + 99); }
    floatx4 c[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) c[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][k], b[j][k], c[i][j], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += c[i][j][0] + c[i][j][1] + c[i][j][2] + c[i][j][3];
    out[seed] = s;
}

// as k16, the A operands (64 rows x 128 k per tile, h16q-style 1 KiB blocks)
// read from LDS each tile: 8 ds_read_b128 per 16 MFMAs of a half tile, like
// wv_bf_h16q_kernel's mfma_half; BAR: a workgroup barrier every 2 tiles
template <bool BAR, bool FENCE = false>
__global__ __launch_bounds__(512, 1) void k16lds(int iters, float* out) {
    __shared__ uint4 img[4][8][64];   // 3 stages' worth is not needed: one static tile
    const int lane = threadIdx.x & 63;
    const uint32_t seed = blockIdx.x * 512 + threadIdx.x;
    for (int i = threadIdx.x; i < 4 * 8 * 64; i += 512) {
        half8 h = rnd8(i * 7 + 3);
        (&img[0][0][0])[i] = __builtin_bit_cast(uint4, h);
    }
    __syncthreads();
    half8 b[4][4];
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k) b[i][k] = rnd8(seed * 17 + i * 4 + k + 99);
    floatx4 c[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) c[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (FENCE) __builtin_amdgcn_sched_barrier(0);   // no hoisting of the next half's reads
            uint4 a[2][4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int r = 0; r < 2; ++r) a[r][k] = img[2 * h + r][(k + it) & 7][lane];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        c[2 * h + r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a[r][k]), b[j][k],
                                                                                  c[2 * h + r][j], 0, 0, 0);
        }
        if (BAR && (it & 1)) __syncthreads();
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += c[i][j][0] + c[i][j][1] + c[i][j][2] + c[i][j][3];
    out[seed] = s;
}

// the kernel's half-tile structure (wv_bf_h16q_kernel's mfma_half): each half
// tile's accumulators restart from a C-in read from LDS, and the 8-key minima
// of the other half (MIN) are interleaved 1:1 with this half's MFMAs by
// sched_group_barrier, as in the kernel
template <bool MIN>
__global__ __launch_bounds__(512, 1) void k16half(int iters, float* out) {
    __shared__ uint4 img[4][8][64];
    __shared__ float xn[64];
    const int lane = threadIdx.x & 63;
    const uint32_t seed = blockIdx.x * 512 + threadIdx.x;
    for (int i = threadIdx.x; i < 4 * 8 * 64; i += 512) {
        half8 h = rnd8(i * 7 + 3);
        (&img[0][0][0])[i] = __builtin_bit_cast(uint4, h);
    }
    if (threadIdx.x < 64) xn[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    half8 b[4][4];
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k) b[i][k] = rnd8(seed * 17 + i * 4 + k + 99);
    floatx4 c[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) c[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    float sink = 0.f;
    const int lq = lane >> 4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            floatx4 xc[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const float4 v = *reinterpret_cast<const float4*>(&xn[16 * (2 * h + r) + 4 * lq]);
                xc[r] = floatx4{v.x, v.y, v.z, v.w};
            }
            __builtin_amdgcn_sched_barrier(0);
            uint4 a[2][4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int r = 0; r < 2; ++r) a[r][k] = img[2 * h + r][(k + it) & 7][lane];
            if (MIN) {
                const int o = 1 - h;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const floatx4& A = c[2 * o][g];
                    const floatx4& B = c[2 * o + 1][g];
                    sink = fminf(sink, fminf(fminf(fminf(A[0], A[1]), fminf(A[2], A[3])), fminf(fminf(B[0], B[1]), fminf(B[2], B[3]))));
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        c[2 * h + r][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a[r][k]), b[j][k],
                                                                                  k == 0 ? xc[r] : c[2 * h + r][j], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
        }
        if (it & 1) __syncthreads();
    }
    float s = sink;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += c[i][j][0] + c[i][j][1] + c[i][j][2] + c[i][j][3];
    out[seed] = s;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int nb = cus;   // one 512-thread workgroup per CU (two waves per SIMD)
    float* out;
    hipMalloc(&out, (size_t)nb * 512 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double flop = 2.0 * 64 * 64 * 128 * (double)iters * 8 * nb;   // 8 waves x 64x64x128 per iter
    for (int rep = 0; rep < 3; ++rep) {
        for (int shape = 0; shape < 8; ++shape) {
            void (*kf)(int, float*) = shape == 0 ? k32 : shape == 1 ? k16 : shape == 2 ? k16lds<false> : shape == 3 ? k16lds<true>
                                    : shape == 4 ? k16lds<false, true> : shape == 5 ? k16lds<true, true>
                                    : shape == 6 ? k16half<false> : k16half<true>;
            const char* nm[8] = {"32x32x16_f16", "16x16x32_f16", "16x16x32_f16 A from LDS", "16x16x32_f16 A from LDS + barrier/2 tiles",
                                 "16x16x32_f16 A from LDS, reads fenced per half", "16x16x32_f16 A from LDS, fenced + barrier/2 tiles",
                                 "16x16x32_f16 kernel half-tile structure (C-in restart), no minima",
                                 "16x16x32_f16 kernel half-tile structure + minima of the other half"};
            hipLaunchKernelGGL(kf, dim3(nb), dim3(512), 0, 0, iters / 10, out);   // warm
            hipEventRecord(e0);
            hipLaunchKernelGGL(kf, dim3(nb), dim3(512), 0, 0, iters, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%s  %.3f ms  %.1f TF/s\n", nm[shape], ms, flop / (ms * 1e-3) / 1e12);
        }
    }
    hipFree(out);
    return 0;
}
