// wv_h16.hip -- f16 key pass of the exact brute force (flatSearch,
// adapters/repos/db/vector/hnsw/flat_search.go:19-74) for D <= 128.
//
// The keys only rank candidates: the finalize (wv_bf.hip) re-ranks the best
// FIN_KF exactly in the reference's summation order and certifies the answer
// with a rigorous bound on |key - reference distance|.  So the key of a
// (query, row) pair needs one f16 MFMA product per fp32 product, not the three
// bf16 products of the bf16x3 pass: f16 keeps 11 mantissa bits, and the f16
// rounding of each row / query is measured exactly (its residual norm) and
// added to the certificate's eps, so integer-valued data (SIFT) keys exactly.
//
// Layout (one 512-thread workgroup per CU, 8 waves, two per SIMD):
//  * query block of 512 = 8 waves x 64 queries; a wave holds its 64 queries'
//    B operands (v_mfma_f32_32x32x16_f16, 2 column blocks x ns k-steps) in
//    registers for the whole segment -- the query side never touches LDS;
//  * corpus tiles of 64 rows stream global -> LDS by LDS-DMA
//    (global_load_lds_dwordx4, no VGPR staging) into two stages, together
//    with the tile's s|x|^2 (L2 C-in) and its exclusion / allow words: one
//    fetch of a tile feeds all 512 queries of the block;
//  * each wave computes 64 rows x 64 queries per tile (2 x 2 accumulators of
//    32 x 32, 4 MFMAs per k-step); the epilogue keeps per-lane sorted
//    candidate lists exactly as the split pass does (wv_topk.h);
//  * an optional per-query seed threshold (from a pre-pass over every
//    H_SAMPLE-th tile, wv_api.hip) starts every list with a tail, so the rare
//    extraction runs on hits below the seed only.
#include "wv_device.h"
#include "wv_params.h"
#include "wv_topk.h"

#include <float.h>

namespace wv {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(src, lds_wave_base, 4, 0, 0);
}

// LDS stage: [2 row blocks][ns k-steps][64 lanes] uint4 image, then 64 floats
// of s|x|^2, then the exclusion and allow words of the tile.
template <int NS>
struct H16Stage {
    static constexpr int IMG_U4 = 2 * NS * 64;
    static constexpr int U4 = IMG_U4 + 16 + 1;
};

template <int NS, bool L2>
__global__ __launch_bounds__(512, 2) void wv_bf_h16_kernel(H16Params p) {
    extern __shared__ uint4 lds[];
    using St = H16Stage<NS>;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int khalf = lane >> 5;
    const int l31 = lane & 31;
    const uint4* __restrict__ X = reinterpret_cast<const uint4*>(p.X);
    const uint4* __restrict__ Qg = reinterpret_cast<const uint4*>(p.Q);
    const bool has_allow = p.allow != nullptr;
    // key scale s = s_x * s_q: the seed thresholds arrive in true units
    const float s = p.sx * p.qscale[0];
    int lb = (int)blockIdx.x;
    if ((p.locality & 1) && gridDim.x >= 8) {   // bijective XCD remap (blocks b, b + 8, ... share an XCD)
        const int nwg = (int)gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = (int)blockIdx.x % 8;
        lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (int)blockIdx.x / 8;
    }
    const uint64_t u_first = (uint64_t)lb * p.units_per_block;
    uint64_t u_last = u_first + p.units_per_block;
    if (u_last > (uint64_t)p.n_qblocks * p.ntiles) u_last = (uint64_t)p.n_qblocks * p.ntiles;

    auto fill = [&](uint64_t t, int st) {
        const uint64_t tile = t * (uint64_t)p.tile_stride;
        uint4* dst = lds + st * St::U4;
        const uint4* src = X + tile * St::IMG_U4;
#pragma unroll
        for (int i = wave; i < St::IMG_U4 / 64; i += H_WAVES) glds16(src + i * 64 + lane, dst + i * 64);
        if (wave == 0) {
            if (L2) glds4(p.xns + tile * H_BN + lane, dst + St::IMG_U4);
        } else if (wave == 1) {
            // lanes 0-1: exclusion word, 2-3: allow word (dword halves)
            const uint32_t* w = lane < 2 ? reinterpret_cast<const uint32_t*>(p.excl + tile) + lane
                                         : reinterpret_cast<const uint32_t*>(p.allow + tile) + (lane - 2);
            if (lane < 2 || (lane < 4 && has_allow)) glds4(w, dst + St::IMG_U4 + 16);
        }
    };

    for (uint64_t u = u_first; u < u_last;) {
        const int qb = (int)(u / p.ntiles);
        const uint64_t t_begin = u % p.ntiles;
        uint64_t t_end = t_begin + (u_last - u);
        if (t_end > p.ntiles) t_end = p.ntiles;
        u += t_end - t_begin;
        const int slot = lb - bf_first_block(qb, p.ntiles, p.units_per_block);
        const int jq0 = qb * H_BQ + wave * 64 + l31;
        const int jq1 = jq0 + 32;
        const int ntile = (int)(t_end - t_begin);

        // the wave's 64 queries as B operands, for the whole segment
        uint4 bq0[NS], bq1[NS];
        {
            const uint64_t g0 = (uint64_t)qb * (H_BQ / 32) + 2 * wave;
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                bq0[st] = Qg[(g0 * NS + st) * 64 + lane];
                bq1[st] = Qg[((g0 + 1) * NS + st) * 64 + lane];
            }
        }
        float tau0 = FLT_MAX, tau1 = FLT_MAX;
        if (p.tau) {
            if (jq0 < p.nq) tau0 = fminf(FLT_MAX, p.tau[jq0] * s);
            if (jq1 < p.nq) tau1 = fminf(FLT_MAX, p.tau[jq1] * s);
        }
        float l0d[BF_KP], l1d[BF_KP];
        uint32_t l0i[BF_KP], l1i[BF_KP];
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            l0d[i] = FLT_MAX; l1d[i] = FLT_MAX;
            l0i[i] = WV_NIL; l1i[i] = WV_NIL;
        }
        __syncthreads();   // the previous segment's reads of both stages are done
        if (ntile > 0) fill(t_begin, 0);
        __syncthreads();   // drains the B loads and tile 0 (vmcnt(0) + barrier)

        for (int t = 0; t < ntile; ++t) {
            const int st = t & 1;
            if (t + 1 < ntile) fill(t_begin + t + 1, st ^ 1);
            const uint4* img = lds + st * St::U4;
            const uint64_t tile = (t_begin + t) * (uint64_t)p.tile_stride;
            const uint64_t row0 = tile * H_BN;
            // lanes l and l ^ 32 keep lists for the same query column (see the split pass)
            const float pt0 = fminf(__shfl_xor(l0d[BF_KP - 1], 32, 64), tau0);
            const float pt1 = fminf(__shfl_xor(l1d[BF_KP - 1], 32, 64), tau1);

            floatx16 acc00, acc01, acc10, acc11;
            floatx16 xc0, xc1;
            if (L2) {
                const float* xn = reinterpret_cast<const float*>(img + St::IMG_U4);
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const float4 a = *reinterpret_cast<const float4*>(xn + 4 * khalf + 8 * g4);
                    const float4 b = *reinterpret_cast<const float4*>(xn + 32 + 4 * khalf + 8 * g4);
                    xc0[4 * g4] = a.x; xc0[4 * g4 + 1] = a.y; xc0[4 * g4 + 2] = a.z; xc0[4 * g4 + 3] = a.w;
                    xc1[4 * g4] = b.x; xc1[4 * g4 + 1] = b.y; xc1[4 * g4 + 2] = b.z; xc1[4 * g4 + 3] = b.w;
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) { xc0[r] = 0.f; xc1[r] = 0.f; }
            }
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                const half8 a0 = __builtin_bit_cast(half8, img[k * 64 + lane]);
                const half8 a1 = __builtin_bit_cast(half8, img[(NS + k) * 64 + lane]);
                const half8 b0 = __builtin_bit_cast(half8, bq0[k]);
                const half8 b1 = __builtin_bit_cast(half8, bq1[k]);
                acc00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, k == 0 ? xc0 : acc00, 0, 0, 0);
                acc01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, k == 0 ? xc0 : acc01, 0, 0, 0);
                acc10 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, k == 0 ? xc1 : acc10, 0, 0, 0);
                acc11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, k == 0 ? xc1 : acc11, 0, 0, 0);
            }
            // ---- epilogue of one 64-row tile ----
            uint64_t okw;
            {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(img + St::IMG_U4 + 16);
                const uint64_t ex = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
                const uint64_t al = has_allow ? ((uint64_t)w[2] | ((uint64_t)w[3] << 32)) : ~0ull;
                okw = ~ex & al;
                if (row0 + H_BN > p.N) okw &= p.N > row0 ? ((1ull << (p.N - row0)) - 1) : 0ull;
            }
            const uint32_t rb0 = (uint32_t)row0 + 4 * khalf;
            const float INF = __builtin_inff();
            if (okw != ~0ull || (qb + 1) * H_BQ > p.nq) {
                const uint64_t o0 = (jq0 < p.nq ? okw : 0ull) >> (4 * khalf);
                const uint64_t o1 = (jq1 < p.nq ? okw : 0ull) >> (4 * khalf);
                const uint32_t o0lo = (uint32_t)o0, o0hi = (uint32_t)(o0 >> 32);
                const uint32_t o1lo = (uint32_t)o1, o1hi = (uint32_t)(o1 >> 32);
                constexpr uint32_t LANE_ROWS = 0x0F0F0F0Fu;
                if (!__all((o0lo & o0hi & o1lo & o1hi & LANE_ROWS) == LANE_ROWS)) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int bit = (r & 3) + 8 * (r >> 2);
                        acc00[r] = (o0lo >> bit) & 1u ? acc00[r] : INF;
                        acc10[r] = (o0hi >> bit) & 1u ? acc10[r] : INF;
                        acc01[r] = (o1lo >> bit) & 1u ? acc01[r] : INF;
                        acc11[r] = (o1hi >> bit) & 1u ? acc11[r] : INF;
                    }
                }
            }
            float m0 = INF, m1 = INF;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                m0 = min3_raw(m0, acc00[r], acc10[r]);
                m1 = min3_raw(m1, acc01[r], acc11[r]);
            }
            split_extract(m0, acc00, acc10, l0d, l0i, pt0, rb0);
            split_extract(m1, acc01, acc11, l1d, l1i, pt1, rb0);
            __syncthreads();   // the next stage has landed; this stage is free for the tile after
        }

        const size_t per_q = (size_t)p.n_slots * H_PROD * BF_KP;
        if (jq0 < p.nq) {
            const size_t base = (size_t)jq0 * per_q + ((size_t)slot * H_PROD + khalf) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l0d[i]; p.out_id[base + i] = l0i[i]; }
        }
        if (jq1 < p.nq) {
            const size_t base = (size_t)jq1 * per_q + ((size_t)slot * H_PROD + khalf) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l1d[i]; p.out_id[base + i] = l1i[i]; }
        }
    }
}

// ---------------------------------------------------------------------------
// f16 images.  One wave per row: lane handles k = lane and lane + 64 (D <= 128).
// v = scale * sign * in (powers of two and -1 / -2: exact), h = f16(v) (round
// to nearest even; overflow gives inf, which makes the residual inf and every
// certificate fail: still exact, through the fallback), residual
// |sign * in - h / scale| summed in fp32 and rounded up.
__device__ __forceinline__ float pow2_scale_for(float maxabs) {
    if (!(maxabs > 0.f) || !(maxabs < FLT_MAX)) return 1.f;
    int e;
    frexpf(maxabs, &e);                 // maxabs < 2^e
    e = 14 - e;                         // maxabs * 2^(14 - e) < 2^14
    e = e > 100 ? 100 : (e < -100 ? -100 : e);
    return ldexpf(1.f, e);
}

__global__ void wv_h16_rows_kernel(const float* in, int ld_in, const uint64_t* ids, uint64_t n, int D, int ns,
                                   float sign, float scale, const unsigned int* scale_from_max, uint16_t* out,
                                   uint64_t out_row0, unsigned int* res_max_bits, float* res_out) {
    const uint64_t r = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    if (scale_from_max) scale = pow2_scale_for(__uint_as_float(*scale_from_max) * fabsf(sign));
    const uint64_t row = ids ? ids[r] : r;
    const int kmax = ns * 16;
    float acc = 0.f;
    for (int k = lane; k < kmax; k += 64) {
        const float x = k < D ? sign * in[row * (uint64_t)ld_in + k] : 0.f;
        const _Float16 h = (_Float16)(scale * x);
        const float back = (float)h / scale;
        const float e = x - back;           // exact (Sterbenz) unless h overflowed
        acc = __builtin_fmaf(e, e, acc);
        out[h16_index(out_row0 + row, k, ns)] = __builtin_bit_cast(uint16_t, h);
    }
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if (lane == 0) {
        // inflate for the fp32 sum (D terms) and the sqrt
        const float res = acc == 0.f ? 0.f : sqrtf(acc * (1.0f + 2e-5f)) * (1.0f + 1e-6f) + 1e-30f;
        if (res_max_bits) atomicMax(res_max_bits, __float_as_uint(res));
        if (res_out) res_out[row] = res;
    }
}

// max |v| over n rows of D (float bits: positive floats order as integers)
__global__ void wv_absmax_kernel(const float* in, int ld, uint64_t n, int D, unsigned int* max_bits) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float m = 0.f;
    for (uint64_t j = i; j < n * (uint64_t)D; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = j / (uint64_t)D, c = j % (uint64_t)D;
        m = fmaxf(m, fabsf(in[r * ld + c]));
    }
    for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(max_bits, __float_as_uint(m));
}

// s_q from the batch max, and s * |x|^2 for the L2 C-in
__global__ void wv_h16_qscale_kernel(const unsigned int* max_bits, float bsign, float* qscale) {
    if (threadIdx.x == 0 && blockIdx.x == 0) qscale[0] = pow2_scale_for(__uint_as_float(*max_bits) * fabsf(bsign));
}
__global__ void wv_h16_xns_kernel(const float* xnorm, uint64_t n, float sx, const float* qscale, float* xns) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) xns[i] = xnorm[i] * (sx * qscale[0]);
}

}  // namespace wv

extern "C" {

float wv_h16_pow2_scale(float maxabs) {
    if (!(maxabs > 0.f) || !(maxabs < FLT_MAX)) return 1.f;
    int e;
    frexpf(maxabs, &e);
    e = 14 - e;
    e = e > 100 ? 100 : (e < -100 ? -100 : e);
    return ldexpf(1.f, e);
}

hipError_t wv_launch_h16_rows(const float* in, int ld_in, const uint64_t* ids, uint64_t n, int D, int ns, float sign,
                              float scale, const unsigned int* scale_from_max, void* out, uint64_t out_row0,
                              unsigned int* res_max_bits, float* res_out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (ns < 1 || ns > wv::H_NS_MAX || D > ns * 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wv::wv_h16_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, in, ld_in, ids, n, D,
                       ns, sign, scale, scale_from_max, static_cast<uint16_t*>(out), out_row0, res_max_bits, res_out);
    return hipGetLastError();
}

hipError_t wv_launch_absmax(const float* in, int ld, uint64_t n, int D, unsigned int* max_bits, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n * (uint64_t)D + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(wv::wv_absmax_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, ld, n, D, max_bits);
    return hipGetLastError();
}

hipError_t wv_launch_h16_qscale(const unsigned int* max_bits, float bsign, float* qscale, hipStream_t s) {
    hipLaunchKernelGGL(wv::wv_h16_qscale_kernel, dim3(1), dim3(64), 0, s, max_bits, bsign, qscale);
    return hipGetLastError();
}

hipError_t wv_launch_h16_xns(const float* xnorm, uint64_t n, float sx, const float* qscale, float* xns, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_h16_xns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, xnorm, n, sx, qscale,
                       xns);
    return hipGetLastError();
}

hipError_t wv_launch_bf_h16(const wv::H16Params* p, int ns, hipStream_t s) {
    const uint64_t total = (uint64_t)p->n_qblocks * p->ntiles;
    const unsigned nb = (unsigned)((total + p->units_per_block - 1) / p->units_per_block);
    if (nb == 0) return hipSuccess;
    if (ns < 1 || ns > wv::H_NS_MAX || !p->X || !p->Q || !p->excl || !p->qscale || p->tile_stride < 1)
        return hipErrorInvalidValue;
    const bool l2 = p->metric == WV_METRIC_L2;
    if (l2 && !p->xns) return hipErrorInvalidValue;
    const size_t lds = 2 * (size_t)(2 * ns * 64 + 17) * 16;
#define WV_H16_LAUNCH(NS)                                                                              \
    if (l2) hipLaunchKernelGGL((wv::wv_bf_h16_kernel<NS, true>), dim3(nb), dim3(512), lds, s, *p);    \
    else hipLaunchKernelGGL((wv::wv_bf_h16_kernel<NS, false>), dim3(nb), dim3(512), lds, s, *p);
    switch (ns) {
        case 1: WV_H16_LAUNCH(1) break;
        case 2: WV_H16_LAUNCH(2) break;
        case 3: WV_H16_LAUNCH(3) break;
        case 4: WV_H16_LAUNCH(4) break;
        case 5: WV_H16_LAUNCH(5) break;
        case 6: WV_H16_LAUNCH(6) break;
        case 7: WV_H16_LAUNCH(7) break;
        default: WV_H16_LAUNCH(8) break;
    }
#undef WV_H16_LAUNCH
    return hipGetLastError();
}

}  // extern "C"
