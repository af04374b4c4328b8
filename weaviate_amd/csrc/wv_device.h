// wv_device.h -- device helpers shared by the CDNA4 (gfx950) kernels.
//
// The exact distance here reproduces the reference's AVX2 assembly bit for bit
// (adapters/repos/db/vector/hnsw/distancer/asm/l2_amd64.s:7-64 and
// dot_amd64.s:7-55): 32 independent FMA chains (4 accumulators x 8 lanes) over
// 32-float blocks, a sequential FMA tail, then the fixed reduction tree.  On
// the GPU the 32 chains are spread over a group of 8 lanes, each lane owning
// one float4 slice (4 chains) of every 32-float block, so a group reads a row
// as fully coalesced 128-byte pieces.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define WV_NIL 0xFFFFFFFFu
#define WV_FLAG 0x80000000u   // "expanded" flag carried in bit 31 of a local id
#define WV_IDMASK 0x7FFFFFFFu

enum { WV_METRIC_L2 = 0, WV_METRIC_DOT = 1, WV_METRIC_COSINE = 2 };

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float shfl_xor_f(float v, int m) { return __shfl_xor(v, m, 64); }

// Exact reference-order distance of one stored row against the query, computed
// by the 8-lane group that contains this lane (g = lane & 7).  Every lane of
// the group returns the result.  q and row are 16-byte aligned, D % 4 == 0.
// BLK > 1: the row's blocks are loaded BLK at a time before their FMAs (same
// order): one memory round trip per BLK blocks instead of one per block when
// the compiler keeps the loop rolled (D = 768: 24 dependent trips a row).
template <int METRIC, int BLK = 1>
__device__ __forceinline__ float exact_dist_group8(const float* __restrict__ q,
                                                   const float* __restrict__ row,
                                                   int D, int g) {
    const int nb = D >> 5;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int b0 = 0; b0 < nb; b0 += BLK) {
      float4 yb[BLK];
#pragma unroll
      for (int bb = 0; bb < BLK; ++bb)
          if (b0 + bb < nb) yb[bb] = ld4(row + 32 * (b0 + bb) + 4 * g);
#pragma unroll
      for (int bb = 0; bb < BLK; ++bb) {
        if (b0 + bb >= nb) break;
        const int b = b0 + bb;
        const float4 x = ld4(q + 32 * b + 4 * g);
        const float4 y = yb[bb];
        if (METRIC == WV_METRIC_L2) {
            const float d0 = x.x - y.x, d1 = x.y - y.y, d2 = x.z - y.z, d3 = x.w - y.w;
            a0 = __builtin_fmaf(d0, d0, a0);
            a1 = __builtin_fmaf(d1, d1, a1);
            a2 = __builtin_fmaf(d2, d2, a2);
            a3 = __builtin_fmaf(d3, d3, a3);
        } else {
            a0 = __builtin_fmaf(x.x, y.x, a0);
            a1 = __builtin_fmaf(x.y, y.y, a1);
            a2 = __builtin_fmaf(x.z, y.z, a2);
            a3 = __builtin_fmaf(x.w, y.w, a3);
        }
      }
    }
    // tail (l2_amd64.s:40-52 / dot_amd64.s:36-43): one sequential chain
    float t = 0.f;
    for (int i = nb * 32; i < D; i += 4) {
        const float4 x = ld4(q + i);
        const float4 y = ld4(row + i);
        if (METRIC == WV_METRIC_L2) {
            float d = x.x - y.x; t = __builtin_fmaf(d, d, t);
            d = x.y - y.y;       t = __builtin_fmaf(d, d, t);
            d = x.z - y.z;       t = __builtin_fmaf(d, d, t);
            d = x.w - y.w;       t = __builtin_fmaf(d, d, t);
        } else {
            t = __builtin_fmaf(x.x, y.x, t);
            t = __builtin_fmaf(x.y, y.y, t);
            t = __builtin_fmaf(x.z, y.z, t);
            t = __builtin_fmaf(x.w, y.w, t);
        }
    }
    // reduction tree (l2_amd64.s:54-64): lane g holds accumulator j = g>>1,
    // lanes l = 4*(g&1) .. +3.  (acc0+acc1), (acc2+acc3): xor 2
    a0 = a0 + shfl_xor_f(a0, 2); a1 = a1 + shfl_xor_f(a1, 2);
    a2 = a2 + shfl_xor_f(a2, 2); a3 = a3 + shfl_xor_f(a3, 2);
    // (acc0+acc1)+(acc2+acc3): xor 4
    a0 = a0 + shfl_xor_f(a0, 4); a1 = a1 + shfl_xor_f(a1, 4);
    a2 = a2 + shfl_xor_f(a2, 4); a3 = a3 + shfl_xor_f(a3, 4);
    // VEXTRACTF128 + VADDPS: v[l] = s[l] + s[l+4]: xor 1
    a0 = a0 + shfl_xor_f(a0, 1); a1 = a1 + shfl_xor_f(a1, 1);
    a2 = a2 + shfl_xor_f(a2, 1); a3 = a3 + shfl_xor_f(a3, 1);
    // VADDPS X1: v += [t, 0, 0, 0]; two VHADDPS: (v0+v1)+(v2+v3)
    a0 = t + a0;
    a1 = 0.0f + a1;
    a2 = 0.0f + a2;
    a3 = 0.0f + a3;
    const float r = (a0 + a1) + (a2 + a3);
    if (METRIC == WV_METRIC_L2) return r;
    if (METRIC == WV_METRIC_DOT) return -r;
    return 1.0f - r;
}

// Exact reference-order distances of up to 8*RPG rows at once (RPG per 8-lane
// group), all row loads of a 4-block (128-float) slab issued before any FMA so
// one memory round trip serves 8*RPG rows; a tail of one float4 (D = 32 m + 4,
// e.g. GloVe's 100) is loaded with the first slab instead of after it (it was
// a second dependent round trip per call; HOIST_TAIL, 16 more VGPRs).  ids/out live in LDS; rows >= n
// are skipped.  Same arithmetic, in the same order, as exact_dist_group8.
template <int METRIC, int RPG = 4, bool HOIST_TAIL = false>
__device__ __forceinline__ void exact_dist_rows(const float* __restrict__ q, const float* __restrict__ X,
                                                int ldx, int D, const uint32_t* ids, int n, float* out,
                                                int lane) {
    const int g = lane & 7, grp = lane >> 3;
    const int nb = D >> 5;
    const float* row[RPG];
    bool ok[RPG];
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        const int c = grp + 8 * j;
        ok[j] = c < n;
        row[j] = X + (uint64_t)(ok[j] ? ids[c] : ids[0]) * ldx;
    }
    float a[RPG][4];
#pragma unroll
    for (int j = 0; j < RPG; ++j) a[j][0] = a[j][1] = a[j][2] = a[j][3] = 0.f;
    const bool tail1 = HOIST_TAIL && D - nb * 32 > 0 && D - nb * 32 <= 4;
    float4 yt[RPG];
    if (tail1) {
#pragma unroll
        for (int j = 0; j < RPG; ++j)
            if (ok[j]) yt[j] = ld4(row[j] + nb * 32);
    }
    for (int b0 = 0; b0 < nb; b0 += 4) {
        float4 y[RPG][4];
#pragma unroll
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
                if (ok[j] && b0 + bb < nb) y[j][bb] = ld4(row[j] + 32 * (b0 + bb) + 4 * g);
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            if (b0 + bb >= nb) break;
            const float4 x = ld4(q + 32 * (b0 + bb) + 4 * g);
#pragma unroll
            for (int j = 0; j < RPG; ++j) {
                if (!ok[j]) continue;
                const float4 yy = y[j][bb];
                if (METRIC == WV_METRIC_L2) {
                    const float d0 = x.x - yy.x, d1 = x.y - yy.y, d2 = x.z - yy.z, d3 = x.w - yy.w;
                    a[j][0] = __builtin_fmaf(d0, d0, a[j][0]);
                    a[j][1] = __builtin_fmaf(d1, d1, a[j][1]);
                    a[j][2] = __builtin_fmaf(d2, d2, a[j][2]);
                    a[j][3] = __builtin_fmaf(d3, d3, a[j][3]);
                } else {
                    a[j][0] = __builtin_fmaf(x.x, yy.x, a[j][0]);
                    a[j][1] = __builtin_fmaf(x.y, yy.y, a[j][1]);
                    a[j][2] = __builtin_fmaf(x.z, yy.z, a[j][2]);
                    a[j][3] = __builtin_fmaf(x.w, yy.w, a[j][3]);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        float t = 0.f;
        if (ok[j]) {
            for (int i = nb * 32; i < D; i += 4) {
                const float4 x = ld4(q + i);
                const float4 yy = tail1 ? yt[j] : ld4(row[j] + i);
                if (METRIC == WV_METRIC_L2) {
                    float d = x.x - yy.x; t = __builtin_fmaf(d, d, t);
                    d = x.y - yy.y;       t = __builtin_fmaf(d, d, t);
                    d = x.z - yy.z;       t = __builtin_fmaf(d, d, t);
                    d = x.w - yy.w;       t = __builtin_fmaf(d, d, t);
                } else {
                    t = __builtin_fmaf(x.x, yy.x, t);
                    t = __builtin_fmaf(x.y, yy.y, t);
                    t = __builtin_fmaf(x.z, yy.z, t);
                    t = __builtin_fmaf(x.w, yy.w, t);
                }
            }
        }
        float a0 = a[j][0], a1 = a[j][1], a2 = a[j][2], a3 = a[j][3];
        a0 = a0 + shfl_xor_f(a0, 2); a1 = a1 + shfl_xor_f(a1, 2);
        a2 = a2 + shfl_xor_f(a2, 2); a3 = a3 + shfl_xor_f(a3, 2);
        a0 = a0 + shfl_xor_f(a0, 4); a1 = a1 + shfl_xor_f(a1, 4);
        a2 = a2 + shfl_xor_f(a2, 4); a3 = a3 + shfl_xor_f(a3, 4);
        a0 = a0 + shfl_xor_f(a0, 1); a1 = a1 + shfl_xor_f(a1, 1);
        a2 = a2 + shfl_xor_f(a2, 1); a3 = a3 + shfl_xor_f(a3, 1);
        a0 = t + a0;
        a1 = 0.0f + a1;
        a2 = 0.0f + a2;
        a3 = 0.0f + a3;
        float r = (a0 + a1) + (a2 + a3);
        if (METRIC == WV_METRIC_DOT) r = -r;
        else if (METRIC == WV_METRIC_COSINE) r = 1.0f - r;
        if (ok[j] && g == 0) out[grp + 8 * j] = r;
    }
}

// Distance of one product-quantized row to the query, computed by ONE lane:
// DistanceBetweenCompressedAndUncompressedVectors
// (ssdhelpers/product_quantization.go:284-291), which the lookup table of
// :56-75 caches value for value.  Step is the pure-Go loop of the provider
// (distancer/l2.go:63-72, dot_product.go:80-87, cosine_dist.go:57-64): the
// products are rounded before the add (no FMA: the _rn intrinsics keep the
// compiler from contracting), segments summed in order, then Wrap.
template <int METRIC, class PQ>
__device__ __forceinline__ float pq_dist_row(const float* __restrict__ q, const PQ& pq, uint32_t row) {
    const uint8_t* cr = pq.codes + (uint64_t)row * pq.stride;
    float dist = 0.f;
    for (int i0 = 0; i0 < pq.m; i0 += 4) {
        // four codes per 32-bit load (rows are padded to whole words)
        uint32_t w0 = *reinterpret_cast<const uint32_t*>(cr + (pq.wide ? 2 * i0 : i0));
        uint32_t w1 = pq.wide ? *reinterpret_cast<const uint32_t*>(cr + 2 * i0 + 4) : 0u;
        const int nseg = min(4, pq.m - i0);
        for (int t = 0; t < nseg; ++t) {
            const uint32_t c = pq.wide ? (t < 2 ? (w0 >> (16 * t)) : (w1 >> (16 * (t - 2)))) & 0xFFFFu
                                       : (w0 >> (8 * t)) & 0xFFu;
            const int i = i0 + t;
            const float* cp = pq.cent + ((uint64_t)i * pq.ks + c) * pq.ds;
            const float* qs = q + i * pq.ds;
            float s = 0.f;
            for (int j = 0; j < pq.ds; ++j) {
                if (METRIC == WV_METRIC_L2) {
                    const float d = __fsub_rn(qs[j], cp[j]);
                    s = __fadd_rn(s, __fmul_rn(d, d));
                } else {
                    s = __fadd_rn(s, __fmul_rn(qs[j], cp[j]));
                }
            }
            dist = __fadd_rn(dist, s);
        }
    }
    if (METRIC == WV_METRIC_L2) return dist;
    if (METRIC == WV_METRIC_DOT) return -dist;
    return __fsub_rn(1.0f, dist);
}

// asm.L2 (distancer/asm/l2_amd64.s:7-64) of two short rows by ONE lane: the
// same 4 x 8 accumulators, scalar FMA tail and reduction tree as
// exact_dist_group8, written serially (KMeans.Nearest, kmeans.go:78-110).
__device__ __forceinline__ float asm_l2_serial(const float* __restrict__ x, const float* __restrict__ y, int n) {
    float acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[j][l] = 0.f;
    int i = 0;
    for (; n - i >= 32; i += 32) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                const float d = x[i + 8 * j + l] - y[i + 8 * j + l];
                acc[j][l] = __builtin_fmaf(d, d, acc[j][l]);
            }
    }
    float t = 0.f;
    for (; i < n; ++i) {
        const float d = x[i] - y[i];
        t = __builtin_fmaf(d, d, t);
    }
    float s[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) s[l] = (acc[0][l] + acc[1][l]) + (acc[2][l] + acc[3][l]);
    float v0 = s[0] + s[4], v1 = s[1] + s[5], v2 = s[2] + s[6], v3 = s[3] + s[7];
    v0 = t + v0;
    v1 = 0.0f + v1;
    v2 = 0.0f + v2;
    v3 = 0.0f + v3;
    return (v0 + v1) + (v2 + v3);
}

// Key order used for ids: (dist, id) ascending.
__device__ __forceinline__ bool key_less(float da, uint32_t ia, float db, uint32_t ib) {
    return da < db || (da == db && (ia & WV_IDMASK) < (ib & WV_IDMASK));
}
// The same order without short-circuit evaluation, for compares inside
// ballots and selection chains: the || / && form can compile to exec-mask
// branches around each compare (round 5, finalize sorts: ~10x their cost);
// this one is three compares and two mask ops.  (Not the default: in the
// HNSW LDS-path kernels it raised VGPRs 72 -> 139.)
__device__ __forceinline__ bool key_less_nb(float da, uint32_t ia, float db, uint32_t ib) {
    return (da < db) | ((da == db) & ((ia & WV_IDMASK) < (ib & WV_IDMASK)));
}

__device__ __forceinline__ bool bit_test(const uint64_t* __restrict__ bits, uint64_t nbits, uint64_t id) {
    return id < nbits && ((bits[id >> 6] >> (id & 63)) & 1ull);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// exclusive prefix count of set bits below this lane
__device__ __forceinline__ int mbcnt64(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}
