// wv_bf.hip -- exact (and allowList-filtered) brute-force k-NN on CDNA4.
//
// Restates flatSearch (adapters/repos/db/vector/hnsw/flat_search.go:19-74) over
// the whole corpus or an allow list, with ids returned in (distance, id) order.
//
// Pipeline (per query batch):
//   1. wv_bf_mfma_kernel: fp32 MFMA (v_mfma_f32_32x32x2_f32) base x query tiles.
//      The epilogue turns each dot product into a rank-equivalent approximate
//      distance (L2: |x|^2 - 2 q.x, dot/cosine: -q.x), masks tombstones and
//      the allow list, and keeps per-lane sorted candidate lists in registers.
//      Q x N distances never reach HBM.
//   2. wv_bf_finalize_kernel: one wave per query merges the candidate lists,
//      re-ranks the best KF exactly with the reference summation order
//      (wv_device.h exact_dist_group8) and certifies the result: every point
//      not re-ranked has approx >= bound, and bound - eps > d_k, where eps
//      bounds |approx - reference| for any point.  Uncertified queries are
//      flagged and answered by the exact full scan (wv_exact_scan_kernel).
//   3. wv_exact_scan_kernel + radix sort: exact reference-order distances for
//      every id, used for flagged queries and for large k.
#include "wv_device.h"
#include "wv_params.h"
#include "wv_topk.h"

#include <float.h>

namespace wv {


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));




__device__ __forceinline__ void list_insert(float (&ld)[BF_KP], uint32_t (&li)[BF_KP], float d, uint32_t id) {
    // bubble the new element through the sorted list; the largest falls off
#pragma unroll
    for (int i = 0; i < BF_KP; ++i) {
        const bool lt = key_less(d, id, ld[i], li[i]);
        const float td = ld[i];
        const uint32_t ti = li[i];
        ld[i] = lt ? d : ld[i];
        li[i] = lt ? id : li[i];
        d = lt ? td : d;
        id = lt ? ti : id;
    }
}

// LDS: two stages of {base tile [128][LDT], query tile [128][LDT]} plus the
// |x|^2 of the tile's rows (two tile parities).  Rows are k-contiguous; the
// MFMA k order is permuted so each lane streams 16 consecutive k of its row
// with ds_read_b128 (lane half h takes k = 16h .. 16h+15 of the chunk; A and
// B use the same permutation, so the dot products are unchanged).
#ifndef WV_BF_WAVES_PER_SIMD
#define WV_BF_WAVES_PER_SIMD 2
#endif
constexpr int BF_STAGE = 2 * BF_BQ * BF_LDT;     // floats per stage (A + B)
constexpr size_t BF_LDS_BYTES = (2 * BF_STAGE + 2 * BF_BN) * sizeof(float);

// Layout contract (host side, wv_api.hip): the corpus allocation is padded to a
// whole number of BF_BN-row tiles and the B operand to whole BF_BQ-row query
// blocks (zero rows), so tile loads need no row bounds checks; KFULL (D a
// multiple of BF_BK) drops the k check too.  Rows past N and padded queries
// are masked in the epilogue.
template <bool KFULL>
__global__ __launch_bounds__(256, WV_BF_WAVES_PER_SIMD) void wv_bf_mfma_kernel(BfParams p) {
    extern __shared__ float lds[];
    float* xnb = lds + 2 * BF_STAGE;          // [2][BN] |x|^2 per tile parity

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    // wave-uniform values kept in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1;   // base-row half of the tile
    const int wn = wave & 1;    // query half of the tile
    const int nk = (p.D + BF_BK - 1) / BF_BK;
    const int khalf = lane >> 5;
    const int l31 = lane & 31;
    const uint64_t tomb_words = (p.tomb_nbits + 63) / 64;
    const uint64_t allow_words = (p.allow_nbits + 63) / 64;
    const uint64_t* __restrict__ tomb = p.tomb;
    const uint64_t* __restrict__ allow = p.allow;
    // compacted rows (shared allow list below half the corpus): tile row r is
    // corpus row rowidx[r]; p.N counts compacted rows, no bitmap is applied
    const uint32_t* __restrict__ rowidx = p.rowidx;
    // this thread's slice of a chunk load: rows lrow + 32*it, floats 4*lf4..+3
    const int lrow = tid >> 3, lf4 = tid & 7;
    const uint32_t xoff = (uint32_t)lrow * p.ldx + 4 * lf4;
    const uint32_t qoff = (uint32_t)lrow * p.ldq + 4 * lf4;
    // locality bit 1: logical block ids contiguous per XCD (blocks are dealt
    // round-robin over the 8 XCDs), so one XCD's L2 serves the query blocks of
    // ~1/8 of the batch instead of all of them
    int lb = (int)blockIdx.x;
    if ((p.locality & 1) && gridDim.x % 8 == 0) lb = (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8);
    const uint64_t u_first = (uint64_t)lb * p.units_per_block;
    uint64_t u_last = u_first + p.units_per_block;
    if (u_last > (uint64_t)p.n_qblocks * p.ntiles) u_last = (uint64_t)p.n_qblocks * p.ntiles;

    // one segment per query block touched by this block's run of units
    for (uint64_t u = u_first; u < u_last;) {
        const int qb = (int)(u / p.ntiles);
        const uint64_t t_begin = u % p.ntiles;
        uint64_t t_end = t_begin + (u_last - u);
        if (t_end > p.ntiles) t_end = p.ntiles;
        u += t_end - t_begin;
        const int slot = lb - bf_first_block(qb, p.ntiles, p.units_per_block);
        // locality bit 2: query block qb visits its tiles rotated by rot(qb) =
        // the offset of its first block boundary, so every block starts at a
        // corpus tile that is a multiple of units_per_block and concurrent
        // blocks of different query blocks stream the same tiles (one L2/MALL
        // fill serves them all).  A bijection on the tiles of qb; results do
        // not depend on the visiting order (lists compare (key, id)).
        uint64_t rt_begin = t_begin;
        if (p.locality & 2) {
            const uint64_t rot = ((p.units_per_block - (uint64_t)qb * p.ntiles % p.units_per_block) %
                                  p.units_per_block) % p.ntiles;
            rt_begin = t_begin >= rot ? t_begin - rot : t_begin + p.ntiles - rot;
        }
        const int q0 = qb * BF_BQ;
        const int jq0 = q0 + wn * 64 + l31;   // this lane's two query columns
        const int jq1 = jq0 + 32;
        const float* __restrict__ qblk = p.Q + (uint64_t)q0 * p.ldq;

        // per-lane candidate lists (sorted, BF_KP entries) for its two query columns
        float l0d[BF_KP], l1d[BF_KP];
        uint32_t l0i[BF_KP], l1i[BF_KP];
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            l0d[i] = FLT_MAX; l1d[i] = FLT_MAX;
            l0i[i] = WV_NIL; l1i[i] = WV_NIL;
        }
        float4 ra[4], rb[4];
        float rxn = 0.f;
        uint32_t gidx[4] = {0, 0, 0, 0};   // compacted path: corpus rows of the tile being loaded
        const int total = (int)(t_end - t_begin) * nk;   // chunks of this segment

        auto load_chunk = [&](int c) {
#ifdef WV_BF_ABLATE_NO_LOADS
            if (c > 1) return;
#endif
            const int kc = c % nk;
#ifdef WV_BF_ABLATE_SAME_TILE
            const uint64_t tile = 0;
#else
            uint64_t tile = rt_begin + (uint64_t)(c / nk);
            if (tile >= p.ntiles) tile -= p.ntiles;
#endif
            const float* __restrict__ xt = p.X + tile * BF_BN * p.ldx + kc * BF_BK;
            const float* __restrict__ qt = qblk + kc * BF_BK;
            const bool kin = KFULL || kc * BF_BK + 4 * lf4 < p.D;
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const uint32_t ro = (uint32_t)(32 * it);
                if (rowidx && kc == 0) gidx[it] = rowidx[tile * BF_BN + lrow + ro];   // once per tile
                if (kin) {
                    if (rowidx) {   // compacted allow list: row gather
                        ra[it] = ld4(p.X + (uint64_t)gidx[it] * p.ldx + kc * BF_BK + 4 * lf4);
                    } else {
                        ra[it] = ld4(xt + xoff + ro * p.ldx);
                    }
                    rb[it] = ld4(qt + qoff + ro * p.ldq);
                } else {
                    ra[it] = make_float4(0.f, 0.f, 0.f, 0.f);
                    rb[it] = ra[it];
                }
            }
            if (kc == 0 && tid < BF_BN && p.metric == WV_METRIC_L2)
                rxn = p.xnorm[rowidx ? (uint64_t)rowidx[tile * BF_BN + tid] : tile * BF_BN + tid];
        };
        auto store_chunk = [&](int c) {
            float* st = lds + (c & 1) * BF_STAGE;
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const int row = lrow + 32 * it;
                *reinterpret_cast<float4*>(st + row * BF_LDT + 4 * lf4) = ra[it];
                *reinterpret_cast<float4*>(st + BF_BQ * BF_LDT + row * BF_LDT + 4 * lf4) = rb[it];
            }
            if ((c % nk) == 0 && tid < BF_BN) xnb[((c / nk) & 1) * BF_BN + tid] = rxn;
        };

        if (total > 0) {
            load_chunk(0);
            store_chunk(0);
        }
        __syncthreads();

        const int arow = (wm * 64 + l31) * BF_LDT + 16 * khalf;
        const int brow = BF_BQ * BF_LDT + (wn * 64 + l31) * BF_LDT + 16 * khalf;
        const int ntile = (int)(t_end - t_begin);
        int c = 0;   // chunk counter: stage c & 1 holds chunk c
        for (int t = 0; t < ntile; ++t) {
            uint64_t tile = rt_begin + (uint64_t)t;
            if (tile >= p.ntiles) tile -= p.ntiles;
            // eligibility of this wave's 64 base rows, fetched now so the
            // loads complete under the tile's MFMAs: not excluded, < N, and
            // allowed (shared list: wave-uniform; per-query list: per lane)
            const uint64_t row0 = tile * BF_BN + wm * 64;
            const uint64_t word = row0 >> 6;
            uint64_t okw = ~0ull;
            if (row0 + 64 > p.N) okw = p.N > row0 ? ((1ull << (p.N - row0)) - 1) : 0ull;
            if (tomb && word < tomb_words) okw &= ~tomb[word];
            uint64_t aq0 = ~0ull, aq1 = ~0ull;
            if (allow) {
                if (p.allow_stride && rowidx) {
                    // compacted rows + per-query lists: tested per row in the epilogue
                } else if (p.allow_stride) {
                    aq0 = (jq0 < p.nq && word < allow_words) ? allow[(uint64_t)jq0 * p.allow_stride + word] : 0ull;
                    aq1 = (jq1 < p.nq && word < allow_words) ? allow[(uint64_t)jq1 * p.allow_stride + word] : 0ull;
                } else {
                    okw &= word < allow_words ? allow[word] : 0ull;
                }
            }
            // C-in of the tile = |x|^2 of the row (L2) or 0: with B = -2q (L2) or
            // -q (dot, cosine) the accumulator ends as the approximate key
            // lane-pair shared tail (as wv_bf_split_kernel): read at the tile start
            const float pt0 = __shfl_xor(l0d[BF_KP - 1], 32, 64);
            const float pt1 = __shfl_xor(l1d[BF_KP - 1], 32, 64);
            floatx16 acc00, acc01, acc10, acc11;
            {
                const float* xn = xnb + (t & 1) * BF_BN + wm * 64;
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
                    if (p.metric == WV_METRIC_L2) {
                        x0 = *reinterpret_cast<const float4*>(xn + 8 * g4 + 4 * khalf);
                        x1 = *reinterpret_cast<const float4*>(xn + 32 + 8 * g4 + 4 * khalf);
                    }
                    const float a0s[4] = {x0.x, x0.y, x0.z, x0.w}, a1s[4] = {x1.x, x1.y, x1.z, x1.w};
#pragma unroll
                    for (int r3 = 0; r3 < 4; ++r3) {
                        acc00[4 * g4 + r3] = a0s[r3]; acc01[4 * g4 + r3] = a0s[r3];
                        acc10[4 * g4 + r3] = a1s[r3]; acc11[4 * g4 + r3] = a1s[r3];
                    }
                }
            }
            for (int kc = 0; kc < nk; ++kc, ++c) {
                if (c + 1 < total) load_chunk(c + 1);
                const float* st = lds + (c & 1) * BF_STAGE;
                // operands of k-step group s4+1 are read from LDS while the 16
                // MFMAs of group s4 run (register double buffer)
                float4 fa0[2], fa1[2], fb0[2], fb1[2];
                // valid k of this chunk: a k-group whose both lane halves lie past
                // D (the last chunk when D mod 32 <= 16) carries only zeros
                const int kvalid = KFULL ? BF_BK : min(BF_BK, p.D - kc * BF_BK);
                fa0[0] = *reinterpret_cast<const float4*>(st + arow);
                fa1[0] = *reinterpret_cast<const float4*>(st + arow + 32 * BF_LDT);
                fb0[0] = *reinterpret_cast<const float4*>(st + brow);
                fb1[0] = *reinterpret_cast<const float4*>(st + brow + 32 * BF_LDT);
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) {
                    if (!KFULL && 4 * s4 >= kvalid) break;
                    const int cur = s4 & 1, nxt = cur ^ 1;
                    if (s4 < 3) {
                        fa0[nxt] = *reinterpret_cast<const float4*>(st + arow + 4 * (s4 + 1));
                        fa1[nxt] = *reinterpret_cast<const float4*>(st + arow + 32 * BF_LDT + 4 * (s4 + 1));
                        fb0[nxt] = *reinterpret_cast<const float4*>(st + brow + 4 * (s4 + 1));
                        fb1[nxt] = *reinterpret_cast<const float4*>(st + brow + 32 * BF_LDT + 4 * (s4 + 1));
                    }
                    const float4 a0 = fa0[cur], a1 = fa1[cur], b0 = fb0[cur], b1 = fb1[cur];
#define WV_MF(C) \
    acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.C, b0.C, acc00, 0, 0, 0); \
    acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.C, b1.C, acc01, 0, 0, 0); \
    acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.C, b0.C, acc10, 0, 0, 0); \
    acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.C, b1.C, acc11, 0, 0, 0);
                    WV_MF(x) WV_MF(y) WV_MF(z) WV_MF(w)
#undef WV_MF
                    // 4 LDS reads first, then the 16 MFMAs of this group
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
                }
                // the stage of the last chunk is read by every wave before the
                // next tile's first chunk overwrites the other stage below
                if (c + 1 < total) store_chunk(c + 1);
#ifndef WV_BF_ABLATE_NO_SYNC
                __syncthreads();
#endif
            }
#ifdef WV_BF_ABLATE_NO_EPILOGUE
            asm volatile("" ::"v"(acc00[0]), "v"(acc01[0]), "v"(acc10[0]), "v"(acc11[0]));
            if (acc00[3] == 1234.5f) l0d[0] = acc01[5] + (float)(okw + aq0 + aq1);
            continue;
#endif
            // ---- epilogue of one 128x128 tile ----
            // lane (l31, khalf) holds rows (r & 3) + 8 * (r >> 2) + 4 * khalf of
            // each 32-row half: shift the eligibility words once so every row
            // test is a constant-position bit test
            const uint32_t rb0 = (uint32_t)row0 + 4 * khalf;   // row of acc*0[0]
            const uint64_t o0 = (jq0 < p.nq ? okw & aq0 : 0ull) >> (4 * khalf);
            const uint64_t o1 = (jq1 < p.nq ? okw & aq1 : 0ull) >> (4 * khalf);
            uint32_t o0lo = (uint32_t)o0, o0hi = (uint32_t)(o0 >> 32);
            uint32_t o1lo = (uint32_t)o1, o1hi = (uint32_t)(o1 >> 32);
            if (rowidx && allow && p.allow_stride) {
                // per-query lists over gathered rows (the small delta set of
                // wv_index_add): one bit test per row and query column
                const uint64_t* a0 = allow + (uint64_t)min(jq0, p.nq - 1) * p.allow_stride;
                const uint64_t* a1 = allow + (uint64_t)min(jq1, p.nq - 1) * p.allow_stride;
                uint32_t g0lo = 0, g0hi = 0, g1lo = 0, g1hi = 0;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int bit = (r & 3) + 8 * (r >> 2);
                    const uint32_t ia = rowidx[rb0 + bit], ib = rowidx[rb0 + 32 + bit];
                    g0lo |= (uint32_t)bit_test(a0, p.allow_nbits, ia) << bit;
                    g0hi |= (uint32_t)bit_test(a0, p.allow_nbits, ib) << bit;
                    g1lo |= (uint32_t)bit_test(a1, p.allow_nbits, ia) << bit;
                    g1hi |= (uint32_t)bit_test(a1, p.allow_nbits, ib) << bit;
                }
                o0lo &= g0lo; o0hi &= g0hi; o1lo &= g1lo; o1hi &= g1hi;
            }
            constexpr uint32_t LANE_ROWS = 0x0F0F0F0Fu;   // bits (r&3) + 8*(r>>2), r < 16
            const float INF = __builtin_inff();
            // pass 1: the accumulators already hold the approximate keys; mask
            // ineligible rows to +inf and take the per-query minimum.  Almost
            // every tile stops here.
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
            float m0 = INF, m1 = INF;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                m0 = min3_raw(m0, acc00[r], acc10[r]);
                m1 = min3_raw(m1, acc01[r], acc11[r]);
            }
            // pass 2 (rare after the first tiles): extract the minimum while it
            // beats the list tail; rows are scanned in ascending id, so among
            // equal keys the smallest id is taken first
            split_extract(m0, acc00, acc10, l0d, l0i, pt0, rb0, rowidx);
            split_extract(m1, acc01, acc11, l1d, l1i, pt1, rb0, rowidx);
        }

        // write this lane's two lists: out[q][slot][producer][KP]
        const int prod = wm * 2 + khalf;
        const size_t per_q = (size_t)p.n_slots * BF_PROD * BF_KP;
        if (jq0 < p.nq) {
            const size_t base = (size_t)jq0 * per_q + ((size_t)slot * BF_PROD + prod) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l0d[i]; p.out_id[base + i] = l0i[i]; }
        }
        if (jq1 < p.nq) {
            const size_t base = (size_t)jq1 * per_q + ((size_t)slot * BF_PROD + prod) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l1d[i]; p.out_id[base + i] = l1i[i]; }
        }
    }   // segments
}

// ---------------------------------------------------------------------------
// Split key pass: bf16x3 on MFMA-native operand images (wv_split_rows_kernel).
//
// Each 32-k chunk is two k-steps of v_mfma_f32_32x32x16_bf16 x 3 (hi*hi +
// hi*lo + lo*hi; the lo*lo term and the rounding of lo are dropped: |error|
// <= 4 * 2^-16 * |x||b|, which the finalize certificate adds to its eps).  The
// keys only rank candidates; every reported distance is the exact
// reference-order re-rank of the finalize.
//
// Data movement, chosen for CDNA4:
//  * the query block's image (128 queries x ldx, NK x 16 KiB) is copied into
//    LDS once per segment and stays resident while the block streams its
//    corpus tiles -- no per-tile query reloads;
//  * corpus operands go global -> registers directly: in the native image one
//    wave-wide 16-byte load is one contiguous 1 KiB operand block, so there is
//    no LDS staging, no ds_write and no workgroup barrier inside the tile loop;
//    the next chunk is prefetched under the current chunk's 24 MFMAs;
//  * without barriers the two resident workgroups of a CU drift apart, so one
//    wave's epilogue (VALU) overlaps another wave's MFMAs.
// Shared allow list / tombstones only, no compacted rows, ldx <= 128 (the host
// picks the LDS-staged fp32 kernel otherwise).  Wave (wm, wn) owns base rows
// 64 wm .. +63 and queries 64 wn .. +63 of the 128 x (64 WN) tile, as in
// wv_bf_mfma_kernel, so the lists and the finalize are shared.
//
// WN = 4 (the default): one 512-thread workgroup per CU holds a 256-query
// block (128 KiB of LDS at D = 128) and its 8 waves sweep the same corpus
// tiles, so every corpus byte fetched from L2/HBM feeds 256 queries instead of
// 128: the 1M x 128 corpus image is streamed 40 times per 10k batch, not 79
// (measured at WN = 2: 50 GB fetched per launch, 5.5 TB/s -- the bound).
template <int NK, bool L2, int WN>
__global__ __launch_bounds__(128 * WN, 4 / WN) void wv_bf_split_kernel(BfParams p) {
    extern __shared__ uint4 qimg[];            // [2 WN query groups][NK][2 s][2 part][64 lanes]
    constexpr int GRP = NK * 4 * 64;           // uint4 per 32-row group of an image
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int khalf = lane >> 5;
    const int l31 = lane & 31;
    const uint64_t tomb_words = (p.tomb_nbits + 63) / 64;
    const uint64_t allow_words = (p.allow_nbits + 63) / 64;
    const uint64_t* __restrict__ tomb = p.tomb;
    const uint64_t* __restrict__ allow = p.allow;
    const uint4* __restrict__ X = reinterpret_cast<const uint4*>(p.X);
    const uint4* __restrict__ Qg = reinterpret_cast<const uint4*>(p.Q);
    int lb = (int)blockIdx.x;
    if ((p.locality & 1) && gridDim.x % 8 == 0) lb = (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8);
    const uint64_t u_first = (uint64_t)lb * p.units_per_block;
    uint64_t u_last = u_first + p.units_per_block;
    if (u_last > (uint64_t)p.n_qblocks * p.ntiles) u_last = (uint64_t)p.n_qblocks * p.ntiles;

    for (uint64_t u = u_first; u < u_last;) {
        const int qb = (int)(u / p.ntiles);
        const uint64_t t_begin = u % p.ntiles;
        uint64_t t_end = t_begin + (u_last - u);
        if (t_end > p.ntiles) t_end = p.ntiles;
        u += t_end - t_begin;
        const int slot = lb - bf_first_block(qb, p.ntiles, p.units_per_block);
        uint64_t rt_begin = t_begin;   // aligned rotation, as in wv_bf_mfma_kernel
        if (p.locality & 2) {
            const uint64_t rot = ((p.units_per_block - (uint64_t)qb * p.ntiles % p.units_per_block) %
                                  p.units_per_block) % p.ntiles;
            rt_begin = t_begin >= rot ? t_begin - rot : t_begin + p.ntiles - rot;
        }
        const int jq0 = qb * 64 * WN + wn * 64 + l31;
        const int jq1 = jq0 + 32;

        __syncthreads();   // the previous segment's reads of qimg are done
        {
            const uint4* __restrict__ src = Qg + (uint64_t)qb * 2 * WN * GRP;
#pragma unroll
            for (int i = 0; i < GRP / 64; ++i) qimg[tid + 128 * WN * i] = src[tid + 128 * WN * i];
        }
        __syncthreads();

        float l0d[BF_KP], l1d[BF_KP];
        uint32_t l0i[BF_KP], l1i[BF_KP];
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            l0d[i] = FLT_MAX; l1d[i] = FLT_MAX;
            l0i[i] = WV_NIL; l1i[i] = WV_NIL;
        }
        const uint4* __restrict__ qw = qimg + 2 * wn * GRP + lane;   // query groups 2 wn, 2 wn + 1
        // corpus operand block of (tile, 32-row half h, chunk c, step s, part)
        auto xsrc = [&](uint64_t tile, int c) { return X + (tile * 4 + 2 * wm) * GRP + c * 256 + lane; };
        // operand ping-pong: chunk c reads xb[c & 1] while chunk c + 1 loads
        // into xb[(c + 1) & 1] (distinct registers, so the loads issue at the
        // chunk start, a whole chunk ahead of their first use)
        uint4 xb[2][8];   // [h][s][part]
        auto load_x = [&](uint4 (&dst)[8], const uint4* src) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 4; ++j) dst[4 * h + j] = src[h * GRP + 64 * j];
        };
        // C-in of a tile's accumulators (L2): |x|^2 of this lane's 32 rows, as
        // the accumulator layout holds them (rows (r & 3) + 8 (r >> 2) + 4 khalf
        // of each 32-row half).  It depends on the row only, so xc0 / xc1 enter
        // as the C operand of the tile's first MFMA on both query halves (no
        // accumulator init moves); dot / cosine start from the constant 0.  The
        // wave stages its 64 norms in a private LDS slot: one dword per lane is
        // loaded a tile ahead (1 VGPR in flight instead of 32) and written at
        // the end of the tile; the layout read is 8 ds_read_b128 at the tile start.
        float* __restrict__ xnl = reinterpret_cast<float*>(qimg + 2 * WN * GRP) + wave * 64;
        float xv = 0.f;
        const int ntile = (int)(t_end - t_begin);
        if (ntile > 0) {
            load_x(xb[0], xsrc(rt_begin, 0));
            if (L2) xnl[lane] = p.xnorm[rt_begin * BF_BN + wm * 64 + lane];
        }
        // eligibility words of a tile's 64 rows (this wave's half): tombstones
        // and the shared allow list, fetched raw one tile ahead with |x|^2 and
        // combined only in that tile's epilogue (a load whose value is used at
        // once is waited for on the spot, and vmcnt drains in issue order)
        uint64_t tw_next = 0, aw_next = ~0ull;
        auto load_words = [&](uint64_t tile) {
            const uint64_t w = (tile * BF_BN + wm * 64) >> 6;
            tw_next = tomb && w < tomb_words ? tomb[w] : 0ull;
            if (allow) aw_next = w < allow_words ? allow[w] : 0ull;
        };
        if (ntile > 0) load_words(rt_begin);
        for (int t = 0; t < ntile; ++t) {
            uint64_t tile = rt_begin + (uint64_t)t;
            if (tile >= p.ntiles) tile -= p.ntiles;
            uint64_t ntl = tile + 1;
            if (ntl >= p.ntiles) ntl -= p.ntiles;
            const uint64_t row0 = tile * BF_BN + wm * 64;
#ifndef WV_BF_NO_SHARED_TAIL
            // lanes l and l ^ 32 keep lists for the same query column: either
            // tail is a valid rejection threshold for both (tails only
            // decrease, so the partner's value from the tile start is still
            // >= its final tail, which the finalize's bound is taken over)
            const float pt0 = __shfl_xor(l0d[BF_KP - 1], 32, 64);
            const float pt1 = __shfl_xor(l1d[BF_KP - 1], 32, 64);
#else
            const float pt0 = FLT_MAX, pt1 = FLT_MAX;
#endif

            floatx16 acc00, acc01, acc10, acc11;
            floatx16 xc0, xc1;
            if (L2) {
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const float4 a = *reinterpret_cast<const float4*>(xnl + 4 * khalf + 8 * g4);
                    const float4 b = *reinterpret_cast<const float4*>(xnl + 32 + 4 * khalf + 8 * g4);
                    xc0[4 * g4] = a.x; xc0[4 * g4 + 1] = a.y; xc0[4 * g4 + 2] = a.z; xc0[4 * g4 + 3] = a.w;
                    xc1[4 * g4] = b.x; xc1[4 * g4 + 1] = b.y; xc1[4 * g4 + 2] = b.z; xc1[4 * g4 + 3] = b.w;
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) { xc0[r] = 0.f; xc1[r] = 0.f; }
            }
#pragma unroll
            for (int c = 0; c < NK; ++c) {
#ifdef WV_BF_ABLATE_NO_LOADS
                if (t == 0 && c == 0)
#endif
                {
                    // unconditional (the last tile prefetches the wrapped next
                    // tile, in bounds and unused): a load issued on one path
                    // only makes the waitcnt pass merge counter states
                    // pessimistically, and the last chunk's MFMAs then wait
                    // for the next tile's operands (vmcnt(0) mid-chunk)
                    if (c + 1 < NK) load_x(xb[(c + 1) & 1], xsrc(tile, c + 1));
                    else load_x(xb[NK & 1], xsrc(ntl, 0));
                }
                if (L2 && c == 0) xv = p.xnorm[ntl * BF_BN + wm * 64 + lane];
                // issue the prefetch before anything of the chunk (the machine
                // scheduler otherwise sinks it behind the first MFMAs)
#ifndef WV_BF_NO_SGB
                __builtin_amdgcn_sched_group_barrier(0x020, 9, 0);
#endif
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int qo = c * 256 + s2 * 128;
                    const bf16x8 bh0 = __builtin_bit_cast(bf16x8, qw[qo]);
                    const bf16x8 bl0 = __builtin_bit_cast(bf16x8, qw[qo + 64]);
                    const bf16x8 bh1 = __builtin_bit_cast(bf16x8, qw[GRP + qo]);
                    const bf16x8 bl1 = __builtin_bit_cast(bf16x8, qw[GRP + qo + 64]);
                    const uint4* cur = xb[c & 1];
                    const bf16x8 ah0 = __builtin_bit_cast(bf16x8, cur[2 * s2]);
                    const bf16x8 al0 = __builtin_bit_cast(bf16x8, cur[2 * s2 + 1]);
                    const bf16x8 ah1 = __builtin_bit_cast(bf16x8, cur[4 + 2 * s2]);
                    const bf16x8 al1 = __builtin_bit_cast(bf16x8, cur[4 + 2 * s2 + 1]);
#ifdef WV_BF_ABLATE_NO_MFMA
                    asm volatile("" ::"v"(ah0), "v"(al0), "v"(ah1), "v"(al1), "v"(bh0), "v"(bl0), "v"(bh1), "v"(bl1));
                    continue;
#endif
                    const bool first = c == 0 && s2 == 0;
                    acc00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al0, bh0, first ? xc0 : acc00, 0, 0, 0);
                    acc01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al0, bh1, first ? xc0 : acc01, 0, 0, 0);
                    acc10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al1, bh0, first ? xc1 : acc10, 0, 0, 0);
                    acc11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al1, bh1, first ? xc1 : acc11, 0, 0, 0);
                    acc00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah0, bl0, acc00, 0, 0, 0);
                    acc01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah0, bl1, acc01, 0, 0, 0);
                    acc10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1, bl0, acc10, 0, 0, 0);
                    acc11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1, bl1, acc11, 0, 0, 0);
                    acc00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah0, bh0, acc00, 0, 0, 0);
                    acc01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah0, bh1, acc01, 0, 0, 0);
                    acc10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1, bh0, acc10, 0, 0, 0);
                    acc11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah1, bh1, acc11, 0, 0, 0);
                }
                // keep each chunk's LDS reads next to its MFMAs (register pressure)
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (NK & 1) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xb[0][j] = xb[1][j];
            }
            if (L2) xnl[lane] = xv;   // this wave's reads of xnl were at the tile start
            // the words are the same on every lane: combine them on the scalar unit
            auto uni64 = [](uint64_t v) {
                return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
            };
            // consume this tile's words before the next tile's load reuses their
            // registers: no loop-carried copy, so the back edge carries no
            // vmcnt(0) (which would wait for the corpus prefetch of the next tile)
            uint64_t okw = ~uni64(tw_next) & uni64(aw_next);
            load_words(ntl);
            if (row0 + 64 > p.N) okw &= p.N > row0 ? ((1ull << (p.N - row0)) - 1) : 0ull;
#ifdef WV_BF_ABLATE_NO_EPILOGUE
            asm volatile("" ::"v"(acc00[0]), "v"(acc01[0]), "v"(acc10[0]), "v"(acc11[0]));
            if (acc00[3] == 1234.5f) l0d[0] = acc01[5] + (float)okw;
            continue;
#endif
            // ---- epilogue of one 128x128 tile (as wv_bf_mfma_kernel) ----
            const uint32_t rb0 = (uint32_t)row0 + 4 * khalf;
            WV_DBG_COUNT(0)
            const float INF = __builtin_inff();
            // scalar fast path: every row eligible and every query column live
            if (okw != ~0ull || (qb + 1) * 64 * WN > p.nq) {
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
#ifdef WV_BF_ABLATE_NO_EXTRACT
            if (m0 == 1234.5f) l0d[0] = m1;
            continue;
#endif
            split_extract(m0, acc00, acc10, l0d, l0i, pt0, rb0);
            split_extract(m1, acc01, acc11, l1d, l1i, pt1, rb0);
        }

        const int prod = wm * 2 + khalf;
        const size_t per_q = (size_t)p.n_slots * BF_PROD * BF_KP;
        if (jq0 < p.nq) {
            const size_t base = (size_t)jq0 * per_q + ((size_t)slot * BF_PROD + prod) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l0d[i]; p.out_id[base + i] = l0i[i]; }
        }
        if (jq1 < p.nq) {
            const size_t base = (size_t)jq1 * per_q + ((size_t)slot * BF_PROD + prod) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l1d[i]; p.out_id[base + i] = l1i[i]; }
        }
    }
}

// ---------------------------------------------------------------------------
// Finalize: one wave per query.

// (fin_key, fin_unkey, bitonic256_wave: wv_topk.h)

// FAST: every query has <= 256 list entries (n_slots * prod * kp): one
// bitonic selection; otherwise the list heads bound a short list that is
// sorted the same way, or (over 256 entries at or below that bound) per-lane
// top-KF runs and a KF-round merge (separate instantiations: one kernel
// holding both needs 210 VGPRs)
template <int METRIC, bool FAST>
__device__ __forceinline__ void finalize_one(const BfFinParams& p, int q, float* sd, uint32_t* si, float* qv,
                                             float* kept_d, uint32_t* kept_i) {
    const int lane = threadIdx.x & 63;
    const int n_lists = (bf_slots_of((uint64_t)(q / p.bq), p.ntiles, p.units_per_block) + p.extra_slot) * p.prod;
    const int kp = p.kp ? p.kp : BF_KP;   // entries per list
    const int n_ent = n_lists * kp;
    const float* cd = p.cand_d + (size_t)q * p.n_slots * p.prod * kp;
    const uint32_t* ci = p.cand_id + (size_t)q * p.n_slots * p.prod * kp;

    // bound from the producers' last entries: anything a producer dropped is >= its KP-th key
    uint64_t bkey = fin_key(FLT_MAX, WV_NIL);
    for (int l = lane; l < n_lists; l += 64) {
        const uint64_t t = fin_key(cd[l * kp + kp - 1], ci[l * kp + kp - 1]);
        bkey = t < bkey ? t : bkey;
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)bkey, m, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(bkey >> 32), m, 64);
        const uint64_t t = ((uint64_t)hi << 32) | lo;
        bkey = t < bkey ? t : bkey;
    }
    float bound;
    uint32_t bound_id;
    fin_unkey(bkey, bound, bound_id);

    // select the FIN_KF smallest (key, id) among all entries
    if constexpr (FAST) {
        // a wave-wide bitonic sort of the (<= 256) entries
        uint64_t kk[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 64 * j + lane;
            const uint32_t id = e < n_ent ? ci[e] : WV_NIL;
            kk[j] = fin_key(id != WV_NIL ? cd[e] : FLT_MAX, id);
        }
        bitonic256_wave(kk, lane);
        if (lane < FIN_KF) fin_unkey(kk[0], sd[lane], si[lane]);
    } else {
        // More entries (the wide-D pass's 64-slot schedules: 1024).  The
        // lists are sorted, so the FIN_KF-th smallest list head T bounds the
        // FIN_KF smallest entries (FIN_KF heads are <= T): sort the heads,
        // keep the entries <= T (a few dozen; compacted into LDS by ballot)
        // and sort those -- two 256-sorts instead of a private top-KF per lane
        // and KF merge rounds (66 + 28 us of dependent VALU / shuffle chains
        // per 1024-entry query at one wave per SIMD; in-kernel stamps)
        bool done = false;
        if (n_lists <= 256) {
            uint64_t hk[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int l = 64 * j + lane;
                const uint32_t id = l < n_lists ? ci[l * kp] : WV_NIL;
                hk[j] = fin_key(id != WV_NIL ? cd[l * kp] : FLT_MAX, id);
            }
            bitonic256_wave(hk, lane);
            const uint64_t T = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(hk[0] >> 32), FIN_KF - 1, 64) << 32) |
                               (uint32_t)__shfl((int)(uint32_t)hk[0], FIN_KF - 1, 64);
            int n_keep = 0;   // (wave-uniform: the loop runs on every lane)
            for (int e0 = 0; e0 < n_ent; e0 += 64 * 8) {
                float dd[8];
                uint32_t ii[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = e0 + 64 * u + lane;
                    ii[u] = e < n_ent ? ci[e] : WV_NIL;
                    dd[u] = e < n_ent ? cd[e] : FLT_MAX;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const bool keep = ii[u] != WV_NIL && fin_key(dd[u], ii[u]) <= T;
                    const uint64_t m = __ballot(keep);
                    const int pos = n_keep + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (keep && pos < 256) { kept_d[pos] = dd[u]; kept_i[pos] = ii[u]; }
                    n_keep += __popcll(m);
                }
            }
            if (n_keep <= 256) {
                __builtin_amdgcn_wave_barrier();
                uint64_t kk[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int e = 64 * j + lane;
                    kk[j] = e < n_keep ? fin_key(kept_d[e], kept_i[e]) : fin_key(FLT_MAX, WV_NIL);
                }
                bitonic256_wave(kk, lane);
                if (lane < FIN_KF) fin_unkey(kk[0], sd[lane], si[lane]);
                done = true;
            }
        }
        if (!done) {
            // more entries: each lane keeps a private sorted top-KF of its share,
            // then KF rounds of a wave-wide argmin over the lane heads
            if (lane < FIN_KF) { sd[lane] = FLT_MAX; si[lane] = WV_NIL; }
            __builtin_amdgcn_wave_barrier();
            // each lane scans its share and keeps a private top-KF in LDS-free registers
            float td[FIN_KF];
            uint32_t ti[FIN_KF];
#pragma unroll
            for (int i = 0; i < FIN_KF; ++i) { td[i] = FLT_MAX; ti[i] = WV_NIL; }
            // (8 entries per lane loaded before any is inserted: one memory
            // round trip per 512 entries, not per 64 -- the wide-D pass's 1000-query
            // batches run one wave per SIMD, where each trip is exposed)
            for (int e0 = lane; e0 < n_ent; e0 += 64 * 8) {
                float dd[8];
                uint32_t ii[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = e0 + 64 * u;
                    ii[u] = e < n_ent ? ci[e] : WV_NIL;
                    dd[u] = e < n_ent ? cd[e] : FLT_MAX;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    float d = dd[u];
                    uint32_t id = ii[u];
                    if (id == WV_NIL) continue;
                    if (!key_less(d, id, td[FIN_KF - 1], ti[FIN_KF - 1])) continue;
#pragma unroll
                    for (int i = 0; i < FIN_KF; ++i) {
                        const bool lt = key_less(d, id, td[i], ti[i]);
                        const float a = td[i];
                        const uint32_t b = ti[i];
                        td[i] = lt ? d : td[i];
                        ti[i] = lt ? id : ti[i];
                        d = lt ? a : d;
                        id = lt ? b : id;
                    }
                }
            }
            // wave merge: FIN_KF rounds of argmin over the lane heads
            int head = 0;
            for (int r = 0; r < FIN_KF; ++r) {
                float hd = FLT_MAX;
                uint32_t hi = WV_NIL;
#pragma unroll
                for (int i = 0; i < FIN_KF; ++i)
                    if (i == head) { hd = td[i]; hi = ti[i]; }
                float md = hd;
                uint32_t mi = hi;
                for (int m = 32; m >= 1; m >>= 1) {
                    const float od = __shfl_xor(md, m, 64);
                    const uint32_t oi = __shfl_xor(mi, m, 64);
                    if (key_less(od, oi, md, mi)) { md = od; mi = oi; }
                }
                if (hi == mi && hd == md && mi != WV_NIL) head++;
                if (lane == 0) { sd[r] = md; si[r] = mi; }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    // the KF-th approx key bounds every entry not selected
    {
        const float dk = sd[FIN_KF - 1];
        const uint32_t ik = si[FIN_KF - 1];
        if (key_less(dk, ik, bound, bound_id)) { bound = dk; bound_id = ik; }
    }
    // f16 keys carry the power-of-two scale s = s_x * s_q (exact to undo);
    // a seeded pass dropped every key above its threshold, which therefore
    // also bounds what was not seen
    if (p.h16 && bound != FLT_MAX) bound *= 1.0f / (p.sx * p.qscale[0]);
    if (p.tau_in) bound = fminf(bound, p.tau_in[q]);

    // query into LDS for the exact distance
    for (int i = lane; i < ((p.D + 3) & ~3); i += 64) qv[i] = i < p.D ? p.Q[(size_t)q * p.ldq + i] : 0.f;
    __builtin_amdgcn_wave_barrier();

    // exact re-rank of the FIN_KF candidates: 8 lanes per row, all FIN_KF
    // rows' loads of a slab in flight together (exact_dist_rows; the same
    // arithmetic as exact_dist_group8).  The selection put the nil entries
    // (key FLT_MAX, largest id) last, and their keys stay FLT_MAX.
    int n_sel = 0;
    for (int j = 0; j < FIN_KF; ++j) n_sel += (si[j] != WV_NIL);
    __builtin_amdgcn_wave_barrier();
    if (p.rowidx) {
        // compacted scan: positions -> rows; a position past the list (none
        // expected) drops out, and the rows stay a prefix of n_sel entries
        // (exact_dist_rows loads exactly those), the rest keyed FLT_MAX
        const uint64_t nr = p.rowidx_ndev ? (uint64_t)*p.rowidx_ndev : p.rowidx_n;
        uint32_t v = WV_NIL;
        if (lane < FIN_KF && si[lane] != WV_NIL && si[lane] < nr) v = p.rowidx[si[lane]];
        const uint64_t vm = __ballot(v != WV_NIL);
        __builtin_amdgcn_wave_barrier();
        if (lane < FIN_KF) si[lane] = WV_NIL;
        __builtin_amdgcn_wave_barrier();
        if (v != WV_NIL) si[mbcnt64(vm)] = v;
        n_sel = __popcll(vm);
        if (lane < FIN_KF && lane >= n_sel) sd[lane] = FLT_MAX;
        __builtin_amdgcn_wave_barrier();
    }
    exact_dist_rows<METRIC, FIN_KF / 8>(qv, p.X, p.ldx, p.D, si, n_sel, sd, lane);
    __builtin_amdgcn_wave_barrier();
    // sort the FIN_KF exact keys (rank by counting: lane c < FIN_KF)
    float myd = FLT_MAX;
    uint32_t myi = WV_NIL;
    int rank = 0;
    if (lane < FIN_KF) {
        myd = sd[lane];
        myi = si[lane];
        const uint64_t mykey = fin_key(myd, myi);
        for (int j = 0; j < FIN_KF; ++j)
            rank += fin_key(sd[j], si[j]) < mykey;
    }
    __builtin_amdgcn_wave_barrier();
    const int k = p.k;
    int nvalid = 0;
    for (int j = 0; j < FIN_KF; ++j) nvalid += (si[j] != WV_NIL);
    if (lane < FIN_KF && myi != WV_NIL && rank < k && !p.tau_out) {
        p.out_ids[(size_t)q * k + rank] = p.id_base + myi;
        p.out_d[(size_t)q * k + rank] = myd;
    }
    // k-th exact distance
    float dk = -FLT_MAX;
    const int nk = nvalid < k ? nvalid : k;
    if (lane < FIN_KF && myi != WV_NIL && rank == nk - 1) dk = myd;
    for (int m = 32; m >= 1; m >>= 1) dk = fmaxf(dk, __shfl_xor(dk, m, 64));

    // certificate: eps bounds |approx - reference| for every point
    const float u = 5.9604645e-08f;  // 2^-24
    const float D4 = (float)(p.D + 4);
    float eps, bfull;
    // bf16x3 keys: 3x the accumulated terms, plus the split error
    // 4 * 2^-16 * |x| |b| with b = -2q (L2) or -q
    const float acc_f = p.split ? 12.f : 4.f;
    const float split_e = p.split ? 4.f * 1.52587890625e-05f : 0.f;   // 2^-16
    if (METRIC == WV_METRIC_L2) {
        const float qn = sqrtf(p.qnorm[q]);
        const float s = qn + p.xnorm_max;
        eps = acc_f * D4 * u * s * s + 2.f * split_e * qn * p.xnorm_max;
        bfull = bound + p.qnorm[q];
    } else {
        const float qn = p.qnorm[q];
        eps = acc_f * D4 * u * qn * p.xnorm_max + 4.f * u + split_e * qn * p.xnorm_max;
        bfull = METRIC == WV_METRIC_DOT ? bound : 1.0f + bound;
    }
    eps *= 1.0001f;   // the float evaluation of the bound itself
    // f16 keys: |sum f16(s_x x) f16(s_q b) / (s_x s_q) - x.b| <= |x - x~| |b~| +
    // |x| |b - b~|, with the residual norms measured when the images were made
    if (p.h16) eps = h16_eps(METRIC, p.D, p.qnorm[q], p.xnorm_max, p.ex_max, p.qres[q]);
    if (p.tau_out) {
        // seed pre-pass: every point of the true top k has key <= dk - (the
        // key's offset from the distance) + eps, dk being the k-th exact
        // distance of k real points (an upper bound of the true k-th)
        float tau = __builtin_inff();
        if (nvalid >= k && dk < FLT_MAX) {
            const float off = METRIC == WV_METRIC_L2 ? p.qnorm[q] : (METRIC == WV_METRIC_DOT ? 0.f : 1.0f);
            tau = dk - off + eps;
            tau += 4.f * u * (fabsf(dk) + fabsf(off) + eps) + 1e-3f * eps;   // the rounding of this sum
        }
        if (lane == 0) p.tau_out[q] = tau;
        return;
    }
    bool certified;
    if (nvalid < k) certified = bound == FLT_MAX;     // everything eligible was seen
    else certified = (bound == FLT_MAX) || (bfull - eps > dk);
    if (lane == 0) {
        p.out_n[q] = nk;
        p.fail[q] = certified ? 0 : 1;
        // the re-ranked set holds nk real points with exact distance <= dk:
        // dk bounds the true k-th distance from above (all when nvalid < k)
        p.fail_thr[q] = nvalid < k ? __builtin_inff() : dk;
    }
}

template <bool FAST>
__global__ __launch_bounds__(64) void wv_bf_finalize_kernel(BfFinParams p) {
    // one dynamic region: query (16-byte aligned base), then the KF keys
    extern __shared__ float qv[];
    const int dpad = (p.D + 3) & ~3;
    float* sd = qv + dpad;
    uint32_t* si = reinterpret_cast<uint32_t*>(sd + FIN_KF);
    // (non-FAST: + 256 kept entries)
    float* kept_d = reinterpret_cast<float*>(si + FIN_KF);
    uint32_t* kept_i = reinterpret_cast<uint32_t*>(kept_d + 256);
    const int q = blockIdx.x;
    if (q >= p.nq) return;
    if (p.metric == WV_METRIC_L2) finalize_one<WV_METRIC_L2, FAST>(p, q, sd, si, qv, kept_d, kept_i);
    else if (p.metric == WV_METRIC_DOT) finalize_one<WV_METRIC_DOT, FAST>(p, q, sd, si, qv, kept_d, kept_i);
    else finalize_one<WV_METRIC_COSINE, FAST>(p, q, sd, si, qv, kept_d, kept_i);
}

// ---------------------------------------------------------------------------
// Wide finalize (k > FIN_KF, up to BF_WIDE_KMAX): one 256-thread workgroup per
// query sorts all its list entries in LDS, re-ranks exactly (reference order)
// every entry whose key could still be in the top k -- key <= the k-th key +
// 3 eps -- and certifies the result exactly as finalize_one does: the bound on
// what was not re-ranked is the smallest full-list tail, the first key not
// re-ranked and the seed threshold.
__device__ __forceinline__ void bitonic_sort_lds(float* sd, uint32_t* si, int len) {
    for (int kk = 2; kk <= len; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < len; i += blockDim.x) {
                const int o = i ^ j;
                if (o > i) {
                    const bool asc = (i & kk) == 0;
                    if (key_less(sd[o], si[o], sd[i], si[i]) == asc) {
                        const float td = sd[i]; sd[i] = sd[o]; sd[o] = td;
                        const uint32_t ti = si[i]; si[i] = si[o]; si[o] = ti;
                    }
                }
            }
            __syncthreads();
        }
    }
}

template <int METRIC>
__device__ void finalize_wide(const BfFinParams& p, int q, float* qv, float* sd, uint32_t* si, float* red_d,
                              uint32_t* red_i, int* cnt) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const int n_lists = bf_slots_of((uint64_t)(q / p.bq), p.ntiles, p.units_per_block) * p.prod;
    const int kp = p.kp ? p.kp : BF_KP;   // entries per list
    const int n_ent = n_lists * kp;
    const float* cd = p.cand_d + (size_t)q * p.n_slots * p.prod * kp;
    const uint32_t* ci = p.cand_id + (size_t)q * p.n_slots * p.prod * kp;
    const int NE = p.finw_ne ? p.finw_ne : FINW_NE;   // LDS entry capacity
    // smallest full-list tail: everything a list dropped is >= its tail
    float bound = FLT_MAX;
    uint32_t bound_id = WV_NIL;
    for (int l = tid; l < n_lists; l += nt) {
        const float d = cd[l * kp + kp - 1];
        const uint32_t i = ci[l * kp + kp - 1];
        if (key_less(d, i, bound, bound_id)) { bound = d; bound_id = i; }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const float od = __shfl_xor(bound, m, 64);
        const uint32_t oi = __shfl_xor(bound_id, m, 64);
        if (key_less(od, oi, bound, bound_id)) { bound = od; bound_id = oi; }
    }
    if (tid == 0) *cnt = 0;
    if ((tid & 63) == 0) { red_d[tid >> 6] = bound; red_i[tid >> 6] = bound_id; }
    __syncthreads();
    for (int w = 0; w < (nt >> 6); ++w)
        if (key_less(red_d[w], red_i[w], bound, bound_id)) { bound = red_d[w]; bound_id = red_i[w]; }
    // every valid entry into LDS (the host sizes the lists so they fit)
    for (int e = tid; e < n_ent; e += nt) {
        const uint32_t id = ci[e];
        if (id == WV_NIL) continue;
        const int pos = atomicAdd(cnt, 1);
        if (pos < NE) { sd[pos] = cd[e]; si[pos] = id; }
    }
    __syncthreads();
    const int n_all = *cnt;
    const int n = n_all < NE ? n_all : NE;
    int len = 1;
    while (len < n) len <<= 1;
    for (int i = n + tid; i < len; i += nt) { sd[i] = FLT_MAX; si[i] = WV_NIL; }
    for (int i = tid; i < ((p.D + 3) & ~3); i += nt) qv[i] = i < p.D ? p.Q[(size_t)q * p.ldq + i] : 0.f;
    __syncthreads();
    bitonic_sort_lds(sd, si, len);

    // certificate eps (true units) and the key scale
    const float u = 5.9604645e-08f;
    const float D4 = (float)(p.D + 4);
    float eps;
    const float acc_f = p.split ? 12.f : 4.f;
    const float split_e = p.split ? 4.f * 1.52587890625e-05f : 0.f;
    if (METRIC == WV_METRIC_L2) {
        const float qn = sqrtf(p.qnorm[q]);
        const float s = qn + p.xnorm_max;
        eps = acc_f * D4 * u * s * s + 2.f * split_e * qn * p.xnorm_max;
    } else {
        const float qn = p.qnorm[q];
        eps = acc_f * D4 * u * qn * p.xnorm_max + 4.f * u + split_e * qn * p.xnorm_max;
    }
    eps *= 1.0001f;
    if (p.h16) eps = h16_eps(METRIC, p.D, p.qnorm[q], p.xnorm_max, p.ex_max, p.qres[q]);
    const float ks = p.h16 ? p.sx * p.qscale[0] : 1.f;   // key = ks * true-unit key
    const int k = p.k;
    // re-rank every entry that may beat the k-th key by the keys' error
    int kf = n < k ? n : k;
    if (n > k) {
        const float lim = sd[k - 1] + 3.f * eps * ks * 1.001f;
        // sd is sorted: count entries <= lim among the first FINW_KF
        int c = 0;
        for (int i = tid; i < n && i < FINW_KF; i += nt) c += sd[i] <= lim;
        for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
        __syncthreads();
        if ((tid & 63) == 0) red_i[tid >> 6] = (uint32_t)c;
        __syncthreads();
        c = 0;
        for (int w = 0; w < (nt >> 6); ++w) c += (int)red_i[w];
        kf = c > kf ? c : kf;
        if (kf > FINW_KF) kf = FINW_KF;
        if (kf < n && key_less(sd[kf], si[kf], bound, bound_id)) { bound = sd[kf]; bound_id = si[kf]; }
    }
    if (n_all > NE) bound = -FLT_MAX;   // entries were lost: never certify
    if (p.h16 && bound != FLT_MAX && bound != -FLT_MAX) bound *= 1.0f / ks;
    if (p.tau_in) bound = fminf(bound, p.tau_in[q]);
    __syncthreads();
    // exact distances of the kf candidates (8 lanes per row), in place
    const int g = tid & 7, grp = tid >> 3, ngrp = nt >> 3;
    for (int c0 = 0; c0 < kf; c0 += ngrp) {
        const int c = c0 + grp;
        float d = FLT_MAX;
        uint32_t id = WV_NIL;
        if (c < kf) {
            id = si[c];
            d = exact_dist_group8<METRIC, 8>(qv, p.X + (size_t)id * p.ldx, p.D, g);
        }
        __syncthreads();
        if (c < kf && g == 0) sd[c] = d;
        __syncthreads();
    }
    int len2 = 1;
    while (len2 < kf) len2 <<= 1;
    for (int i = kf + tid; i < len2; i += nt) { sd[i] = FLT_MAX; si[i] = WV_NIL; }
    __syncthreads();
    bitonic_sort_lds(sd, si, len2);
    const int nk = kf < k ? kf : k;
    for (int i = tid; i < nk; i += nt) {
        p.out_ids[(size_t)q * k + i] = p.id_base + si[i];
        p.out_d[(size_t)q * k + i] = sd[i];
    }
    if (tid == 0) {
        const float dk = nk > 0 ? sd[nk - 1] : -FLT_MAX;
        float bfull;
        if (METRIC == WV_METRIC_L2) bfull = bound + p.qnorm[q];
        else bfull = METRIC == WV_METRIC_DOT ? bound : 1.0f + bound;
        bool certified;
        if (n < k) certified = bound == FLT_MAX;
        else certified = (bound == FLT_MAX) || (bfull - eps > dk);
        p.out_n[q] = nk;
        p.fail[q] = certified ? 0 : 1;
        p.fail_thr[q] = n < k ? __builtin_inff() : dk;
    }
}

__global__ __launch_bounds__(256) void wv_bf_finalize_wide_kernel(BfFinParams p) {
    extern __shared__ float lds_w[];
    const int dpad = (p.D + 3) & ~3;
    float* qv = lds_w;
    float* sd = qv + dpad;
    const int NE = p.finw_ne ? p.finw_ne : FINW_NE;
    uint32_t* si = reinterpret_cast<uint32_t*>(sd + NE);
    float* red_d = reinterpret_cast<float*>(si + NE);
    uint32_t* red_i = reinterpret_cast<uint32_t*>(red_d + 4);
    int* cnt = reinterpret_cast<int*>(red_i + 4);
    const int q = blockIdx.x;
    if (q >= p.nq) return;
    if (p.metric == WV_METRIC_L2) finalize_wide<WV_METRIC_L2>(p, q, qv, sd, si, red_d, red_i, cnt);
    else if (p.metric == WV_METRIC_DOT) finalize_wide<WV_METRIC_DOT>(p, q, qv, sd, si, red_d, red_i, cnt);
    else finalize_wide<WV_METRIC_COSINE>(p, q, qv, sd, si, red_d, red_i, cnt);
}

// ---------------------------------------------------------------------------
// Exact full scan for one query: dist[i] = reference-order distance, or +inf
// when ineligible.  8 lanes per row, 32 rows per 256-thread block pass.

template <int METRIC>
__device__ void scan_rows(const ScanParams& p, const float* qv) {
    const int g = threadIdx.x & 7;
    const uint64_t grp = (uint64_t)blockIdx.x * (blockDim.x >> 3) + (threadIdx.x >> 3);
    const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 3);
    for (uint64_t r = grp; r < p.N; r += stride) {
        const float d = exact_dist_group8<METRIC>(qv, p.X + r * p.ldx, p.D, g);
        bool ok = true;
        if (p.tomb) ok = !bit_test(p.tomb, p.tomb_nbits, r);
        if (p.allow && ok) ok = bit_test(p.allow, p.allow_nbits, r);
        if (g == 0) {
            p.dist[r] = ok ? d : __builtin_inff();
            p.ids[r] = (uint32_t)r;
        }
    }
}

__global__ __launch_bounds__(256) void wv_exact_scan_kernel(ScanParams p) {
    extern __shared__ float qv[];
    // the tail reads whole float4s: zero-fill up to the padded length
    for (int i = threadIdx.x; i < ((p.D + 3) & ~3); i += blockDim.x) qv[i] = i < p.D ? p.q[i] : 0.f;
    __syncthreads();
    if (p.metric == WV_METRIC_L2) scan_rows<WV_METRIC_L2>(p, qv);
    else if (p.metric == WV_METRIC_DOT) scan_rows<WV_METRIC_DOT>(p, qv);
    else scan_rows<WV_METRIC_COSINE>(p, qv);
}

// ---------------------------------------------------------------------------
// Certificate fallback, batched over failed queries (see FbParams).
template <int METRIC>
__device__ void fb_filter(const FbParams& p, const float* qv, int f) {
    const int g = threadIdx.x & 7;
    const uint64_t grp = (uint64_t)blockIdx.x * (blockDim.x >> 3) + (threadIdx.x >> 3);
    const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 3);
    const int q = p.qidx[f];
    const float thr = p.thr[q];
    const uint64_t* al = p.allow ? p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0) : nullptr;
    for (uint64_t r = grp; r < p.N; r += stride) {
        const float d = exact_dist_group8<METRIC>(qv, p.X + r * p.ldx, p.D, g);
        if (g == 0 && d <= thr) {
            bool ok = true;
            if (p.tomb) ok = !bit_test(p.tomb, p.tomb_nbits, r);
            if (al && ok) ok = bit_test(al, p.allow_nbits, r);
            if (ok) {
                const uint32_t pos = atomicAdd(&p.cand_n[f], 1u);
                if (pos < FB_CAP) {
                    p.cand_d[(size_t)f * FB_CAP + pos] = d;
                    p.cand_id[(size_t)f * FB_CAP + pos] = (uint32_t)r;
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void wv_fb_filter_kernel(FbParams p) {
    extern __shared__ float qv[];
    const int f = blockIdx.y;
    const int dpad = (p.D + 3) & ~3;
    for (int i = threadIdx.x; i < dpad; i += blockDim.x)
        qv[i] = i < p.D ? p.Q[(size_t)p.qidx[f] * p.ldq + i] : 0.f;
    __syncthreads();
    if (p.metric == WV_METRIC_L2) fb_filter<WV_METRIC_L2>(p, qv, f);
    else if (p.metric == WV_METRIC_DOT) fb_filter<WV_METRIC_DOT>(p, qv, f);
    else fb_filter<WV_METRIC_COSINE>(p, qv, f);
}

// one workgroup per failed query: bitonic sort of the survivors by (d, id)
__global__ __launch_bounds__(1024) void wv_fb_select_kernel(FbParams p) {
    __shared__ float sd[FB_CAP];
    __shared__ uint32_t si[FB_CAP];
    const int f = blockIdx.x;
    const uint32_t n_all = p.cand_n[f];
    const int n = (int)(n_all < (uint32_t)FB_CAP ? n_all : (uint32_t)FB_CAP);
    int len = 1;
    while (len < n) len <<= 1;
    for (int i = threadIdx.x; i < len; i += blockDim.x) {
        sd[i] = i < n ? p.cand_d[(size_t)f * FB_CAP + i] : __builtin_inff();
        si[i] = i < n ? p.cand_id[(size_t)f * FB_CAP + i] : WV_NIL;
    }
    __syncthreads();
    for (int kk = 2; kk <= len; kk <<= 1) {
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < len; i += blockDim.x) {
                const int o = i ^ j;
                if (o > i) {
                    const bool asc = (i & kk) == 0;
                    const bool gt = key_less(sd[o], si[o], sd[i], si[i]);
                    if (gt == asc) {
                        const float td = sd[i]; sd[i] = sd[o]; sd[o] = td;
                        const uint32_t ti = si[i]; si[i] = si[o]; si[o] = ti;
                    }
                }
            }
            __syncthreads();
        }
    }
    const int q = p.qidx[f];
    const int m = n < p.k ? n : p.k;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        p.out_ids[(size_t)q * p.k + i] = p.id_base + si[i];
        p.out_d[(size_t)q * p.k + i] = sd[i];
    }
    if (threadIdx.x == 0) {
        p.out_n[q] = m;
        p.overflow[f] = n_all > (uint32_t)FB_CAP ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// Device-resolved certificate fallback (wv_api.hip queues it after every keyed
// pass and after the HNSW kernel, so a batch needs no host round trip):
//  1. compact: the failed queries (flag != 0) listed in query order, count;
//  2. filter: for each listed query, rows with exact distance <= thr[q] (an
//     upper bound of its true k-th distance) kept, up to FB_CAP;
//  3. select: the survivors sorted by (dist, id), first k written;
//  4. full: a query whose survivors overflowed FB_CAP (ties, thr = +inf for an
//     HNSW query whose side state overflowed) gets every row's distance in a
//     scratch slot, a radix select of the k-th (dist, id) and an ordered
//     collection -- the result of a full sort, as exact_full computes it.
__global__ __launch_bounds__(1024) void wv_fbd_compact_kernel(const int32_t* __restrict__ flags, int nq,
                                                              int32_t* __restrict__ list, int32_t* __restrict__ count,
                                                              unsigned long long* total, uint32_t* __restrict__ cand_n) {
    // each thread owns a contiguous run of flags; one block-wide exclusive
    // scan of the runs' counts places them (two barriers in all)
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (nq + 1023) / 1024;
    const int q0 = tid * per, q1 = min(nq, q0 + per);
    int c = 0;
    for (int q = q0; q < q1; ++q) c += flags[q] != 0;
    int incl = c;   // inclusive scan over the wave
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int off = incl - c, all = 0;
    for (int i = 0; i < 16; ++i) {
        if (i < w) off += wsum[i];
        all += wsum[i];
    }
    for (int q = q0; q < q1; ++q)
        if (flags[q] != 0) list[off++] = q;
    // the filter's per-slot candidate counters start at zero
    for (int i = tid; i < all; i += 1024) cand_n[i] = 0;
    if (tid == 0) {
        *count = all;
        if (total && all) atomicAdd(total, (unsigned long long)all);
    }
}

// HNSW per-query counters [nq][2] (distance evaluations, expansions) summed
// into acc[0], acc[1] on the device (read only when stats are asked for)
__global__ void wv_hnsw_stats_kernel(const uint32_t* __restrict__ ct, int nq, unsigned long long* acc) {
    unsigned long long a = 0, b = 0;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
        a += ct[2 * q];
        b += ct[2 * q + 1];
    }
    for (int m = 32; m >= 1; m >>= 1) {
        a += __shfl_xor(a, m, 64);
        b += __shfl_xor(b, m, 64);
    }
    if ((threadIdx.x & 63) == 0 && (a || b)) {
        atomicAdd(&acc[0], a);
        atomicAdd(&acc[1], b);
    }
}

__global__ void wv_fbd_mark_kernel(const int32_t* __restrict__ status, int nq, int32_t* __restrict__ flags,
                                   float* __restrict__ thr, const float* __restrict__ out_d,
                                   const int32_t* __restrict__ out_n, int k) {
    // HNSW queries whose side state overflowed: exact answer.  Their results
    // so far are eligible rows with exact distances, so the k-th of them (when
    // there are k) bounds the true k-th distance: the filter keeps only rows
    // at or under it (no threshold otherwise)
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const bool f = status[q] != 0;
    flags[q] = f;
    thr[q] = f && out_n && out_n[q] >= k && k > 0 ? out_d[(size_t)q * k + k - 1] : __builtin_inff();
}

template <int METRIC>
__device__ void fbd_filter_one(const FbParams& p, const float* qv, int f, int q) {
    const int g = threadIdx.x & 7;
    const uint64_t grp = (uint64_t)blockIdx.x * (blockDim.x >> 3) + (threadIdx.x >> 3);
    const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 3);
    const float thr = p.thr[q];
    const uint64_t* al = p.allow ? p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0) : nullptr;
    for (uint64_t r = grp; r < p.N; r += stride) {
        const float d = exact_dist_group8<METRIC>(qv, p.X + r * p.ldx, p.D, g);
        if (g == 0 && d <= thr) {
            bool ok = true;
            if (p.tomb) ok = !bit_test(p.tomb, p.tomb_nbits, r);
            if (al && ok) ok = bit_test(al, p.allow_nbits, r);
            if (ok) {
                const uint32_t pos = atomicAdd(&p.cand_n[f], 1u);
                if (pos < FB_CAP) {
                    p.cand_d[(size_t)f * FB_CAP + pos] = d;
                    p.cand_id[(size_t)f * FB_CAP + pos] = (uint32_t)r;
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void wv_fbd_filter_kernel(FbParams p) {
    extern __shared__ float qv[];
    const int nf = *p.d_nf;
    const int dpad = (p.D + 3) & ~3;
    for (int f = 0; f < nf; ++f) {
        const int q = p.qidx[f];
        for (int i = threadIdx.x; i < dpad; i += blockDim.x) qv[i] = i < p.D ? p.Q[(size_t)q * p.ldq + i] : 0.f;
        __syncthreads();
        if (p.metric == WV_METRIC_L2) fbd_filter_one<WV_METRIC_L2>(p, qv, f, q);
        else if (p.metric == WV_METRIC_DOT) fbd_filter_one<WV_METRIC_DOT>(p, qv, f, q);
        else fbd_filter_one<WV_METRIC_COSINE>(p, qv, f, q);
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void wv_fbd_select_kernel(FbParams p) {
    __shared__ float sd[FB_CAP];
    __shared__ uint32_t si[FB_CAP];
    const int nf = *p.d_nf;
    for (int f = blockIdx.x; f < nf; f += gridDim.x) {
        const uint32_t n_all = p.cand_n[f];
        const int n = (int)(n_all < (uint32_t)FB_CAP ? n_all : (uint32_t)FB_CAP);
        int len = 1;
        while (len < n) len <<= 1;
        for (int i = threadIdx.x; i < len; i += blockDim.x) {
            sd[i] = i < n ? p.cand_d[(size_t)f * FB_CAP + i] : __builtin_inff();
            si[i] = i < n ? p.cand_id[(size_t)f * FB_CAP + i] : WV_NIL;
        }
        __syncthreads();
        bitonic_sort_lds(sd, si, len);
        const int q = p.qidx[f];
        const bool over = n_all > (uint32_t)FB_CAP;
        if (!over) {
            const int m = n < p.k ? n : p.k;
            for (int i = threadIdx.x; i < m; i += blockDim.x) {
                p.out_ids[(size_t)q * p.k + i] = p.id_base + si[i];
                p.out_d[(size_t)q * p.k + i] = sd[i];
            }
            if (threadIdx.x == 0) p.out_n[q] = m;
        }
        if (threadIdx.x == 0) p.overflow[f] = over ? 1 : 0;
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t fkey(float d) {   // order-preserving (d1 < d2 <=> key1 < key2)
    const uint32_t b = __float_as_uint(d);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

template <int METRIC>
__device__ void fbd_scan_slot(const FbParams& p, const float* qv, int q, uint32_t* sk) {
    const int g = threadIdx.x & 7;
    const uint64_t* al = p.allow ? p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0) : nullptr;
    for (uint64_t r = threadIdx.x >> 3; r < p.N; r += blockDim.x >> 3) {
        const float d = exact_dist_group8<METRIC>(qv, p.X + r * p.ldx, p.D, g);
        if (g == 0) {
            bool ok = true;
            if (p.tomb) ok = !bit_test(p.tomb, p.tomb_nbits, r);
            if (al && ok) ok = bit_test(al, p.allow_nbits, r);
            sk[r] = ok ? fkey(d) : 0xFFFFFFFFu;
        }
    }
}

constexpr int FBD_K = 256;   // largest k the full-scan slot collects (BF_WIDE_KMAX)

__global__ __launch_bounds__(256) void wv_fbd_full_kernel(FbParams p) {
    extern __shared__ float qv[];
    __shared__ uint32_t hist[256];
    __shared__ float od[FBD_K];
    __shared__ uint32_t oi[FBD_K];
    __shared__ uint32_t s_T, s_need, s_n, s_eq_base;
    __shared__ int wsum[4];
    const int nf = *p.d_nf;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int dpad = (p.D + 3) & ~3;
    uint32_t* sk = reinterpret_cast<uint32_t*>(p.scratch) + (size_t)blockIdx.x * p.N;
    const uint32_t INFK = fkey(__builtin_inff());
    const int k = p.k < FBD_K ? p.k : FBD_K;
    for (int f = blockIdx.x; f < nf; f += gridDim.x) {
        if (!p.overflow[f]) continue;
        const int q = p.qidx[f];
        for (int i = tid; i < dpad; i += blockDim.x) qv[i] = i < p.D ? p.Q[(size_t)q * p.ldq + i] : 0.f;
        __syncthreads();
        if (p.metric == WV_METRIC_L2) fbd_scan_slot<WV_METRIC_L2>(p, qv, q, sk);
        else if (p.metric == WV_METRIC_DOT) fbd_scan_slot<WV_METRIC_DOT>(p, qv, q, sk);
        else fbd_scan_slot<WV_METRIC_COSINE>(p, qv, q, sk);
        __syncthreads();
        // eligible rows (finite distance, as exact_full keeps)
        uint32_t c = 0;
        for (uint64_t r = tid; r < p.N; r += blockDim.x) c += sk[r] < INFK;
        for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m, 64);
        if (lane == 0) wsum[w] = (int)c;
        __syncthreads();
        const uint32_t n_el = (uint32_t)(wsum[0] + wsum[1] + wsum[2] + wsum[3]);
        __syncthreads();
        // T = the k-th smallest key (radix select, 8 bits per pass); need =
        // how many rows equal to T belong to the top k (the smallest ids)
        if (tid == 0) { s_T = INFK; s_need = 0; s_n = 0; s_eq_base = 0; }
        if (n_el > (uint32_t)k) {
            uint32_t prefix = 0, pmask = 0, kk = (uint32_t)k;
            for (int shift = 24; shift >= 0; shift -= 8) {
                hist[tid] = 0;
                __syncthreads();
                for (uint64_t r = tid; r < p.N; r += blockDim.x) {
                    const uint32_t v = sk[r];
                    if ((v & pmask) == prefix) atomicAdd(&hist[(v >> shift) & 255u], 1u);
                }
                __syncthreads();
                if (tid == 0) {
                    uint32_t cum = 0, b = 0;
                    for (; b < 256; ++b) {
                        if (cum + hist[b] >= kk) break;
                        cum += hist[b];
                    }
                    s_need = kk - cum;
                    s_T = prefix | (b << shift);
                }
                __syncthreads();
                kk = s_need;
                prefix = s_T;
                pmask |= 255u << shift;
                __syncthreads();
            }
        }
        __syncthreads();
        const uint32_t T = s_T, need = s_need;
        // ordered collection: every key < T, and the first `need` keys == T
        for (uint64_t c0 = 0; c0 < p.N; c0 += blockDim.x) {
            const uint64_t r = c0 + tid;
            const uint32_t v = r < p.N ? sk[r] : 0xFFFFFFFFu;
            const bool lt = v < T && v < INFK;
            const bool eq = v == T && T < INFK;
            if (lt) {
                const uint32_t pos = atomicAdd(&s_n, 1u);
                if (pos < (uint32_t)FBD_K) { od[pos] = fkey_inv(v); oi[pos] = (uint32_t)r; }
            }
            const uint64_t b = __ballot(eq);
            if (lane == 0) wsum[w] = __popcll(b);
            __syncthreads();
            uint32_t rank = s_eq_base + __popcll(b & ((1ull << lane) - 1ull));
            for (int i = 0; i < w; ++i) rank += (uint32_t)wsum[i];
            if (eq && rank < need) {
                const uint32_t pos = atomicAdd(&s_n, 1u);
                if (pos < (uint32_t)FBD_K) { od[pos] = fkey_inv(v); oi[pos] = (uint32_t)r; }
            }
            __syncthreads();
            if (tid == 0) s_eq_base += (uint32_t)(wsum[0] + wsum[1] + wsum[2] + wsum[3]);
            __syncthreads();
        }
        const int n = (int)(s_n < (uint32_t)k ? s_n : (uint32_t)k);
        int len = 1;
        while (len < n) len <<= 1;
        for (int i = n + tid; i < len; i += blockDim.x) { od[i] = __builtin_inff(); oi[i] = WV_NIL; }
        __syncthreads();
        bitonic_sort_lds(od, oi, len);
        for (int i = tid; i < n; i += blockDim.x) {
            p.out_ids[(size_t)q * p.k + i] = p.id_base + oi[i];
            p.out_d[(size_t)q * p.k + i] = od[i];
        }
        if (tid == 0) p.out_n[q] = n;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// |x|^2 (fp32, any order: only feeds the approximate distance) and max |x|.
__global__ void wv_rownorm_kernel(const float* X, uint64_t N, int D, int ldx, float* norm2,
                                  unsigned int* max_norm_bits) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const float* row = X + r * ldx;
    float s = 0.f;
    for (int i = 0; i < D; i += 4) {
        const float4 v = ld4(row + i);
        s = __builtin_fmaf(v.x, v.x, s);
        s = __builtin_fmaf(v.y, v.y, s);
        s = __builtin_fmaf(v.z, v.z, s);
        s = __builtin_fmaf(v.w, v.w, s);
    }
    if (norm2) norm2[r] = s;
    // slightly inflated |x| (covers the rounding of s and sqrt)
    const float n = sqrtf(s) * (1.0f + 1e-6f);
    atomicMax(max_norm_bits, __float_as_uint(n));
}

// Normalize (distancer/normalize.go:16-32): sequential, unfused sum of squares,
// sqrt in double, IEEE division.  One thread per row, in place or out of place.
__global__ void wv_normalize_kernel(const float* in, float* out, uint64_t n, int D, int ld) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float* v = in + r * ld;
    float* o = out + r * ld;
    float norm = 0.f;
    for (int i = 0; i < D; ++i) {
        const float sq = __fmul_rn(v[i], v[i]);
        norm = __fadd_rn(norm, sq);
    }
    if (norm == 0.f) {
        for (int i = 0; i < D; ++i) o[i] = 0.f;
        return;
    }
    const float nn = (float)sqrt((double)norm);
    for (int i = 0; i < D; ++i) o[i] = __fdiv_rn(v[i], nn);
}

// bf16 hi/lo image of rows for the split key pass, in the MFMA-native layout
// of split_hi_index (wv_params.h): hi = bf16(v), lo = bf16(v - float(hi)),
// v = scale * in (an exact power-of-two scaling), zero past D and for rows >=
// n_valid.  Round to nearest even.  Row r of the launch reads in row
// (ids ? ids[r] : r) and writes image row out_row0 + that.
__device__ __forceinline__ uint16_t bf16_rn(float v) {
    const uint32_t b = __float_as_uint(v);
    return (uint16_t)((b + 0x7FFFu + ((b >> 16) & 1u)) >> 16);
}
__global__ void wv_split_rows_kernel(const float* in, int ld_in, const uint64_t* ids, uint64_t n, uint64_t n_valid,
                                     int D, float scale, uint16_t* out, int ld_out, uint64_t out_row0) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t r = t / (uint64_t)ld_out;
    const int k = (int)(t % (uint64_t)ld_out);
    if (r >= n) return;
    const uint64_t row = ids ? ids[r] : r;
    const float v = (k < D && r < n_valid) ? scale * in[row * ld_in + k] : 0.f;
    const uint16_t hi = bf16_rn(v);
    const uint16_t lo = bf16_rn(v - __uint_as_float((uint32_t)hi << 16));
    const uint64_t o = split_hi_index(out_row0 + row, k, ld_out / BF_BK);
    out[o] = hi;
    out[o + 512] = lo;
}

// B operand of the MFMA pass: -2q (L2) or -q (dot, cosine); exact scalings
__global__ void wv_scale_rows_kernel(const float* in, float* out, uint64_t n, float s) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = s * in[i];
}

// |q|^2 for L2, |q| for dot/cosine (feeds eps only)
// |q|^2 (L2) or |q| per query row: one wave per row (coalesced), optionally
// each block's max |q_i| (absmax_part[block], 4 rows per block).
// The summation order is the wave's tree: the certificate's eps bounds the
// rounding of any order (D u sum q_i^2).
__global__ __launch_bounds__(256) void wv_qnorm_kernel(const float* Q, int nq, int D, int ldq, int metric, float* out,
                                                       float* absmax_part) {
    __shared__ float wmax[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 4 + w;
    float s = 0.f, m = 0.f;
    if (r < nq) {
        const float* q = Q + (size_t)r * ldq;
        for (int i = lane; i < D; i += 64) {
            const float v = q[i];
            s = __builtin_fmaf(v, v, s);
            m = fmaxf(m, fabsf(v));
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        m = fmaxf(m, __shfl_xor(m, o, 64));
    }
    // L2: |q|^2 enters the bound additively (no inflation; eps covers its
    // rounding).  dot/cosine: |q| only scales eps, so it is rounded up.
    if (r < nq && lane == 0) out[r] = metric == WV_METRIC_L2 ? s : sqrtf(s * (1.0f + 1e-6f)) * (1.0f + 1e-6f);
    if (absmax_part) {
        // one partial per block (wv_h16_qscale_kernel reduces them): atomics
        // on one address from thousands of blocks serialise (25 us at 10k)
        if (lane == 0) wmax[w] = m;
        __syncthreads();
        if (threadIdx.x == 0) absmax_part[blockIdx.x] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    }
}

}  // namespace wv

// ---- launch wrappers (host side of this TU) --------------------------------
extern "C" {

hipError_t wv_launch_bf_mfma(const wv::BfParams* p, hipStream_t s) {
    if (p->X == nullptr || p->Q == nullptr) return hipErrorInvalidValue;
    const uint64_t total = (uint64_t)p->n_qblocks * p->ntiles;
    const unsigned nb = (unsigned)((total + p->units_per_block - 1) / p->units_per_block);
    if (nb == 0) return hipSuccess;
    if (p->split) {
        // native images: whole 32-k chunks, query image stride = corpus stride,
        // shared lists only (no compacted rows, no per-query lists)
        const int nk = p->ldx / wv::BF_BK;
        if (p->ldx % wv::BF_BK || p->ldq != p->ldx || nk < 1 || nk > 4 || p->rowidx || p->allow_stride)
            return hipErrorInvalidValue;
        const bool l2 = p->metric == WV_METRIC_L2;
        const bool wide = p->bq == 2 * wv::BF_BQ;
        if (!wide && p->bq != wv::BF_BQ) return hipErrorInvalidValue;
        const size_t lds = (size_t)nk * (wide ? 32768 : 16384) + (wide ? 8 : 4) * 256;   // + per-wave norm slots
#define WV_SPLIT_LAUNCH(NK)                                                                                   \
        if (wide) {                                                                                           \
            if (l2) hipLaunchKernelGGL((wv::wv_bf_split_kernel<NK, true, 4>), dim3(nb), dim3(512), lds, s, *p);  \
            else hipLaunchKernelGGL((wv::wv_bf_split_kernel<NK, false, 4>), dim3(nb), dim3(512), lds, s, *p);    \
        } else {                                                                                              \
            if (l2) hipLaunchKernelGGL((wv::wv_bf_split_kernel<NK, true, 2>), dim3(nb), dim3(256), lds, s, *p);  \
            else hipLaunchKernelGGL((wv::wv_bf_split_kernel<NK, false, 2>), dim3(nb), dim3(256), lds, s, *p);    \
        }
        switch (nk) {
            case 1: WV_SPLIT_LAUNCH(1) break;
            case 2: WV_SPLIT_LAUNCH(2) break;
            case 3: WV_SPLIT_LAUNCH(3) break;
            default: WV_SPLIT_LAUNCH(4) break;
        }
#undef WV_SPLIT_LAUNCH
        return hipGetLastError();
    }
    const size_t lds = wv::BF_LDS_BYTES;
    if (p->D % wv::BF_BK == 0)
        hipLaunchKernelGGL((wv::wv_bf_mfma_kernel<true>), dim3(nb), dim3(256), lds, s, *p);
    else
        hipLaunchKernelGGL((wv::wv_bf_mfma_kernel<false>), dim3(nb), dim3(256), lds, s, *p);
    return hipGetLastError();
}

hipError_t wv_launch_split_rows(const float* in, int ld_in, const uint64_t* ids, uint64_t n, uint64_t n_valid, int D,
                                float scale, void* out, int ld_out, uint64_t out_row0, hipStream_t s) {
    const uint64_t total = n * (uint64_t)ld_out;
    if (total == 0) return hipSuccess;
    if (ld_out % wv::BF_BK) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wv::wv_split_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in, ld_in,
                       ids, n, n_valid, D, scale, static_cast<uint16_t*>(out), ld_out, out_row0);
    return hipGetLastError();
}

hipError_t wv_launch_bf_finalize(const wv::BfFinParams* p, hipStream_t s) {
    const bool fast = (uint64_t)p->n_slots * p->prod * (p->kp ? p->kp : wv::BF_KP) <= 256;
    const size_t lds = (((p->D + 3) & ~3) + 2 * wv::FIN_KF + (fast ? 0 : 512)) * sizeof(float);
    if (fast) hipLaunchKernelGGL(wv::wv_bf_finalize_kernel<true>, dim3(p->nq), dim3(64), lds, s, *p);
    else hipLaunchKernelGGL(wv::wv_bf_finalize_kernel<false>, dim3(p->nq), dim3(64), lds, s, *p);
    return hipGetLastError();
}

hipError_t wv_launch_bf_finalize_wide(const wv::BfFinParams* p, hipStream_t s) {
    if (p->nq == 0) return hipSuccess;
    if (p->k < 1 || p->k > wv::BF_WIDE_KMAX ||
        (uint64_t)p->n_slots * p->prod * (p->kp ? p->kp : wv::BF_KP) > 4ull * wv::FINW_NE)
        return hipErrorInvalidValue;
    // LDS sized by the entries the lists can hold (a power of two, at least
    // the re-rank's FINW_KF): 2048 entries are 17 KB, so 8 workgroups share a
    // CU instead of the 2 that FINW_NE's 64 KB allowed
    const uint64_t ent = (uint64_t)p->n_slots * p->prod * (p->kp ? p->kp : wv::BF_KP);
    int ne = wv::FINW_KF;
    while ((uint64_t)ne < ent && ne < wv::FINW_NE) ne <<= 1;
    wv::BfFinParams pp = *p;
    pp.finw_ne = ne;
    p = &pp;
    const size_t lds = (((p->D + 3) & ~3) + 2 * (size_t)ne + 9) * sizeof(float);
    hipLaunchKernelGGL(wv::wv_bf_finalize_wide_kernel, dim3(p->nq), dim3(256), lds, s, *p);
    return hipGetLastError();
}

hipError_t wv_launch_fb(const wv::FbParams* p, hipStream_t s) {
    if (p->nf == 0) return hipSuccess;
    uint64_t blocks = (p->N + 255) / 256;
    const uint64_t cap = (uint64_t)(2048 / (p->nf > 0 ? p->nf : 1)) + 64;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    const size_t lds = ((p->D + 3) & ~3) * sizeof(float);
    hipLaunchKernelGGL(wv::wv_fb_filter_kernel, dim3((unsigned)blocks, p->nf), dim3(256), lds, s, *p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(wv::wv_fb_select_kernel, dim3(p->nf), dim3(1024), 0, s, *p);
    return hipGetLastError();
}

// the device fallback over `flags` [nq]: fb->qidx / d_nf / overflow / cand_* /
// scratch are [nq]-sized device buffers; flags and fb->thr are read on the device
hipError_t wv_launch_fbd(const int32_t* flags, int nq, const wv::FbParams* fb, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    if (fb->k < 1 || fb->k > wv::FBD_K || !fb->d_nf || !fb->scratch || fb->n_scr < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wv::wv_fbd_compact_kernel, dim3(1), dim3(1024), 0, s, flags, nq, const_cast<int32_t*>(fb->qidx),
                       const_cast<int32_t*>(fb->d_nf), fb->fb_total, fb->cand_n);
    uint64_t blocks = (fb->N + 255) / 256;
    if (blocks > 512) blocks = 512;
    if (blocks == 0) blocks = 1;
    const size_t lds = ((fb->D + 3) & ~3) * sizeof(float);
    hipLaunchKernelGGL(wv::wv_fbd_filter_kernel, dim3((unsigned)blocks), dim3(256), lds, s, *fb);
    hipLaunchKernelGGL(wv::wv_fbd_select_kernel, dim3(64), dim3(1024), 0, s, *fb);
    hipLaunchKernelGGL(wv::wv_fbd_full_kernel, dim3(fb->n_scr), dim3(256), lds, s, *fb);
    return hipGetLastError();
}

hipError_t wv_launch_hnsw_stats(const uint32_t* counters, int nq, unsigned long long* acc, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    unsigned blocks = (unsigned)((nq + 255) / 256);
    if (blocks > 64) blocks = 64;
    hipLaunchKernelGGL(wv::wv_hnsw_stats_kernel, dim3(blocks), dim3(256), 0, s, counters, nq, acc);
    return hipGetLastError();
}

hipError_t wv_launch_fbd_mark(const int32_t* status, int nq, int32_t* flags, float* thr, const float* out_d,
                              const int32_t* out_n, int k, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_fbd_mark_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, status, nq, flags, thr, out_d,
                       out_n, k);
    return hipGetLastError();
}

hipError_t wv_launch_exact_scan(const wv::ScanParams* p, hipStream_t s) {
    uint64_t blocks = (p->N + 31) / 32;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(wv::wv_exact_scan_kernel, dim3((unsigned)blocks), dim3(256), p->D * sizeof(float), s, *p);
    return hipGetLastError();
}

hipError_t wv_launch_rownorm(const float* X, uint64_t N, int D, int ldx, float* norm2, unsigned int* maxbits,
                             hipStream_t s) {
    if (N == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_rownorm_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, X, N, D, ldx,
                       norm2, maxbits);
    return hipGetLastError();
}

hipError_t wv_launch_normalize(const float* in, float* out, uint64_t n, int D, int ld, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_normalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, n, D,
                       ld);
    return hipGetLastError();
}

hipError_t wv_launch_scale(const float* in, float* out, uint64_t n, float scale, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_scale_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, n,
                       scale);
    return hipGetLastError();
}

hipError_t wv_launch_qnorm(const float* Q, int nq, int D, int ldq, int metric, float* out, float* absmax_part,
                           hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_qnorm_kernel, dim3((nq + 3) / 4), dim3(256), 0, s, Q, nq, D, ldq, metric, out,
                       absmax_part);
    return hipGetLastError();
}

}  // extern "C"
