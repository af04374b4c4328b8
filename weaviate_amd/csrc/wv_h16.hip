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

#include "wv_h16_dev.h"

namespace wv {


// SEED: the pre-pass over every H_SAMPLE-th tile keeps only each lane's
// running minimum per query column (distinct rows per (slot, lane half)),
// written as one key per list; wv_h16_seed_kernel turns them into thresholds.
// One 512-query workgroup per CU (two waves per SIMD), H_TPS8 tiles per LDS
// stage, one barrier per stage.
//
// Operand stream (round 4): a half tile's 16 MFMAs read their A fragments two
// k-steps ahead (3 in registers instead of all 8), and the next half's C-in
// and first two fragments are read during the current half's last MFMAs, so
// no half starts by waiting on an LDS round trip (ablation before: the A
// fragments' LDS reads cost 0.35 ms of a 2.66 ms 1M x 10k pass).  The stage
// barrier sits before the first half (A) of a group's last tile: the next
// group's first tile is then landed when A prefetches it.
// the keys min_steps (below) folds at k-steps 0 .. ns - 1: 0-2 at k = 0, 2k+1
// and 2k+2 at k = 1 .. 6, the rest at k = ns - 1
constexpr bool min_steps_cover(int ns) {
    unsigned m = 0;
    for (int k = 0; k < ns; ++k) {
        if (k == 0) m |= 7u;
        else if (k <= 6) m |= 3u << (2 * k + 1);
        if (k == ns - 1)
            for (int r = ns <= 7 ? 2 * ns + 1 : 15; r < 16; ++r) m |= 1u << r;
    }
    return m == 0xFFFFu;
}

template <int NS, bool L2, bool SEED, bool XS = false>
__global__ __launch_bounds__(512, 1) void wv_bf_h16_kernel(H16Params p) {
    static_assert(min_steps_cover(NS), "the spread tile minima must cover all 16 keys of a half");
    constexpr int WAVES = 8, TPS = H_TPS8;
    constexpr int BQ = WAVES * 64;
    constexpr int NSTG = H_STAGES;
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
    if (p.block_order) lb = p.block_order[lb];
    const uint64_t u_first = (uint64_t)lb * p.units_per_block;
    uint64_t u_last = u_first + p.units_per_block;
    if (u_last > (uint64_t)p.n_qblocks * p.ntiles) u_last = (uint64_t)p.n_qblocks * p.ntiles;

    const uint32_t lds0 = lds_addr(lds);
#ifdef WV_H16_PRIO
    // the second-dispatched half of the workgroup loses every issue
    // arbitration to its SIMD partner: static priority for it (guide T5)
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    // this wave's LDS-DMA ops per tile (the counted waits below)
    const int n_ops = (wave < St::IMG_U4 / 64 ? (St::IMG_U4 / 64 - 1 - wave) / WAVES + 1 : 0) +
                      ((wave == 0 && L2) ? 1 : 0);
    // the image words this wave moves per tile (its share, and the s|x|^2
    // word on wave 0): a lane offset per share, computed once
    const uint32_t voff = (uint32_t)(wave * 1024 + lane * 16);
    auto fill = [&](uint64_t t, int st) {
        const uint64_t tile = p.tile_base + t * (uint64_t)p.tile_stride;
        const uint32_t dst = lds0 + (uint32_t)(st * St::U4 * 16) + (uint32_t)(wave * 1024);
        const uint4* src = uniform_ptr(X + tile * St::IMG_U4);
#pragma unroll
        for (int i = 0; i < St::IMG_U4 / 64; i += WAVES)
            if (wave + i < St::IMG_U4 / 64) glds16s(src, voff + (uint32_t)(i * 1024), dst + (uint32_t)(i * 1024));
        if (wave == 0 && L2) glds4(p.xns + tile * H_BN + lane, dst + St::IMG_U4 * 16);
    };

    // the tiles of stage-group g (TPS consecutive tiles) into LDS stage g % 3
    // (locality bit 2: a query block's tiles rotated by its first block's
    // offset, so that every query block's slot boundaries fall on the same
    // tiles -- the blocks scanning a tile together, in one XCD's L2 with the
    // block order; shift 0 otherwise)
    uint64_t shift = 0;
    auto phys = [&](uint64_t t) {
        const uint64_t v = t + shift;
        return v >= p.ntiles ? v - p.ntiles : v;
    };
    auto fill_group = [&](uint64_t t_begin, int g, int ntile) {
        const int st = g % NSTG;
        int n = 0;
#pragma unroll
        for (int j = 0; j < TPS; ++j) {
            const int t = g * TPS + j;
            if (t < ntile) { fill(phys(t_begin + t), st * TPS + j); ++n; }
        }
        return n * n_ops;   // this wave's DMA ops for the group
    };
    // (in the tile loop: the slot of tile t advances by one, wrapping at the ring)
    auto next_slot = [](int sl) { return sl + 1 == NSTG * TPS ? 0 : sl + 1; };

    for (uint64_t u = u_first; u < u_last;) {
        const int qb = (int)(u / p.ntiles);
        const uint64_t t_begin = u % p.ntiles;
        uint64_t t_end = t_begin + (u_last - u);
        if (t_end > p.ntiles) t_end = p.ntiles;
        u += t_end - t_begin;
        const int slot = lb - bf_first_block(qb, p.ntiles, p.units_per_block);
        shift = (p.locality & 2) ? (uint64_t)qb * p.ntiles % p.units_per_block % p.ntiles : 0;
        const int jq0 = qb * BQ + wave * 64 + l31;
        const int jq1 = jq0 + 32;
        // (an aligned schedule's grid pads the corpus's tiles: no work past them)
        const uint64_t t_stop = t_end < p.ntiles_real ? t_end : p.ntiles_real;
        const int ntile = t_stop > t_begin ? (int)(t_stop - t_begin) : 0;

        // the wave's 64 queries as B operands, for the whole segment
        uint4 bq0[NS], bq1[NS];
        {
            const uint64_t g0 = (uint64_t)qb * (BQ / 32) + 2 * wave;
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                bq0[st] = Qg[(g0 * NS + st) * 64 + lane];
                bq1[st] = Qg[((g0 + 1) * NS + st) * 64 + lane];
            }
        }
        float tau0 = FLT_MAX, tau1 = FLT_MAX;
        if (!SEED && p.gtau) {
            if (jq0 < p.nq) tau0 = fminf(FLT_MAX, h16_key_dec(p.gtau[jq0]));
            if (jq1 < p.nq) tau1 = fminf(FLT_MAX, h16_key_dec(p.gtau[jq1]));
        } else if (p.tau) {
            if (jq0 < p.nq) tau0 = fminf(FLT_MAX, p.tau[jq0] * s);
            if (jq1 < p.nq) tau1 = fminf(FLT_MAX, p.tau[jq1] * s);
        }
        // the padding columns of a partial query block never extract (every
        // later threshold update is a min): their tiles need no row mask
        if (jq0 >= p.nq) tau0 = -__builtin_inff();
        if (jq1 >= p.nq) tau1 = -__builtin_inff();
        // the running threshold's margin: 2 eps (scaled) + the rounding of the sum
        float marg0 = 0.f, marg1 = 0.f;
        if (!SEED && p.kth) {
            if (jq0 < p.nq) marg0 = p.marg[jq0];
            if (jq1 < p.nq) marg1 = p.marg[jq1];
        }
        // consume the ordinary loads here, before any LDS-DMA is in flight:
        // the compiler's wait for them is then not a wait for the tile stream
#pragma unroll
        for (int st = 0; st < NS; ++st) asm volatile("" ::"v"(bq0[st].x), "v"(bq1[st].x));
        asm volatile("" ::"v"(tau0), "v"(tau1), "v"(marg0), "v"(marg1));
        float l0d[BF_KP], l1d[BF_KP];
        uint32_t l0i[BF_KP], l1i[BF_KP];
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            l0d[i] = FLT_MAX; l1d[i] = FLT_MAX;
            l0i[i] = WV_NIL; l1i[i] = WV_NIL;
        }
        // Two-phase software pipeline over half tiles (rows 0-31: H0 =
        // acc00/acc01, rows 32-63: H1 = acc10/acc11).  Iteration t:
        //   (group's last tile: group g + 1 landed, barrier)
        //   A  MFMAs of H1(t)       beside the tile minima of H0(t); at its
        //      end the C-in and first fragments of H0(t + 1) are read
        //   B  extraction of H0(t)  (rare)
        //   E  MFMAs of H0(t + 1)   beside the tile minima of H1(t); at its
        //      end the head of H1(t + 1) is read
        //   F  extraction of H1(t)
        const float INF = __builtin_inff();
        floatx16 acc00, acc01, acc10, acc11;
        // the head of the next half: its C-in and k-step 0 / 1 A fragments
        floatx16 xcn;
        uint4 an0, an1;
        auto head = [&](const uint4* img, int rb) {
            if (L2) {
                const float* xn = reinterpret_cast<const float*>(img + St::IMG_U4) + 32 * rb;
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const float4 v = *reinterpret_cast<const float4*>(xn + 4 * khalf + 8 * g4);
                    xcn[4 * g4] = v.x; xcn[4 * g4 + 1] = v.y; xcn[4 * g4 + 2] = v.z; xcn[4 * g4 + 3] = v.w;
                }
            }
            an0 = img[(rb * NS) * 64 + lane];
            if (NS > 1) an1 = img[(rb * NS + 1) * 64 + lane];
        };
        // one half tile's 16 MFMAs (k-interleaved over the two accumulators),
        // its fragments read two k-steps ahead, the VALU work of the other
        // half (`between(k)`, a share per k-step) beside them, and the next
        // half's head read during the last k-steps (after the last tile: a
        // harmless re-read of img).  The order is pinned with scheduling
        // fences: the compiler's own schedule hoisted every read to the
        // front and drained them all before the first MFMA.
        auto mfma_half = [&](const uint4* img, int rb, floatx16& accA, floatx16& accB, auto&& between,
                             const uint4* nimg, int nrb) {
            floatx16 xc;
            if (L2) xc = xcn;
            else {
#pragma unroll
                for (int r = 0; r < 16; ++r) xc[r] = 0.f;
            }
            uint4 a[3];
            a[0] = an0;
            a[1] = an1;
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                __builtin_amdgcn_sched_barrier(0);
#ifdef WV_H16_ABLATE_NO_LDS
                if (k + 2 < NS) { a[(k + 2) % 3] = bq1[k + 2]; a[(k + 2) % 3].x ^= (uint32_t)rb; }
#else
                if (k + 2 < NS) a[(k + 2) % 3] = img[(rb * NS + k + 2) * 64 + lane];
#endif
                // (unconditional: a branch here would make every later wait
                // drain these reads too; with one k-step at k = 0, after the
                // copies above)
                if (k == (NS >= 2 ? NS - 2 : 0)) head(nimg, nrb);
                const half8 ak = __builtin_bit_cast(half8, a[k % 3]);
                accA = __builtin_amdgcn_mfma_f32_32x32x16_f16(ak, __builtin_bit_cast(half8, bq0[k]), k == 0 ? xc : accA,
                                                              0, 0, 0);
                accB = __builtin_amdgcn_mfma_f32_32x32x16_f16(ak, __builtin_bit_cast(half8, bq1[k]), k == 0 ? xc : accB,
                                                              0, 0, 0);
#ifndef WV_H16_XC_INPLACE
                // (xc stays live past both first MFMAs: neither accumulator
                // is allocated in place of the C-in, whose registers the next
                // half's head then reuses -- in place, the head landed on a
                // live accumulator and the compiler copied it out: 8
                // v_mov_b64 + s_nop per half, and the loop-carried C-in once
                // more per tile)
                if (k == 0) asm volatile("" ::"v"(xc));
#endif
                between(k);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        // the minima of a half's two accumulators as `between` work: four
        // v_min3 chains per accumulator, two ops per k-step
        auto min_steps = [&](const floatx16& A, const floatx16& B, float& mA, float& mB) {
            return [&](int k) {
                // (each step pinned by an asm use: IR sinking otherwise moved
                // the whole chain past the MFMAs of phase E to the join with
                // the last tile's min16 -- 16 serial v_min3 per tile)

                // chain c of A covers keys 4c .. 4c + 3; B likewise
                if (k == 0) { mA = fminf(fminf(A[0], A[1]), A[2]); mB = fminf(fminf(B[0], B[1]), B[2]); }
                else if (k == 1) { mA = fminf(fminf(mA, A[3]), A[4]); mB = fminf(fminf(mB, B[3]), B[4]); }
                else if (k == 2) { mA = fminf(fminf(mA, A[5]), A[6]); mB = fminf(fminf(mB, B[5]), B[6]); }
                else if (k == 3) { mA = fminf(fminf(mA, A[7]), A[8]); mB = fminf(fminf(mB, B[7]), B[8]); }
                else if (k == 4) { mA = fminf(fminf(mA, A[9]), A[10]); mB = fminf(fminf(mB, B[9]), B[10]); }
                else if (k == 5) { mA = fminf(fminf(mA, A[11]), A[12]); mB = fminf(fminf(mB, B[11]), B[12]); }
                else if (k == 6) { mA = fminf(fminf(mA, A[13]), A[14]); mB = fminf(fminf(mB, B[13]), B[14]); }
                if (k == NS - 1) {   // (the remaining keys at the last k-step: those after
                                     // key 2 NS when the steps above ran to k = NS - 1, key 15 when
                                     // they stopped at k = 6)
#pragma unroll
                    for (int r = NS <= 7 ? 2 * NS + 1 : 15; r < 16; ++r) { mA = fminf(mA, A[r]); mB = fminf(mB, B[r]); }
                }
                asm volatile("" : "+v"(mA), "+v"(mB));
            };
        };
        // eligibility of a tile's 64 rows for this lane's two columns (bits of
        // rows 4 khalf + ..., low word: rows 0-31, high word: rows 32-63)
        // (the lane-dependent shifts happen only when a tile needs the mask)
        auto tile_ok = [&](uint64_t t, uint64_t& okw) -> bool {
            const uint64_t ct = p.tile_base + t * (uint64_t)p.tile_stride;
            if (ct < p.clean_tiles) {   // (the host's clean prefix: no word to read)
                okw = ~0ull;
                return false;
            }
            okw = tile_okw(p, ct, has_allow);
            return okw != ~0ull;
        };
        auto lane_ok = [&](uint64_t okw, int jq) -> uint64_t { return (jq < p.nq ? okw : 0ull) >> (4 * khalf); };
        // mask a half's ineligible rows to +inf (rows (r & 3) + 8 (r >> 2) of its 32)
        auto mask_half = [&](floatx16& A, floatx16& B, uint32_t oa, uint32_t ob) {
            constexpr uint32_t LANE_ROWS = 0x0F0F0F0Fu;
            if (__all((oa & ob & LANE_ROWS) == LANE_ROWS)) return;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int bit = (r & 3) + 8 * (r >> 2);
                A[r] = (oa >> bit) & 1u ? A[r] : INF;
                B[r] = (ob >> bit) & 1u ? B[r] : INF;
            }
        };
        auto min16 = [&](const floatx16& A) {
#ifdef WV_H16_ABLATE_NO_MIN
            return A[0];
#endif
            // four independent chains (short dependency depth), v_min3 each
            float m0 = fminf(fminf(A[0], A[1]), A[2]), m1 = fminf(fminf(A[3], A[4]), A[5]);
            float m2 = fminf(fminf(A[6], A[7]), A[8]), m3 = fminf(fminf(A[9], A[10]), A[11]);
            m0 = fminf(fminf(m0, A[12]), A[13]);
            m1 = fminf(fminf(m1, A[14]), A[15]);
            return fminf(fminf(m0, m1), fminf(m2, m3));
        };

        uint64_t okw = 0;
        bool need_mask = false;
        // extraction thresholds: min(partner's list tail, running threshold),
        // refreshed only when a list or the threshold changed
        float pt0 = 0.f, pt1 = 0.f;
        auto refresh_pt = [&] {
            pt0 = fminf(__shfl_xor(l0d[BF_KP - 1], 32, 64), tau0);
            pt1 = fminf(__shfl_xor(l1d[BF_KP - 1], 32, 64), tau1);
        };
        refresh_pt();
        // running threshold: k of the pair's list entries bound the k-th key
        // (ia from this lane's list, ib from the partner's), + 2 eps
        // (entries picked by select chains over an opaque VGPR index: a
        // uniform index into register arrays would hold one SGPR mask per
        // entry for the whole loop; the partner's entries arrive by shuffle)
        const int ia = (p.kth + 1) >> 1, ib = p.kth >> 1;
        auto publish = [&] {
            int va = ia - 1, vb = ib - 1;
            asm volatile("" : "+v"(va), "+v"(vb));
            float a0 = -FLT_MAX, a1 = -FLT_MAX, b0 = -FLT_MAX, b1 = -FLT_MAX;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) {
                a0 = va == i ? l0d[i] : a0;
                a1 = va == i ? l1d[i] : a1;
                b0 = vb == i ? l0d[i] : b0;
                b1 = vb == i ? l1d[i] : b1;
            }
            b0 = __shfl_xor(b0, 32, 64);
            b1 = __shfl_xor(b1, 32, 64);
            const float k0 = fmaxf(a0, b0), k1 = fmaxf(a1, b1);
            if (khalf == 0) {
                const float u4 = 4.f * 5.9604645e-08f;
                if (jq0 < p.nq && k0 < FLT_MAX) {
                    const float t = k0 + marg0;
                    atomicMin(&p.gtau[jq0], h16_key_enc(t + u4 * (fabsf(k0) + marg0)));
                }
                if (jq1 < p.nq && k1 < FLT_MAX) {
                    const float t = k1 + marg1;
                    atomicMin(&p.gtau[jq1], h16_key_enc(t + u4 * (fabsf(k1) + marg1)));
                }
            }
            if (jq0 < p.nq) tau0 = fminf(tau0, h16_key_dec(__atomic_load_n(&p.gtau[jq0], __ATOMIC_RELAXED)));
            if (jq1 < p.nq) tau1 = fminf(tau1, h16_key_dec(__atomic_load_n(&p.gtau[jq1], __ATOMIC_RELAXED)));
            refresh_pt();
        };
        const bool running = !SEED && p.kth > 0 && p.gtau != nullptr && !p.xslot;
        // cross-slot threshold: the slots of a query block run side by side
        // over equal tile ranges, so at a fraction f of the segment the heads
        // of all 2 n_slots lists are the minima of disjoint row sets covering
        // f of the corpus; their k-th smallest (+ 2 eps) bounds the k-th key
        // at rank ~ k / f instead of the seed's ~ k H_SAMPLE.  Stored at 1/8,
        // 1/4, 1/2 of the segment, read at 1/4, 1/2, 3/4 (the values the
        // other slots stored one step earlier).  Lane half 0 selects for
        // jq0, lane half 1 for jq1.
        const bool xs = XS && !SEED && p.kth > 0;   // (its own instantiation: the code costs SGPRs)
        auto xslot_step = [&](bool rd, bool wr) {
            const int nv = 2 * p.n_slots;
            if (rd) {
                const int jq = khalf ? jq1 : jq0;
                int nvv = jq < p.nq ? nv : 0;   // (opaque VGPR, as ve below)
                asm volatile("" : "+v"(nvv));
                const float* g = p.gslot + (size_t)jq * nv;
                float v[32];
#pragma unroll
                for (int i = 0; i < 32; ++i)
                    v[i] = i < nvv ? __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : FLT_MAX;
                // ascending bitonic network over the 32 values, then entry k - 1
#pragma unroll
                for (int size = 2; size <= 32; size <<= 1)
#pragma unroll
                    for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
                        for (int i = 0; i < 32; ++i) {
                            const int j = i ^ stride;
                            if (j > i) {
                                const float a = v[i], b = v[j];
                                const bool up = (i & size) == 0;
                                v[i] = up ? fminf(a, b) : fmaxf(a, b);
                                v[j] = up ? fmaxf(a, b) : fminf(a, b);
                            }
                        }
                // (an opaque VGPR index: a uniform one would keep 32 SGPR
                // masks live across the tile loop)
                int ve = p.kth - 1;
                asm volatile("" : "+v"(ve));
                float kv = FLT_MAX;
#pragma unroll
                for (int i = 0; i < 32; ++i) kv = i == ve ? v[i] : kv;
                const float mg = khalf ? marg1 : marg0;
                const float u4 = 4.f * 5.9604645e-08f;
                float b = kv < 1e30f ? kv + mg + u4 * (fabsf(kv) + mg) : FLT_MAX;
                // publish it: the finalize's tau_in (wv_h16_gtau_kernel) must
                // be <= every threshold a key was dropped above
                if (jq < p.nq && b < FLT_MAX) atomicMin(&p.gtau[jq], h16_key_enc(b));
                const float bo = __shfl_xor(b, 32, 64);   // the other half's query
                tau0 = fminf(tau0, khalf ? bo : b);
                tau1 = fminf(tau1, khalf ? b : bo);
                refresh_pt();
            }
            if (wr) {
                const int s2 = 2 * slot + khalf;
                if (jq0 < p.nq && l0d[0] < FLT_MAX)
                    __hip_atomic_store(p.gslot + (size_t)jq0 * nv + s2, l0d[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (jq1 < p.nq && l1d[0] < FLT_MAX)
                    __hip_atomic_store(p.gslot + (size_t)jq1 * nv + s2, l1d[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        // a half's candidates: the column minima against the thresholds, and
        // (rare) insertion of the column minimum (wv_topk.h min_extract)
        auto extract_half = [&](float m0, float m1, floatx16& A, floatx16& B, uint32_t rb) -> bool {
#ifdef WV_H16_ABLATE_NO_EXTRACT
            if (m0 == 1234.5f) l0d[0] = m1 + pt0 + pt1;
            return false;
#endif
#ifdef WV_H16_ABLATE_NO_EVENTS
            // (ablation: the extraction code stays, no event ever fires)
            float nev = -INF;
            asm volatile("" : "+v"(nev));
            const bool x0 = m0 <= fminf(fminf(l0d[BF_KP - 1], pt0), nev), x1 = m1 <= fminf(fminf(l1d[BF_KP - 1], pt1), nev);
#else
            const bool x0 = m0 <= fminf(l0d[BF_KP - 1], pt0), x1 = m1 <= fminf(l1d[BF_KP - 1], pt1);
#endif
            const bool any = __any(x0 || x1);
            if (__builtin_expect(any, 0)) {
                WV_DBG_COUNT(3)
                // (the smallest key by its position; the per-key scan only
                // for a second key under the threshold: 2.645 -> 2.622 ms)
                if (__any(x0)) min_extract(m0, x0, A, pt0, l0d, l0i, rb);
                if (__any(x1)) min_extract(m1, x1, B, pt1, l1d, l1i, rb);
            }
            return any;
        };
        const int xs1 = ntile / 8, xs2 = ntile / 4, xs3 = ntile / 2, xs4 = (3 * ntile) / 4;
        const int ngroups = (ntile + TPS - 1) / TPS;
        // (the previous segment ended with every stage read and every DMA landed)
        int ops_in_flight = 0;   // this wave's DMA ops of the newest group issued
        if (ngroups > 0) fill_group(t_begin, 0, ntile);
        if (ngroups > 1) ops_in_flight = fill_group(t_begin, 1, ntile);
        vm_wait(ops_in_flight);   // this wave's part of group 0
        block_barrier();          // everyone's
        if (ntile > 0) {
            head(lds, 0);
            mfma_half(lds, 0, acc00, acc01, [](int) {}, lds, 1);   // H0(0), then the head of H1(0)
            need_mask = tile_ok(phys(t_begin), okw);
        }
        int slot_t = 0;   // LDS slot of tile t
        // row base of tile t (scalar; wraps with the rotation)
        uint32_t rbase = (uint32_t)(phys(t_begin) * (uint64_t)p.tile_stride * H_BN);
        const uint32_t rb_step = (uint32_t)(p.tile_stride * H_BN), rb_wrap = (uint32_t)(p.ntiles * p.tile_stride * H_BN);
        const uint32_t rb_base = (uint32_t)(p.tile_base * H_BN);   // (rows of the scanned range's first tile)
        int xs_next = XS && xs ? xs1 : -1;   // the next cross-slot exchange tile
        for (int t = 0; t < ntile; ++t) {
            const uint32_t rb0 = rb_base + rbase + 4 * khalf;
            rbase += rb_step;
            if (rbase >= rb_wrap) rbase -= rb_wrap;
            WV_DBG_COUNT(0)
            const int g = t / TPS;
            const uint4* img = lds + slot_t * St::U4;
            slot_t = next_slot(slot_t);
            const bool more = t + 1 < ntile;
            // the group's last tile: group g + 1 landed and every wave is
            // done with tile t - 1, hence with group g - 1's stage (its last
            // reads: phase A of that group's last tile); only then is group
            // g + 2 issued into it -- (g + 2) % 3 = (g - 1) % 3 -- a group's
            // time ahead of its first read.  (Issued at the start of group g
            // instead, a wave could overwrite that stage while a slower wave
            // still ran phase A of group g - 1's last tile.)
            if (t % TPS == TPS - 1 && g + 1 < ngroups) {
                vm_wait(0);
                block_barrier();
#ifndef WV_H16_ABLATE_NO_FILL
                if (g + 2 < ngroups) fill_group(t_begin, g + 2, ntile);
#endif
            }
            // lanes l and l ^ 32 keep lists for the same query column (see the split pass)
            const bool mask_t = need_mask;
            const uint64_t mo0 = mask_t ? lane_ok(okw, jq0) : 0ull, mo1 = mask_t ? lane_ok(okw, jq1) : 0ull;
            const uint4* nimg = more ? lds + slot_t * St::U4 : img;
            // ---- A: H1(t) MFMAs, H0(t) minima, head of H0(t + 1) ----
            if (mask_t) mask_half(acc00, acc01, (uint32_t)mo0, (uint32_t)mo1);
            float m0, m1;
#ifdef WV_H16_ABLATE_NO_MIN
            m0 = acc00[0]; m1 = acc01[0];
            mfma_half(img, 1, acc10, acc11, [](int) {}, nimg, 0);
#else
            mfma_half(img, 1, acc10, acc11, min_steps(acc00, acc01, m0, m1), nimg, 0);
#endif
            // ---- B ----
            bool grew = false;   // a list of this wave changed: thresholds to refresh
            if constexpr (SEED) {
                l0d[0] = fminf(l0d[0], m0);
                l1d[0] = fminf(l1d[0], m1);
            } else {
                grew = extract_half(m0, m1, acc00, acc01, rb0);
            }
            // ---- E: H0(t + 1) MFMAs, H1(t) minima, head of H1(t + 1) ----
            if (mask_t) mask_half(acc10, acc11, (uint32_t)(mo0 >> 32), (uint32_t)(mo1 >> 32));
            if (more) {
#ifdef WV_H16_ABLATE_NO_MIN
                m0 = acc10[0]; m1 = acc11[0];
                mfma_half(nimg, 0, acc00, acc01, [](int) {}, nimg, 1);
#else
                mfma_half(nimg, 0, acc00, acc01, min_steps(acc10, acc11, m0, m1), nimg, 1);
#endif
                need_mask = tile_ok(phys(t_begin + t + 1), okw);
            } else {
                m0 = min16(acc10);
                m1 = min16(acc11);
            }
            // ---- F ----
            if constexpr (SEED) {
                l0d[0] = fminf(l0d[0], m0);
                l1d[0] = fminf(l1d[0], m1);
            } else {
                grew = extract_half(m0, m1, acc10, acc11, rb0 + 32) || grew;
                if (running && (t & 15) == 15) publish();
                else if (grew) refresh_pt();
                if constexpr (XS) {
                    if (t == xs_next) {
                        xslot_step(t != xs1, t != xs4);
                        // (equal points of a short segment collapse into one step)
                        xs_next = t < xs2 && xs2 > t ? xs2 : t < xs3 && xs3 > t ? xs3 : t < xs4 && xs4 > t ? xs4 : -1;
                    }
                }
            }
        }
        // every stage read and every DMA landed before the next segment's fills
        vm_wait(0);
        block_barrier();

        if constexpr (SEED) {
            if (jq0 < p.nq) p.out_d[((size_t)jq0 * p.n_slots + slot) * H_PROD + khalf] = l0d[0];
            if (jq1 < p.nq) p.out_d[((size_t)jq1 * p.n_slots + slot) * H_PROD + khalf] = l1d[0];
            continue;
        }
        const size_t per_q = (size_t)(p.out_slots ? p.out_slots : p.n_slots) * H_PROD * BF_KP;
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
// f16 key pass for D > 128 (C4's 768-d dot product): both operands through
// LDS.  Workgroup = 512 threads, one per CU; tile = 2 WR corpus rows x 256
// queries; wave w computes rows WR (w & 1) .. +WR x queries 64 (w >> 1) .. +64
// (WR / 32 x 2 accumulators of 32 x 32).  WR = 128 (the default): 256 x 256
// tiles, 2-step chunks -- per MFMA half the query-side bytes and LDS-DMA ops
// of WR = 64 (128 x 256 tiles, 4-step chunks; 48 KiB per chunk and CU for 16
// MFMAs a wave, which left the loop waiting on the DMA: ablation, DESIGN
// §3.2).  The corpus and query images are h16_index images with ns 16-k steps
// (ns a multiple of HW_KC, zero padded), so a chunk (KC steps) of a 32-row
// group is KC contiguous 1 KiB operand blocks: LDS-DMA'd as is, read back as
// one ds_read_b128 per operand.  Chunks go through a 3-stage ring (wait for
// chunk g, barrier, issue chunk g + 2, compute g); per tile a 2-slot ring
// holds s|x|^2 (the L2 C-in) and the tile's exclusion / allow words.  The
// epilogue -- mask, minima, candidate extraction into the same per-lane lists
// as the D <= 128 pass -- runs once per tile, i.e. once per ns / KC chunks.
template <int WR>
struct HWStage {
    static constexpr int RG = WR / 32;              // row groups per wave
    static constexpr int BN = 2 * WR;               // corpus rows per tile
    static constexpr int KC = WR == 64 ? HW_KC : HW_KC / 2;   // 16-k steps per chunk
    static constexpr int A_U4 = 2 * RG * KC * 64;   // the tile's row groups x KC steps x 64 lanes (16 KiB)
    static constexpr int B_U4 = 8 * KC * 64;        // 8 query groups
    static constexpr int U4 = A_U4 + B_U4;
    static constexpr int WORDS = BN / 64;           // exclusion (and allow) words per tile
    static constexpr int EX_U4 = BN / 4 + WORDS / 2 * 2;   // s|x|^2 of the tile, then excl and allow words
    static constexpr int OPS = 2 + KC;              // a wave's LDS-DMA blocks per chunk (extras aside)
};
constexpr int HW_STAGES = 3;

template <bool L2, int WR>
__global__ __launch_bounds__(512, 1) void wv_bf_h16w_kernel(H16Params p) {
    extern __shared__ uint4 lds[];
    using St = HWStage<WR>;
    constexpr int RG = St::RG, KC = St::KC, BN = St::BN;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int khalf = lane >> 5;
    const int l31 = lane & 31;
    const int rh = wave & 1, qq = wave >> 1;
    const int ns = p.ns, nch = ns / KC;
    const uint4* __restrict__ Qg = reinterpret_cast<const uint4*>(p.Q);
    const bool has_allow = p.allow != nullptr;
    if (p.n_dev) {   // the schedule of a device-counted row list
        const uint64_t S = (uint64_t)(p.n_slots - 1), nt = ((uint64_t)*p.n_dev + BN - 1) / BN;
        const uint64_t U = nt > S ? (nt + S - 1) / S : 1;
        p.ntiles = S * U;
        p.ntiles_real = nt;
        p.units_per_block = U;
    }
    int lb = (int)blockIdx.x;
    if ((p.locality & 1) && gridDim.x >= 8) {
        const int nwg = (int)gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = (int)blockIdx.x % 8;
        lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (int)blockIdx.x / 8;
    }
    if (p.block_order) lb = p.block_order[lb];
    const uint64_t u_first = (uint64_t)lb * p.units_per_block;
    uint64_t u_last = u_first + p.units_per_block;
    if (u_last > (uint64_t)p.n_qblocks * p.ntiles) u_last = (uint64_t)p.n_qblocks * p.ntiles;
    const uint32_t lds0 = lds_addr(lds);
    const uint32_t ex0 = lds0 + (uint32_t)(HW_STAGES * St::U4 * 16);
    const uint4* ex_lds = lds + HW_STAGES * St::U4;

    for (uint64_t u = u_first; u < u_last;) {
        const int qb = (int)(u / p.ntiles);
        const uint64_t t_begin = u % p.ntiles;
        uint64_t t_end = t_begin + (u_last - u);
        if (t_end > p.ntiles) t_end = p.ntiles;
        u += t_end - t_begin;
        const int slot = lb - bf_first_block(qb, p.ntiles, p.units_per_block);
        const int jq0 = qb * HW_BQ + qq * 64 + l31;
        const int jq1 = jq0 + 32;
        // (an aligned schedule's grid pads the corpus's tiles: no work past them)
        const uint64_t t_stop = t_end < p.ntiles_real ? t_end : p.ntiles_real;
        const int ntile = t_stop > t_begin ? (int)(t_stop - t_begin) : 0;
        const int nchunks = ntile * nch;

        // The chunks stream in order: chunk (t, c) into a stage of the 3-ring,
        // with c == 0 also the tile's extras into slot t & 1.  A chunk is 16
        // corpus blocks (block b = group * KC + step) and 8 KC query blocks;
        // this wave's share is fixed: blocks b = wave + 8 j (group wave / KC +
        // (8 / KC) j, step wave % KC) -- j < 2 on the corpus side, j < KC on
        // the query side -- so their sources are one base each plus a chunk
        // offset: no per-block index arithmetic on the scalar unit (the
        // round-2 loop spent 20 SALU per MFMA there, PMC).
        const int wg = wave / KC, wsk = wave % KC;
        const uint64_t gstride = (uint64_t)(8 / KC) * ns * 64;   // 8 / KC groups, in uint4
        const uint4* b_src0 = Qg + (((uint64_t)qb * (HW_BQ / 32) + wg) * ns + wsk) * 64;
        // Corpus side (round 5): the image is h16w_index (16-row groups of
        // 1 KiB panels, 64 B of a row per chunk), and the stage's A image is
        // the tile's 256 rows x 64 B, row after row.  This wave fills pieces
        // wave and wave + 8 (16 rows each); lane i loads 16 B of row 16 piece
        // + i / 4 -- row (tile, that row), or that entry of the compacted row
        // list: a compacted scan needs no gathered image.  The list entries of
        // tile t + 1 are LDS-DMA'd with tile t's first chunk into a 2-slot
        // ring and read at the tile change (nch - 1 >= 5 counted waits later;
        // a VGPR load the compiler does not track could be copied before it
        // lands).  The 16 B slot i % 4 of a row holds its chunk (i % 4) ^
        // ((row >> 2) & 3): the MFMA's ds_read_b128 lane groups then hit 16
        // distinct bank slots.
        static_assert(KC == 2, "a chunk is one 64 B panel per row");
        const uint64_t gsb = (uint64_t)ns * 512;   // bytes per 16-row group
        const char* Xb = reinterpret_cast<const char*>(p.X) + 16 * ((lane & 3) ^ ((lane >> 4) & 3));
        auto rid_of = [&](uint64_t tile, int j) -> uint64_t {
            return tile * BN + 16 * (wave + 8 * j) + (lane >> 2);
        };
        uint32_t rid_cur[2];
        const uint32_t rid_ring = ex0 + (uint32_t)(2 * St::EX_U4 * 16 + 8 * 256 + wave * 512);   // + slot 4 KiB + j 256
        const uint32_t* rid_lds = reinterpret_cast<const uint32_t*>(ex_lds + 2 * St::EX_U4) + 8 * 64 + wave * 128 + lane;
        // a row's first panel in the image (row group, row in group)
        uint64_t rbase[2];
        auto set_rbase = [&] {
#pragma unroll
            for (int j = 0; j < 2; ++j) rbase[j] = (uint64_t)(rid_cur[j] >> 4) * gsb + (uint64_t)((rid_cur[j] & 15) * 64);
        };
        // running sources of the next chunk to fill: +1 chunk (KC KiB steps)
        // per chunk; at a tile's end the corpus side moves on to the next
        // tile's row groups (2 RG ns steps per tile: + (2 RG - 1) ns past the
        // last chunk) and the query side starts over
        const uint4* b_cur = b_src0;
        int ft = 0, fc = 0;   // the next chunk to fill
        auto fill_next = [&](int stage) {
            // (ft, fc are wave-uniform; the divergence analysis loses that
            // through the lambda's captured state)
            ft = __builtin_amdgcn_readfirstlane(ft);
            fc = __builtin_amdgcn_readfirstlane(fc);
            stage = __builtin_amdgcn_readfirstlane(stage);
            const uint64_t tile = t_begin + ft;
            const uint32_t dst = lds0 + (uint32_t)(stage * St::U4 * 16) + (uint32_t)(wave * 1024);
            // (wave-uniform by construction; readfirstlane tells the compiler,
            // which must keep the LDS-DMA bases in SGPRs)
            const uint4* b = uniform_ptr(b_cur);
#ifndef WV_H16W_ABLATE_NO_A
            {
                const uint32_t kofs = (uint32_t)(fc * 1024);
                glds16(Xb + rbase[0] + kofs, dst);
                glds16(Xb + rbase[1] + kofs, dst + 8 * 1024);
            }
#endif
#ifndef WV_H16W_ABLATE_NO_B
#pragma unroll
            for (int j = 0; j < KC; ++j)
                glds16s(uniform_ptr(b + j * gstride), (uint32_t)(lane * 16), dst + (uint32_t)(St::A_U4 * 16 + 8 * j * 1024));
#endif
            if (fc == 0) {
                if (p.rowidx) {
                    const uint64_t tn = tile + 1 < p.ntiles_real ? tile + 1 : p.ntiles_real - 1;
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        glds4(p.rowidx + rid_of(tn, j), rid_ring + (uint32_t)(((ft + 1) & 1) * 4096 + 256 * j));
                }
                const uint32_t xd = ex0 + (uint32_t)((ft & 1) * St::EX_U4 * 16);
                if (wave == 0 && L2) {
#pragma unroll
                    for (int j = 0; j < BN / 64; ++j) glds4(p.xns + tile * BN + 64 * j + lane, xd + 256 * j);
                } else if (wave == 1) {
                    // lanes 0 .. 2 WORDS - 1: the tile's exclusion words (as
                    // u32 halves), then as many lanes for its allow words
                    const uint32_t* w = lane < 2 * St::WORDS
                                            ? reinterpret_cast<const uint32_t*>(p.excl + St::WORDS * tile) + lane
                                            : reinterpret_cast<const uint32_t*>(p.allow + St::WORDS * tile) + (lane - 2 * St::WORDS);
                    if (lane < 2 * St::WORDS || (lane < 4 * St::WORDS && has_allow)) glds4(w, xd + (BN / 4) * 16);
                }
            }
            b_cur = b + KC * 64;
            if (++fc == nch) {
                fc = 0;
                ++ft;
                b_cur = b_src0;
                // the next tile's rows: fetched a tile ago, covered by every
                // chunk's counted wait since (nch >= 3 chunks of >= 4 ops)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    rid_cur[j] = p.rowidx ? rid_lds[(ft & 1) * 1024 + 64 * j] : (uint32_t)rid_of(t_begin + ft, j);
                set_rbase();
            }
        };

        float l0d[BF_KP], l1d[BF_KP];
        uint32_t l0i[BF_KP], l1i[BF_KP];
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            l0d[i] = FLT_MAX; l1d[i] = FLT_MAX;
            l0i[i] = WV_NIL; l1i[i] = WV_NIL;
        }
        const float INF = __builtin_inff();
        // extraction thresholds beside the list tails: the running per-query
        // threshold every slot publishes (as wv_bf_h16_kernel's publish: k of
        // the lane pair's 2 BF_KP entries bound the k-th key, + 2 eps), and
        // -inf for the padding columns of a partial query block, which then
        // never extract and need no row mask
        float tau0 = jq0 < p.nq ? FLT_MAX : -INF, tau1 = jq1 < p.nq ? FLT_MAX : -INF;
        const bool running = p.kth > 0 && p.gtau != nullptr;
        float marg0 = 0.f, marg1 = 0.f;
        if (running) {
            if (jq0 < p.nq) marg0 = p.marg[jq0];
            if (jq1 < p.nq) marg1 = p.marg[jq1];
        }
        const int ia = (p.kth + 1) >> 1, ib = p.kth >> 1;
        // this wave's gtau return slot (64 words after the extras) and its
        // source word (clamped for the padding columns, whose tau stays -inf)
        const unsigned int* tau_lds = reinterpret_cast<const unsigned int*>(ex_lds + 2 * St::EX_U4) + 64 * wave;
        const uint32_t tau_dst = ex0 + (uint32_t)(2 * St::EX_U4 * 16 + 256 * wave);
        const int tau_src = min(jq0 - l31 + lane, p.nq - 1);
        if (running) reinterpret_cast<unsigned int*>(lds + HW_STAGES * St::U4 + 2 * St::EX_U4)[64 * wave + lane] = 0xFFFFFFFFu;
        auto publish = [&] {
            int va = ia - 1, vb = ib - 1;
            asm volatile("" : "+v"(va), "+v"(vb));   // (select chains over a VGPR index)
            float a0 = -FLT_MAX, a1 = -FLT_MAX, b0 = -FLT_MAX, b1 = -FLT_MAX;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) {
                a0 = va == i ? l0d[i] : a0;
                a1 = va == i ? l1d[i] : a1;
                b0 = vb == i ? l0d[i] : b0;
                b1 = vb == i ? l1d[i] : b1;
            }
            b0 = __shfl_xor(b0, 32, 64);
            b1 = __shfl_xor(b1, 32, 64);
            const float k0 = fmaxf(a0, b0), k1 = fmaxf(a1, b1);
            if (khalf == 0) {
                const float u4 = 4.f * 5.9604645e-08f;
                if (jq0 < p.nq && k0 < FLT_MAX) atomicMin(&p.gtau[jq0], h16_key_enc(k0 + marg0 + u4 * (fabsf(k0) + marg0)));
                if (jq1 < p.nq && k1 < FLT_MAX) atomicMin(&p.gtau[jq1], h16_key_enc(k1 + marg1 + u4 * (fabsf(k1) + marg1)));
            }
            // every slot's published thresholds come back by an LDS-DMA of the
            // wave's 64 gtau words (lane l: query jq0 - l31 + l), read at the
            // next publish: a plain load here would be waited for with
            // vmcnt(0), i.e. behind the chunk DMAs in flight (the compiler does
            // not see them) -- a drain of the operand stream per publish
            tau0 = fminf(tau0, h16_key_dec(tau_lds[l31]));
            tau1 = fminf(tau1, h16_key_dec(tau_lds[32 + l31]));
            glds4_dev(p.gtau + tau_src, tau_dst);
        };
        floatx16 acc[RG][2];
        auto min16 = [&](const floatx16& A) {
            float m0 = fminf(fminf(A[0], A[1]), A[2]), m1 = fminf(fminf(A[3], A[4]), A[5]);
            float m2 = fminf(fminf(A[6], A[7]), A[8]), m3 = fminf(fminf(A[9], A[10]), A[11]);
            m0 = fminf(fminf(m0, A[12]), A[13]);
            m1 = fminf(fminf(m1, A[14]), A[15]);
            return fminf(fminf(m0, m1), fminf(m2, m3));
        };
        // (the previous segment ended with every stage read and every DMA
        // landed: the first tile's rows are waited for alone)
        if (nchunks > 0) {
#pragma unroll
            for (int j = 0; j < 2; ++j) rid_cur[j] = p.rowidx ? p.rowidx[rid_of(t_begin, j)] : (uint32_t)rid_of(t_begin, j);
            set_rbase();
        }
        if (nchunks > 0) fill_next(0);
        if (nchunks > 1) fill_next(1);
        int t = 0, c = 0, stg = 0;   // the chunk computed: (tile, chunk), its stage
        for (int g = 0; g < nchunks; ++g) {
            // chunk g landed (g + 1 may stay in flight), for every wave: at
            // most OPS of this wave's ops still outstanding -- chunk g + 1's
            // blocks are its first OPS (its extras, issued after them, may
            // then have to land as well: a chunk's compute later, long done)
#if defined(WV_H16W_ABLATE_NO_A) && defined(WV_H16W_ABLATE_NO_B)
            vm_wait(0);
#elif defined(WV_H16W_ABLATE_NO_A)
            if (g + 1 < nchunks) vm_wait(KC);
            else vm_wait(0);
#elif defined(WV_H16W_ABLATE_NO_B)
            if (g + 1 < nchunks) vm_wait(2);
            else vm_wait(0);
#else
            if (g + 1 < nchunks) vm_wait(St::OPS);
            else vm_wait(0);
#endif
            block_barrier();
#ifdef WV_H16W_FILL_EARLY
            if (g + 2 < nchunks) fill_next(stg == 0 ? 2 : stg - 1);
#endif
            const uint4* st = lds + stg * St::U4;
            if (c == 0) {
                // C-in: s|x|^2 of the wave's rows (L2) or zero
                if (L2) {
                    const float* xn = reinterpret_cast<const float*>(ex_lds + (t & 1) * St::EX_U4) + WR * rh;
#pragma unroll
                    for (int i = 0; i < RG; ++i)
#pragma unroll
                        for (int g4 = 0; g4 < 4; ++g4) {
                            const float4 v = *reinterpret_cast<const float4*>(xn + 32 * i + 4 * khalf + 8 * g4);
                            acc[i][0][4 * g4] = v.x; acc[i][0][4 * g4 + 1] = v.y;
                            acc[i][0][4 * g4 + 2] = v.z; acc[i][0][4 * g4 + 3] = v.w;
                        }
#pragma unroll
                    for (int i = 0; i < RG; ++i) acc[i][1] = acc[i][0];
                } else {
#pragma unroll
                    for (int i = 0; i < RG; ++i)
#pragma unroll
                        for (int r = 0; r < 16; ++r) { acc[i][0][r] = 0.f; acc[i][1][r] = 0.f; }
                }
            }
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const half8 b0 = __builtin_bit_cast(half8, st[St::A_U4 + ((2 * qq) * KC + k) * 64 + lane]);
                const half8 b1 = __builtin_bit_cast(half8, st[St::A_U4 + ((2 * qq + 1) * KC + k) * 64 + lane]);
                // row 32 G + l31's chunk 2 k + khalf (swizzled slot)
                const int aslot = 4 * l31 + ((2 * k + khalf) ^ ((l31 >> 2) & 3));
#ifndef WV_H16W_JIT_READS
                // every operand of the k-step read before its first MFMA: the
                // scheduler otherwise reuses one A register set, each A read
                // then waits for the MFMAs of the last (lgkmcnt(0) per MFMA
                // pair: the LDS latency exposed RG times per k-step)
                half8 a[RG];
#pragma unroll
                for (int i = 0; i < RG; ++i) a[i] = __builtin_bit_cast(half8, st[128 * (RG * rh + i) + aslot]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < RG; ++i) {
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b0, acc[i][0], 0, 0, 0);
                    acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b1, acc[i][1], 0, 0, 0);
                }
#else
#pragma unroll
                for (int i = 0; i < RG; ++i) {
                    const half8 a = __builtin_bit_cast(half8, st[128 * (RG * rh + i) + aslot]);
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b0, acc[i][0], 0, 0, 0);
                    acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b1, acc[i][1], 0, 0, 0);
                }
#endif
#ifndef WV_H16W_FILL_EARLY
                // the next fill between this chunk's MFMAs, not beside the
                // partner wave's fill after the barrier (2.33 -> 2.23 ms per
                // C4-shaped pass, profiles/r03_h16w_fill_schedule_ablation.log)
                if (k == KC / 2 - 1 || KC == 1) {
                    __builtin_amdgcn_sched_barrier(0);
                    if (g + 2 < nchunks) fill_next(stg == 0 ? 2 : stg - 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
#endif
            }
            const int tc = t;   // (the chunk just computed)
            stg = stg == 2 ? 0 : stg + 1;
            if (++c != nch) continue;
            c = 0;
            ++t;
            // ---- tile epilogue ----
            const uint64_t tile = t_begin + tc;
            const uint32_t* w = reinterpret_cast<const uint32_t*>(ex_lds + (tc & 1) * St::EX_U4 + BN / 4);
            const uint64_t row0 = tile * BN + WR * rh;
            const float pt0 = fminf(__shfl_xor(l0d[BF_KP - 1], 32, 64), tau0);
            const float pt1 = fminf(__shfl_xor(l1d[BF_KP - 1], 32, 64), tau1);
#ifdef WV_H16W_ABLATE_NO_EPI
            {
                float z = pt0 + pt1;
#pragma unroll
                for (int i = 0; i < RG; ++i) z += acc[i][0][0] + acc[i][1][0];
                if (z == 1234.5f) l0d[0] = 0.f;
            }
            continue;
#endif
            // the wave's rows are the tile's words RG / 2 rh ..: 64 rows (two
            // row groups) per word
#pragma unroll
            for (int h = 0; h < RG / 2; ++h) {
                const int wi = RG / 2 * rh + h;
                uint64_t okw = ~((uint64_t)w[2 * wi] | ((uint64_t)w[2 * wi + 1] << 32));
                if (has_allow) okw &= (uint64_t)w[2 * St::WORDS + 2 * wi] | ((uint64_t)w[2 * St::WORDS + 2 * wi + 1] << 32);
                const uint64_t r0 = row0 + 64 * h;
                if (r0 + 64 > p.N) okw &= p.N > r0 ? ((1ull << (p.N - r0)) - 1) : 0ull;
                floatx16& A0 = acc[2 * h][0];
                floatx16& A1 = acc[2 * h][1];
                floatx16& B0 = acc[2 * h + 1][0];
                floatx16& B1 = acc[2 * h + 1][1];
                if (okw != ~0ull) {
                    const uint64_t o = okw >> (4 * khalf);
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int bit = (r & 3) + 8 * (r >> 2);
                        A0[r] = (o >> bit) & 1u ? A0[r] : INF;
                        A1[r] = (o >> bit) & 1u ? A1[r] : INF;
                        B0[r] = (o >> (32 + bit)) & 1u ? B0[r] : INF;
                        B1[r] = (o >> (32 + bit)) & 1u ? B1[r] : INF;
                    }
                }
                const uint32_t rb = (uint32_t)r0 + 4 * khalf;
                WV_DBG_COUNT(0)
#ifdef WV_H16W_ABLATE_NO_EXTRACT
                if (fminf(fminf(min16(A0), min16(B0)), fminf(min16(A1), min16(B1))) == 1234.5f) l0d[0] = pt0;
#else
                // insertion of a column's minimum (wv_topk.h min_extract)
                auto xt = [&](floatx16& A, float (&ld)[BF_KP], uint32_t (&li)[BF_KP], float pt, uint32_t rr) {
                    const float th = fminf(ld[BF_KP - 1], pt);
                    const float m = min16(A);
                    const bool x = m <= th;
                    if (__any(x)) {
                        WV_DBG_COUNT(3)
                        // (the minimum by position, the per-key scan only for a
                        // second hit: 2.364 -> 2.249 ms per C4-shaped pass; A is
                        // reloaded from the C-in at the next tile)
                        min_extract(m, x, A, pt, ld, li, rr);
                    }
                };
                xt(A0, l0d, l0i, pt0, rb);
                xt(B0, l0d, l0i, pt0, rb + 32);
                xt(A1, l1d, l1i, pt1, rb);
                xt(B1, l1d, l1i, pt1, rb + 32);
#endif
            }
            // every tile while the lists fill, then every 4th
            if (running && (tc < 8 || (tc & 3) == 3)) publish();
        }
        vm_wait(0);
        block_barrier();   // every stage read before the next segment's fills
        const int prod = rh * 2 + khalf;
        const size_t per_q = (size_t)p.n_slots * HW_PROD * BF_KP;
        if (jq0 < p.nq) {
            const size_t base = (size_t)jq0 * per_q + ((size_t)slot * HW_PROD + prod) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l0d[i]; p.out_id[base + i] = l0i[i]; }
        }
        if (jq1 < p.nq) {
            const size_t base = (size_t)jq1 * per_q + ((size_t)slot * HW_PROD + prod) * BF_KP;
#pragma unroll
            for (int i = 0; i < BF_KP; ++i) { p.out_d[base + i] = l1d[i]; p.out_id[base + i] = l1i[i]; }
        }
    }
}

// ---------------------------------------------------------------------------
// Seed thresholds from the pre-pass minima: the n_lists minima of a query are
// approximate keys of distinct rows, so the k-th smallest of them, m_k, has k
// real points with key <= m_k, i.e. true distance <= m_k + offset + eps: the
// true k-th distance is no larger, and a point of the true top k has key <=
// its distance - offset + eps <= m_k + 2 eps.  One wave per query.
__global__ __launch_bounds__(64) void wv_h16_seed_kernel(H16SeedParams p) {
    const int q = blockIdx.x;
    const int lane = threadIdx.x;
    if (q >= p.nq) return;
    const int prod = p.prod ? p.prod : H_PROD;
    const int n = bf_slots_of((uint64_t)(q / p.bq), p.ntiles, p.units_per_block) * prod;
    const float* m = p.minima + (size_t)q * p.n_slots * prod;
    const float inv_s = 1.0f / (p.sx * p.qscale[0]);
    float mk = __builtin_inff();
    if (p.ids) {
        // list mode (n <= 256, k <= 64: the host's condition): every entry
        // sorted by (key, id); the k-th a real row's, or none
        const size_t off = (size_t)q * p.n_slots * prod;
        uint64_t kk[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 64 * j + lane;
            const uint32_t id = e < n ? p.ids[off + e] : WV_NIL;
            kk[j] = fin_key(id != WV_NIL ? p.minima[off + e] : FLT_MAX, id);
        }
        bitonic256_wave(kk, lane);
        float d;
        uint32_t id;
        fin_unkey(kk[0], d, id);
        const float dk = __shfl(d, p.k - 1, 64);
        const uint32_t ik = (uint32_t)__shfl((int)id, p.k - 1, 64);
        if (ik != WV_NIL) mk = dk;
        // the 2 BF_KP smallest: one more slot of the main pass's lists (even
        // ranks, odd ranks), after the query block's own slots
        const int os = bf_slots_of((uint64_t)(q / p.bq), p.out_ntiles, p.out_upb);
        const size_t ob = ((size_t)q * p.out_slots + os) * H_PROD * BF_KP;
        if (lane < H_PROD * BF_KP) {
            const size_t o = ob + (size_t)(lane & 1) * BF_KP + (lane >> 1);
            p.out_d[o] = d;
            p.out_id[o] = id;
        }
    } else if (n <= 256) {
        // the k-th smallest by a wave-wide bitonic sort of the (<= 256)
        // minima, element i = 64 j + lane in register j
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = 64 * j + lane < n ? m[64 * j + lane] : __builtin_inff();
#pragma unroll
        for (int kk = 2; kk <= 256; kk <<= 1) {
#pragma unroll
            for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                if (jj >= 64) {
                    const int mm = jj >> 6;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int pj = j ^ mm;
                        if (pj <= j) continue;
                        const bool up = ((64 * j + lane) & kk) == 0;
                        const float lo = fminf(v[j], v[pj]), hi = fmaxf(v[j], v[pj]);
                        v[j] = up ? lo : hi;
                        v[pj] = up ? hi : lo;
                    }
                } else {
                    const bool lower = (lane & jj) == 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float o = __shfl_xor(v[j], jj, 64);
                        const bool up = ((64 * j + lane) & kk) == 0;
                        v[j] = (lower == up) ? fminf(v[j], o) : fmaxf(v[j], o);
                    }
                }
            }
        }
        // element k - 1 (k <= 256): register (k - 1) / 64 of lane (k - 1) % 64
        const int e = p.k - 1;
        float sel = v[0];
#pragma unroll
        for (int j = 1; j < 4; ++j) sel = (e >> 6) == j ? v[j] : sel;
        mk = __shfl(sel, e & 63, 64);
    } else {
        // k rounds of a wave-wide minimum over the lanes' shares
        float taken = -__builtin_inff();
        int n_taken = 0;
        for (int r = 0; r < p.k; ++r) {
            float best = __builtin_inff();
            int where = 0x7FFFFFFF;
            for (int i = lane; i < n; i += 64) {
                const float v = m[i];
                // strictly after the last taken (value, index) in (value, index) order
                const bool after = v > taken || (v == taken && i > n_taken);
                if (after && v < __builtin_inff() && (v < best || (v == best && i < where))) { best = v; where = i; }
            }
            for (int o = 32; o >= 1; o >>= 1) {
                const float ob = __shfl_xor(best, o, 64);
                const int ow = __shfl_xor(where, o, 64);
                if (ob < best || (ob == best && ow < where)) { best = ob; where = ow; }
            }
            if (!(best < __builtin_inff())) { mk = __builtin_inff(); break; }
            taken = best;
            n_taken = where;
            mk = best;
        }
    }
    if (lane == 0) {
        float tau = __builtin_inff();
        if (mk < __builtin_inff()) {
            const float key = mk * inv_s;
            const float eps = h16_eps(p.metric, p.D, p.qnorm[q], p.xnorm_max, p.ex_max, p.qres[q]);
            tau = key + 2.f * eps;
            tau += 4.f * 5.9604645e-08f * (fabsf(key) + 2.f * eps) + 1e-3f * eps;   // this sum's rounding
        }
        // (list mode: the list pass dropped keys above the minima pass's
        // threshold, already in p.tau -- the thresholds only decrease)
        if (p.ids) tau = fminf(tau, p.tau[q]);
        p.tau[q] = tau;
        if (p.gtau) p.gtau[q] = h16_key_enc(tau * (p.sx * p.qscale[0]));
    }
}

// the running threshold's per-query margin: 2 eps in scaled key units
__global__ void wv_h16_margin_kernel(int metric, int D, const float* qnorm, const float* qres, float xnorm_max,
                                     float ex_max, float sx, const float* qscale, int nq, float* marg) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq) marg[q] = 2.f * (sx * qscale[0]) * h16_eps(metric, D, qnorm[q], xnorm_max, ex_max, qres[q]) * 1.001f;
}

// the running threshold after the key pass -> true units, for the finalize
// (every key the pass dropped was above it)
__global__ void wv_h16_gtau_kernel(const unsigned int* gtau, int nq, float sx, const float* qscale, float* tau) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq) tau[q] = h16_key_dec(gtau[q]) * (1.0f / (sx * qscale[0]));
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

__global__ void wv_h16_rows_kernel(const float* in, int ld_in, const uint64_t* ids, const uint32_t* gather,
                                   uint64_t n, int D, int ns, float sign, float scale,
                                   const unsigned int* scale_from_max, uint16_t* out, uint64_t out_row0,
                                   unsigned int* res_max_bits, float* res_out, int wide_layout) {
    const uint64_t r = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    if (scale_from_max) scale = pow2_scale_for(__uint_as_float(*scale_from_max) * fabsf(sign));
    // ids: row ids[r] to image row ids[r] (row writes); gather: row gather[r]
    // to image row r (a compacted allow list's rows, in list order)
    const uint64_t src = gather ? gather[r] : ids ? ids[r] : r;
    const uint64_t row = gather ? r : src;
    in += (src - row) * (uint64_t)ld_in;
    const int kmax = ns * 16;
    float acc = 0.f;
    for (int k = lane; k < kmax; k += 64) {
        const float x = k < D ? sign * in[row * (uint64_t)ld_in + k] : 0.f;
        const _Float16 h = (_Float16)(scale * x);
        const float back = (float)h / scale;
        const float e = x - back;           // exact (Sterbenz) unless h overflowed
        acc = __builtin_fmaf(e, e, acc);
        out[wide_layout ? h16w_index(out_row0 + row, k, ns) : h16_index(out_row0 + row, k, ns)] =
            __builtin_bit_cast(uint16_t, h);
    }
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if (lane == 0) {
        // inflate for the fp32 sum (D terms) and the sqrt
        const float res = acc == 0.f ? 0.f : sqrtf(acc * (1.0f + 2e-5f)) * (1.0f + 1e-6f) + 1e-30f;
        if (res_max_bits) atomicMax(res_max_bits, __float_as_uint(res));
        if (res_out) res_out[out_row0 + row] = res;
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
// s_q from the batch max: the qnorm pass's per-block partials (nparts, or a
// single precomputed max when part == nullptr), reduced here; the max is also
// left in max_bits for the query image kernel
__global__ __launch_bounds__(256) void wv_h16_qscale_kernel(const float* part, int nparts, unsigned int* max_bits,
                                                            float bsign, float* qscale) {
    __shared__ float wm[4];
    float m = 0.f;
    if (part)
        for (int i = threadIdx.x; i < nparts; i += blockDim.x) m = fmaxf(m, part[i]);
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float mx = part ? fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])) : __uint_as_float(*max_bits);
        if (part) *max_bits = __float_as_uint(mx);
        qscale[0] = pow2_scale_for(mx * fabsf(bsign));
    }
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
                              unsigned int* res_max_bits, float* res_out, int wide_layout, hipStream_t s) {
    if (n == 0) return hipSuccess;
    // (wide_layout: the h16w_index image of the wide-D kernel; 0: h16_index)
    if (ns < 1 || ns > wv::HW_NS_MAX || D > ns * 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wv::wv_h16_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, in, ld_in, ids,
                       (const uint32_t*)nullptr, n, D, ns, sign, scale, scale_from_max, static_cast<uint16_t*>(out),
                       out_row0, res_max_bits, res_out, wide_layout);
    return hipGetLastError();
}

// The image of rows gather[0..n) (ascending row ids of a compacted allow
// list) as image rows 0..n_pad (h16_index layout, rows past n zero): one
// thread per 16-byte image word -- lane (h, r) of a (32-row group, 16-k step)
// block, 8 halves of one row -- so the stores are whole contiguous 1 KiB
// blocks (wv_h16_rows_kernel scatters 2-byte stores: 1.4 ms for 625k x 768
// rows, measured) and the reads are 32-byte row pieces.
__global__ void wv_h16_img_gather_kernel(const float* __restrict__ in, int ld_in, const uint32_t* __restrict__ gather,
                                         uint64_t n, uint64_t n_pad, int D, int ns, float scale, uint4* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = n_pad / 32 * (uint64_t)ns * 64;
    if (i >= total) return;
    const uint64_t block = i >> 6;
    const int lane = (int)(i & 63);
    const uint64_t grp = block / (uint64_t)ns;
    const int step = (int)(block - grp * ns);
    const uint64_t r = grp * 32 + (lane & 31);
    const int k0 = step * 16 + (lane >> 5) * 8;
    uint32_t h[4] = {0u, 0u, 0u, 0u};
    if (r < n) {
        const float* src = in + (uint64_t)gather[r] * ld_in;
        float x[8];
        if (k0 + 8 <= D) {
            const float4 a = *reinterpret_cast<const float4*>(src + k0);
            const float4 b = *reinterpret_cast<const float4*>(src + k0 + 4);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = k0 + j < D ? src[k0 + j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const _Float16 lo = (_Float16)(scale * x[2 * j]), hi = (_Float16)(scale * x[2 * j + 1]);
            h[j] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
        }
    }
    out[i] = make_uint4(h[0], h[1], h[2], h[3]);
}

hipError_t wv_launch_h16_rows_gather(const float* in, int ld_in, const uint32_t* gather, uint64_t n, uint64_t n_pad,
                                     int D, int ns, float scale, void* out, hipStream_t s) {
    if (n_pad == 0) return hipSuccess;
    // (ld_in a multiple of 4 floats: the corpus rows are 16-byte aligned)
    if (ns < 1 || ns > wv::HW_NS_MAX || D > ns * 16 || !gather || n_pad % 32 || n > n_pad || ld_in % 4)
        return hipErrorInvalidValue;
    const uint64_t total = n_pad / 32 * (uint64_t)ns * 64;
    hipLaunchKernelGGL(wv_h16_img_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in, ld_in,
                       gather, n, n_pad, D, ns, scale, static_cast<uint4*>(out));
    return hipGetLastError();
}

__global__ void wv_gather_f32_kernel(const float* src, const uint32_t* idx, uint64_t n, const uint32_t* n_dev,
                                     float* dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n_dev) n = *n_dev;   // (n: the launch's bound)
    if (i < n) dst[i] = src[idx[i]];
}

// candidate lists of a key pass over compacted rows: list positions -> row ids
// (the map is increasing, so every (key, id) order is unchanged).  Only the
// lists a query's block really produced (bf_slots_of slots, as the finalize
// reads them): the other entries of the [nq][n_slots][per_slot] array hold
// stale words.  A position >= n_rows cannot come out of the pass; it would
// become WV_NIL here rather than an out-of-range read.
__global__ void wv_remap_ids_kernel(uint32_t* ids, int nq, int n_slots, int per_slot, int bq, uint64_t ntiles,
                                    uint64_t units_per_block, const uint32_t* rowidx, uint64_t n_rows,
                                    const uint32_t* n_dev) {
    const int q = blockIdx.x;
    if (q >= nq) return;
    if (n_dev) n_rows = *n_dev;
    const int n_valid = wv::bf_slots_of((uint64_t)(q / bq), ntiles, units_per_block) * per_slot;
    uint32_t* e = ids + (size_t)q * n_slots * per_slot;
    for (int i = threadIdx.x; i < n_valid; i += blockDim.x) {
        const uint32_t v = e[i];
        if (v != WV_NIL) e[i] = v < n_rows ? rowidx[v] : WV_NIL;
    }
}

// exclusion bits of a compacted scan: rows >= n (the last tile's padding)
__global__ void wv_excl_tail_kernel(uint64_t* excl, uint64_t n, const uint32_t* n_dev, uint64_t words) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    if (n_dev) n = *n_dev;
    const uint64_t lo = w * 64;
    excl[w] = lo >= n ? ~0ull : (n - lo >= 64 ? 0ull : ~0ull << (n - lo));
}

// n_dev (nullable): the list's length on the device, n then its bound
hipError_t wv_launch_h16_compact_aux(const float* xnorm, const uint32_t* rowidx, uint64_t n, const uint32_t* n_dev,
                                     float* cxnorm, uint64_t* excl, uint64_t excl_words, hipStream_t s) {
    if (n) hipLaunchKernelGGL(wv_gather_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, xnorm, rowidx, n,
                              n_dev, cxnorm);
    hipLaunchKernelGGL(wv_excl_tail_kernel, dim3((unsigned)((excl_words + 255) / 256)), dim3(256), 0, s, excl, n,
                       n_dev, excl_words);
    return hipGetLastError();
}

hipError_t wv_launch_remap_ids(uint32_t* ids, int nq, int n_slots, int per_slot, int bq, uint64_t ntiles,
                               uint64_t units_per_block, const uint32_t* rowidx, uint64_t n_rows, const uint32_t* n_dev,
                               hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(wv_remap_ids_kernel, dim3((unsigned)nq), dim3(64), 0, s, ids, nq, n_slots, per_slot, bq, ntiles,
                       units_per_block, rowidx, n_rows, n_dev);
    return hipGetLastError();
}

hipError_t wv_launch_absmax(const float* in, int ld, uint64_t n, int D, unsigned int* max_bits, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n * (uint64_t)D + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(wv::wv_absmax_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, ld, n, D, max_bits);
    return hipGetLastError();
}

hipError_t wv_launch_h16_qscale(const float* part, int nparts, unsigned int* max_bits, float bsign, float* qscale,
                                hipStream_t s) {
    hipLaunchKernelGGL(wv::wv_h16_qscale_kernel, dim3(1), dim3(256), 0, s, part, nparts, max_bits, bsign, qscale);
    return hipGetLastError();
}

hipError_t wv_launch_h16_xns(const float* xnorm, uint64_t n, float sx, const float* qscale, float* xns, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_h16_xns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, xnorm, n, sx, qscale,
                       xns);
    return hipGetLastError();
}

hipError_t wv_launch_bf_h16(const wv::H16Params* p, int ns, int seed, hipStream_t s) {
    const uint64_t total = (uint64_t)p->n_qblocks * p->ntiles;
    const unsigned nb = (unsigned)((total + p->units_per_block - 1) / p->units_per_block);
    if (nb == 0) return hipSuccess;
    if (ns < 1 || ns > wv::H_NS_MAX || !p->X || !p->Q || !p->excl || !p->qscale || p->tile_stride < 1 ||
        (p->out_slots && p->out_slots < p->n_slots) || (seed && (p->out_slots || p->tile_base)))
        return hipErrorInvalidValue;
    const bool l2 = p->metric == WV_METRIC_L2;
    if (l2 && !p->xns) return hipErrorInvalidValue;
    const size_t lds = (size_t)wv::H_STAGES * wv::H_TPS8 * (2 * ns * 64 + 17) * 16;
#define WV_H16_GO(NS, L, S)                                                                                    \
    if (!S && p->xslot)                                                                                        \
        hipLaunchKernelGGL((wv::wv_bf_h16_kernel<NS, L, false, true>), dim3(nb), dim3(512), lds, s, *p);       \
    else hipLaunchKernelGGL((wv::wv_bf_h16_kernel<NS, L, S>), dim3(nb), dim3(512), lds, s, *p);
#define WV_H16_LAUNCH(NS)                     \
    if (seed) {                               \
        if (l2) { WV_H16_GO(NS, true, true) } \
        else { WV_H16_GO(NS, false, true) }   \
    } else {                                  \
        if (l2) { WV_H16_GO(NS, true, false) } \
        else { WV_H16_GO(NS, false, false) }  \
    }
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
#undef WV_H16_GO
    return hipGetLastError();
}

hipError_t wv_launch_h16_margin(int metric, int D, const float* qnorm, const float* qres, float xnorm_max,
                                float ex_max, float sx, const float* qscale, int nq, float* marg, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_h16_margin_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, metric, D, qnorm, qres,
                       xnorm_max, ex_max, sx, qscale, nq, marg);
    return hipGetLastError();
}

hipError_t wv_launch_h16_gtau(const unsigned int* gtau, int nq, float sx, const float* qscale, float* tau,
                              hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_h16_gtau_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, gtau, nq, sx, qscale, tau);
    return hipGetLastError();
}

hipError_t wv_launch_bf_h16w(const wv::H16Params* p, hipStream_t s) {
    const uint64_t total = (uint64_t)p->n_qblocks * p->ntiles;
    const unsigned nb = (unsigned)((total + p->units_per_block - 1) / p->units_per_block);
    if (nb == 0) return hipSuccess;
    if (p->ns < 2 * wv::HW_KC || p->ns > wv::HW_NS_MAX || p->ns % wv::HW_KC || !p->X || !p->Q || !p->excl ||
        p->tile_stride != 1 || p->tile_base != 0 || p->out_slots != 0)
        return hipErrorInvalidValue;
    const bool l2 = p->metric == WV_METRIC_L2;
    if (l2 && !p->xns) return hipErrorInvalidValue;
    if (p->wide_rows != 128) return hipErrorInvalidValue;
    using St = wv::HWStage<128>;
    // + the gtau return slots and the row-list ring (2 slots x 8 waves x 2 x 64 ids)
    const size_t lds = ((size_t)wv::HW_STAGES * St::U4 + 2 * St::EX_U4) * 16 + 8 * 256 + 2 * 8 * 2 * 256;
    if (l2) hipLaunchKernelGGL((wv::wv_bf_h16w_kernel<true, 128>), dim3(nb), dim3(512), lds, s, *p);
    else hipLaunchKernelGGL((wv::wv_bf_h16w_kernel<false, 128>), dim3(nb), dim3(512), lds, s, *p);
    return hipGetLastError();
}

hipError_t wv_launch_h16_seed(const wv::H16SeedParams* p, hipStream_t s) {
    if (p->nq == 0) return hipSuccess;
    if (p->k < 1 || p->k > wv::BF_WIDE_KMAX) return hipErrorInvalidValue;
    if (p->ids && (p->k > 64 || p->prod != wv::H_PROD * wv::BF_KP || (size_t)p->n_slots * p->prod > 256 ||
                   !p->out_d || !p->out_id || p->out_slots < 1))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(wv::wv_h16_seed_kernel, dim3(p->nq), dim3(64), 0, s, *p);
    return hipGetLastError();
}

}  // extern "C"
