// wv_h16s.hip -- the 16x16x32 f16 key pass with one wave per SIMD
// (wv_bf_h16s_kernel), the exact brute force's default for D <= 128 with an
// even number of 16-k steps and k <= FIN_KF (flatSearch,
// adapters/repos/db/vector/hnsw/flat_search.go:19-74).  Its own translation
// unit: built with the MFMA's VGPR form (-mllvm -amdgpu-mfma-vgpr-form, the
// Makefile), so the accumulators the epilogue VALU reads are written straight
// to VGPRs, while the query operands are pinned to AGPRs.
#include "wv_h16_dev.h"

namespace wv {

// ---------------------------------------------------------------------------
// The 16x16x32 key pass with ONE wave per SIMD (wv_bf_h16s_kernel, the
// default for D <= 128 since round 3).  A 256-thread workgroup per CU, 4
// waves; each wave holds 8 query groups of 16 (128 queries: 128 VGPRs of B
// operands at D = 128) and computes 32 rows x 128 queries per half tile = 64
// independent MFMAs (2 row groups x 8 query groups x 4 k-steps), twice the
// queries per A fragment of wv_bf_h16q_kernel.  So per half tile a wave reads
// 8 + 2 LDS operands for 64 MFMAs, the minima of the other half (4 VALU per
// query group, 32 per half) fit the MFMA issue gaps of a wave that has its
// SIMD to itself -- no partner wave kept in phase by the stage barrier
// (MI355X_MICROARCH 'Two waves per SIMD') -- and the two accumulator sets
// (halves) alternate: the MFMAs of one half issue while the minima and the
// (rare) extraction of the other are done.  Tiles (64 rows) stream global ->
// LDS by LDS-DMA as in the other f16 kernels (3 stages of HS_TPS tiles, one
// barrier per stage); lists, seed minima and the certificate are those of
// wv_bf_h16q_kernel (one 16-entry list per query column and slot).
//
// XS: the cross-slot threshold over column lists -- each slot stores its
// column list's entries 0 and 1 (two distinct rows of its own row range) in
// gslot[q][2 slot + e] at 1/8, 1/4, 1/2 of its segment and reads the others'
// at 1/4, 1/2, 3/4: the k-th smallest of those <= 2 n_slots values + 2 eps
// bounds the k-th key; every bound is also atomicMin'ed into gtau, so the
// finalize's tau_in covers every key dropped above it.
template <int NS32, bool L2, bool SEED, bool XS>
__global__ __launch_bounds__(256, 1) void wv_bf_h16s_kernel(H16Params p) {
    constexpr int WAVES = 4, QG = HS_QG, BQ = HS_BQ, TPS = HS_TPS;
    extern __shared__ uint4 lds[];
    using St = H16Stage<2 * NS32>;   // 4 row groups x NS32 32-k steps, as the h16q image
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lq = lane >> 4;        // lane quarter: rows 4 lq .. 4 lq + 3 of each 16-row group
    const int l15 = lane & 15;
    const uint4* __restrict__ X = reinterpret_cast<const uint4*>(p.X);
    const uint4* __restrict__ Qg = reinterpret_cast<const uint4*>(p.Q);
    const bool has_allow = p.allow != nullptr;
    const float s = p.sx * p.qscale[0];
    int lb = (int)blockIdx.x;
    if ((p.locality & 1) && gridDim.x >= 8) {   // bijective XCD remap (blocks b, b + 8, ... share an XCD)
        const int nwg = (int)gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = (int)blockIdx.x % 8;
        lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (int)blockIdx.x / 8;
    }
    const uint64_t u_first = (uint64_t)lb * p.units_per_block;
    uint64_t u_last = u_first + p.units_per_block;
    if (u_last > (uint64_t)p.n_qblocks * p.ntiles) u_last = (uint64_t)p.n_qblocks * p.ntiles;
    const uint32_t lds0 = lds_addr(lds);
    // this wave's LDS-DMA ops per tile (4 of the 16 image pieces at D = 128,
    // + the s|x|^2 piece on wave 0)
    const int n_ops = (wave < St::IMG_U4 / 64 ? (St::IMG_U4 / 64 - 1 - wave) / WAVES + 1 : 0) +
                      ((wave == 0 && L2) ? 1 : 0);
    auto fill = [&](uint64_t t, int st) {
        const uint64_t tile = t * (uint64_t)p.tile_stride;
        const uint32_t dst = lds0 + (uint32_t)(st * St::U4 * 16);
        const uint4* src = X + tile * St::IMG_U4;
#pragma unroll
        for (int i = wave; i < St::IMG_U4 / 64; i += WAVES) glds16s(src, (uint32_t)(i * 1024 + lane * 16), dst + i * 1024);
        if (wave == 0 && L2) glds4(p.xns + tile * H_BN + lane, dst + St::IMG_U4 * 16);
    };
    auto fill_group = [&](uint64_t t_begin, int g, int ntile) {
        const int st = g % H_STAGES;
        int n = 0;
#pragma unroll
        for (int j = 0; j < TPS; ++j) {
            const int t = g * TPS + j;
            if (t < ntile) { fill(t_begin + t, st * TPS + j); ++n; }
        }
        return n * n_ops;
    };
    auto tile_lds = [&](int t) { return lds + ((t / TPS) % H_STAGES * TPS + t % TPS) * St::U4; };

    for (uint64_t u = u_first; u < u_last;) {
        const int qb = (int)(u / p.ntiles);
        const uint64_t t_begin = u % p.ntiles;
        uint64_t t_end = t_begin + (u_last - u);
        if (t_end > p.ntiles) t_end = p.ntiles;
        u += t_end - t_begin;
        const int slot = lb - bf_first_block(qb, p.ntiles, p.units_per_block);
        const int ntile = (int)(t_end - t_begin);
        const int jq0 = qb * BQ + wave * 16 * QG + l15;   // query of column l15, group g: jq0 + 16 g
        auto jqof = [&](int g) { return jq0 + 16 * g; };

        // the wave's 128 queries (8 groups of 16) as B operands, for the segment
        half8 bq[QG][NS32];
#pragma unroll
        for (int g = 0; g < QG; ++g) {
            const uint64_t G = (uint64_t)qb * (BQ / 16) + QG * wave + g;
#pragma unroll
            for (int kk = 0; kk < NS32; ++kk) bq[g][kk] = __builtin_bit_cast(half8, Qg[(G * NS32 + kk) * 64 + lane]);
        }
        // (a column past nq -- the partial last query block -- never
        // extracts: threshold -inf, so its tiles need no mask)
        float tau[QG];
#pragma unroll
        for (int g = 0; g < QG; ++g) {
            tau[g] = -__builtin_inff();
            if (jqof(g) < p.nq) {
                tau[g] = FLT_MAX;
                if (!SEED && p.gtau) tau[g] = fminf(FLT_MAX, h16_key_dec(p.gtau[jqof(g)]));
                else if (p.tau) tau[g] = fminf(FLT_MAX, p.tau[jqof(g)] * s);
            }
        }
        // consume the ordinary loads before any LDS-DMA is in flight
        // (and into AGPRs: they are only ever MFMA operands, while every
        // value the VALU touches -- keys, lists, thresholds -- needs the 256
        // VGPRs)
#pragma unroll
        for (int g = 0; g < QG; ++g)
#pragma unroll
            for (int kk = 0; kk < NS32; ++kk) asm volatile("" : "+a"(bq[g][kk]));
#pragma unroll
        for (int g = 0; g < QG; ++g) asm volatile("" ::"v"(tau[g]));
        float ld[QG][HQ_KP];
        uint32_t li[QG][HQ_KP];
#pragma unroll
        for (int g = 0; g < QG; ++g)
#pragma unroll
            for (int i = 0; i < HQ_KP; ++i) { ld[g][i] = FLT_MAX; li[g][i] = WV_NIL; }

        const float INF = __builtin_inff();
        // two accumulator sets of one row group (16 rows x 128 queries) each:
        // the MFMAs of row group j issue into one while the minima and the
        // extraction of row group j - 1 read the other (only 2 x 32 VGPRs of
        // keys live: everything the VALU touches must fit the 256 VGPRs)
        floatx4 accX[QG], accY[QG];
        // A row group's operands: its C-in and NS32 A fragments, read from
        // LDS one step AHEAD (during the previous row group's MFMAs), so no
        // MFMA block waits on an LDS round trip -- with one wave per SIMD
        // there is no partner wave to cover it.  Two sets (P, Q) alternate
        // by step; the fragments live in AGPRs (MFMA operands only).
        struct Frag {
            half8 a[NS32];
            floatx4 xc;
        };
        auto load_frag = [&](const uint4* img, int rg, Frag& f) {
            if (L2) {
                const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(img + St::IMG_U4) +
                                                                  16 * rg + 4 * lq);
                f.xc = floatx4{v.x, v.y, v.z, v.w};
            } else {
                f.xc = floatx4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int kk = 0; kk < NS32; ++kk) f.a[kk] = __builtin_bit_cast(half8, img[(rg * NS32 + kk) * 64 + lane]);
        };
        auto pin_frag = [&](Frag& f) {
#pragma unroll
            for (int kk = 0; kk < NS32; ++kk) asm volatile("" : "+a"(f.a[kk]));
        };
        // one row group's MFMAs (NS32 k-steps x QG query groups) from f;
        // `between` (the other set's minima, the next step's fragment reads)
        // interleaved: MFMA, LDS read, VALU, ...
        auto mfma_rg = [&](const Frag& f, floatx4 (&acc)[QG], auto&& between) {
            __builtin_amdgcn_sched_barrier(0);
            between();
#pragma unroll
            for (int kk = 0; kk < NS32; ++kk)
#pragma unroll
                for (int g = 0; g < QG; ++g)
                    acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.a[kk], bq[g][kk], kk == 0 ? f.xc : acc[g], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < QG * NS32; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (i < NS32 + 1) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        auto tile_ok = [&](uint64_t t, uint64_t& okw) -> bool {
            okw = tile_okw(p, t * (uint64_t)p.tile_stride, has_allow);
            return okw != ~0ull;
        };
        // ineligible keys of row group rg to +inf (row 16 rg + 4 lq + e of the tile)
        auto mask_rg = [&](floatx4 (&acc)[QG], int rg, uint64_t okw) {
            uint32_t ow[QG];
#pragma unroll
            for (int g = 0; g < QG; ++g) ow[g] = (uint32_t)((jqof(g) < p.nq ? okw : 0ull) >> (16 * rg + 4 * lq));
            bool all = true;
#pragma unroll
            for (int g = 0; g < QG; ++g) all = all && (ow[g] & 0xFu) == 0xFu;
            if (__all(all)) return;
#pragma unroll
            for (int g = 0; g < QG; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[g][e] = (ow[g] >> e) & 1u ? acc[g][e] : INF;
        };
        auto min4 = [&](const floatx4& A) {
#ifdef WV_H16_ABLATE_NO_MIN
            return A[0];
#endif
            return fminf(min3_raw(A[0], A[1], A[2]), A[3]);
        };
        // extraction thresholds: min(the column list's tail, tau)
        float pt[QG];
        auto refresh_pt = [&] {
#pragma unroll
            for (int g = 0; g < QG; ++g) pt[g] = fminf(__shfl(ld[g][HQ_KP - 1], l15 + 48, 64), tau[g]);
        };
        refresh_pt();
        // running threshold (no seed, no cross-slot threshold): entry k - 1 of
        // the column list (k distinct rows with keys <= it)
        const int ke = p.kth > 0 ? p.kth - 1 : 0;
        const int ksrc = l15 + 16 * (ke >> 2);
        const float u4 = 4.f * 5.9604645e-08f;
        auto publish = [&] {
            int ve = ke & 3;
            asm volatile("" : "+v"(ve));
#pragma unroll
            for (int g = 0; g < QG; ++g) {
                float v = FLT_MAX;
#pragma unroll
                for (int i = 0; i < HQ_KP; ++i) v = ve == i ? ld[g][i] : v;
                v = __shfl(v, ksrc, 64);
                if (lq == 0 && jqof(g) < p.nq && v < FLT_MAX) {
                    const float mg = p.marg[jqof(g)];
                    atomicMin(&p.gtau[jqof(g)], h16_key_enc(v + mg + u4 * (fabsf(v) + mg)));
                }
            }
#pragma unroll
            for (int g = 0; g < QG; ++g)
                if (jqof(g) < p.nq) tau[g] = fminf(tau[g], h16_key_dec(__atomic_load_n(&p.gtau[jqof(g)], __ATOMIC_RELAXED)));
            refresh_pt();
        };
        const bool xs = XS && !SEED && p.kth > 0;
        const bool running = !SEED && p.kth > 0 && p.gtau != nullptr && !xs;
        // cross-slot exchange (see above); lane (lq, l15) selects for query
        // groups lq and lq + 4 of column l15
        auto xslot_bound = [&](int jq) -> float {
            const int nv = 2 * p.n_slots;
            int nvv = jq < p.nq ? nv : 0;   // (opaque VGPR: a uniform bound keeps SGPR masks live)
            asm volatile("" : "+v"(nvv));
            const float* gs = p.gslot + (size_t)(jq < p.nq ? jq : 0) * nv;
            float v[32];
#pragma unroll
            for (int i = 0; i < 32; ++i)
                v[i] = i < nvv ? __hip_atomic_load(gs + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : FLT_MAX;
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
            int ve = p.kth - 1;
            asm volatile("" : "+v"(ve));
            float kv = FLT_MAX;
#pragma unroll
            for (int i = 0; i < 32; ++i) kv = i == ve ? v[i] : kv;
            if (!(jq < p.nq) || !(kv < 1e30f)) return FLT_MAX;
            const float mg = p.marg[jq];
            const float b = kv + mg + u4 * (fabsf(kv) + mg);
            // the finalize's tau_in must be <= every threshold a key was dropped above
            atomicMin(&p.gtau[jq], h16_key_enc(b));
            return b;
        };
        auto xslot_step = [&](bool rd, bool wr) {
            if (rd) {
                const float ba = xslot_bound(jqof(0) + 16 * lq);       // group lq
                const float bb = xslot_bound(jqof(0) + 16 * (lq + 4)); // group lq + 4
#pragma unroll
                for (int g = 0; g < QG; ++g) tau[g] = fminf(tau[g], __shfl(g < 4 ? ba : bb, l15 + 16 * (g & 3), 64));
                refresh_pt();
            }
            if (wr && lq == 0) {
                const int nv = 2 * p.n_slots;
#pragma unroll
                for (int g = 0; g < QG; ++g) {
                    if (jqof(g) >= p.nq) continue;
                    float* gs = p.gslot + (size_t)jqof(g) * nv + 2 * slot;
                    if (ld[g][0] < FLT_MAX) __hip_atomic_store(gs, ld[g][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (ld[g][1] < FLT_MAX) __hip_atomic_store(gs + 1, ld[g][1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        };
        // the epilogue of a row group: extraction of keys below the thresholds
        auto epilogue = [&](const floatx4 (&acc)[QG], const float (&m)[QG], uint32_t rb) {
            if constexpr (SEED) {
#pragma unroll
                for (int g = 0; g < QG; ++g) ld[g][0] = fminf(ld[g][0], m[g]);
            } else {
#ifdef WV_H16_ABLATE_NO_EXTRACT
                if (m[0] == 1234.5f) ld[0][0] = m[1] + m[2] + m[3] + pt[0];
                return;
#endif
                bool x[QG], anyx = false;
#pragma unroll
                for (int g = 0; g < QG; ++g) {
                    x[g] = m[g] <= pt[g];
                    anyx = anyx || x[g];
                }
                if (__builtin_expect(__any(anyx), 0)) {
                    WV_DBG_COUNT(3)
#pragma unroll
                    for (int g = 0; g < QG; ++g)
                        if (__any(x[g])) qcol_extract4(m[g], acc[g], ld[g], li[g], pt[g], tau[g], rb, lane);
                }
            }
        };

        uint64_t okw = 0;
        bool need_mask = false;
        const int xs1 = ntile / 8, xs2 = ntile / 4, xs3 = ntile / 2, xs4 = (3 * ntile) / 4;
        const int ngroups = (ntile + TPS - 1) / TPS;
        int ops_in_flight = 0;
        if (ngroups > 0) fill_group(t_begin, 0, ntile);
        if (ngroups > 1) ops_in_flight = fill_group(t_begin, 1, ntile);
        vm_wait(ops_in_flight);
        block_barrier();
        Frag fP, fQ;
        if (ntile > 0) {
            load_frag(tile_lds(0), 0, fP);
            pin_frag(fP);
            mfma_rg(fP, accX, [&] { load_frag(tile_lds(0), 1, fQ); });
            pin_frag(fQ);
            need_mask = tile_ok(t_begin, okw);
        }
        for (int t = 0; t < ntile; ++t) {
            WV_DBG_COUNT(0)
            const int g = t / TPS;
#ifndef WV_H16_ABLATE_NO_FILL
            if (t % TPS == 0) ops_in_flight = g + 2 < ngroups ? fill_group(t_begin, g + 2, ntile) : 0;
#endif
            const uint4* img = tile_lds(t);
            const uint32_t rb0 = (uint32_t)((t_begin + t) * (uint64_t)p.tile_stride * H_BN) + 4 * lq;
            const bool mask_t = need_mask;
            const uint64_t mo = okw;
            float m[QG];
            // step r: row group r's MFMAs beside row group r - 1's minima and
            // row group r + 1's fragment reads, then r - 1's extraction
            if (mask_t) mask_rg(accX, 0, mo);
            mfma_rg(fQ, accY, [&] {
                load_frag(img, 2, fP);
#pragma unroll
                for (int q = 0; q < QG; ++q) m[q] = min4(accX[q]);
            });
            pin_frag(fP);
            epilogue(accX, m, rb0);
            if (mask_t) mask_rg(accY, 1, mo);
            mfma_rg(fP, accX, [&] {
                load_frag(img, 3, fQ);
#pragma unroll
                for (int q = 0; q < QG; ++q) m[q] = min4(accY[q]);
            });
            pin_frag(fQ);
            epilogue(accY, m, rb0 + 16);
            // group g + 1 landed, every wave done with group g's stage: before
            // tile t + 1's first fragments are read
            if (t % TPS == TPS - 1 || t == ntile - 1) {
                if (g + 1 < ngroups) vm_wait(ops_in_flight);
                block_barrier();
            }
            const bool more = t + 1 < ntile;
            if (mask_t) mask_rg(accX, 2, mo);
            mfma_rg(fQ, accY, [&] {
                if (more) load_frag(tile_lds(t + 1), 0, fP);
#pragma unroll
                for (int q = 0; q < QG; ++q) m[q] = min4(accX[q]);
            });
            pin_frag(fP);
            epilogue(accX, m, rb0 + 32);
            if (mask_t) mask_rg(accY, 3, mo);
            if (more) {
                mfma_rg(fP, accX, [&] {
                    load_frag(tile_lds(t + 1), 1, fQ);
#pragma unroll
                    for (int q = 0; q < QG; ++q) m[q] = min4(accY[q]);
                });
                pin_frag(fQ);
                need_mask = tile_ok(t_begin + t + 1, okw);
            } else {
#pragma unroll
                for (int q = 0; q < QG; ++q) m[q] = min4(accY[q]);
            }
            epilogue(accY, m, rb0 + 48);
            if constexpr (!SEED) {
                if (running && (t & 15) == 15) publish();
                if constexpr (XS)
                    if (xs && (t == xs1 || t == xs2 || t == xs3 || t == xs4)) xslot_step(t != xs1, t != xs4);
            }
        }

        if constexpr (SEED) {
#pragma unroll
            for (int g = 0; g < QG; ++g)
                if (jqof(g) < p.nq) p.out_d[((size_t)jqof(g) * p.n_slots + slot) * HQ_PROD + lq] = ld[g][0];
            continue;
        }
        const size_t per_q = (size_t)p.n_slots * HQ_PROD * HQ_KP;
#pragma unroll
        for (int g = 0; g < QG; ++g) {
            if (jqof(g) >= p.nq) continue;
            const size_t base = (size_t)jqof(g) * per_q + (size_t)slot * HQ_PROD * HQ_KP + lq * HQ_KP;
#pragma unroll
            for (int i = 0; i < HQ_KP; ++i) { p.out_d[base + i] = ld[g][i]; p.out_id[base + i] = li[g][i]; }
        }
    }
}

}  // namespace wv

extern "C" {

hipError_t wv_launch_bf_h16s(const wv::H16Params* p, int ns32, int seed, hipStream_t s) {
    const uint64_t total = (uint64_t)p->n_qblocks * p->ntiles;
    const unsigned nb = (unsigned)((total + p->units_per_block - 1) / p->units_per_block);
    if (nb == 0) return hipSuccess;
    if (ns32 < 1 || ns32 > wv::H_NS_MAX / 2 || !p->X || !p->Q || !p->excl || !p->qscale || p->tile_stride < 1)
        return hipErrorInvalidValue;
    const bool l2 = p->metric == WV_METRIC_L2;
    if (l2 && !p->xns) return hipErrorInvalidValue;
    if (p->xslot && (!p->gslot || !p->gtau || !p->marg || p->kth < 1 || 2 * p->n_slots > 32)) return hipErrorInvalidValue;
    if (p->kth && (!p->gtau || !p->marg)) return hipErrorInvalidValue;
    const size_t lds = (size_t)wv::H_STAGES * wv::HS_TPS * (4 * ns32 * 64 + 17) * 16;
#define WV_H16S_GO(NS, L, S)                                                                                   \
    if (!S && p->xslot) hipLaunchKernelGGL((wv::wv_bf_h16s_kernel<NS, L, false, true>), dim3(nb), dim3(256), lds, s, *p); \
    else hipLaunchKernelGGL((wv::wv_bf_h16s_kernel<NS, L, S, false>), dim3(nb), dim3(256), lds, s, *p);
#define WV_H16S_LAUNCH(NS)                     \
    if (seed) {                                \
        if (l2) { WV_H16S_GO(NS, true, true) } \
        else { WV_H16S_GO(NS, false, true) }   \
    } else {                                   \
        if (l2) { WV_H16S_GO(NS, true, false) } \
        else { WV_H16S_GO(NS, false, false) }  \
    }
    switch (ns32) {
        case 1: WV_H16S_LAUNCH(1) break;
        case 2: WV_H16S_LAUNCH(2) break;
        case 3: WV_H16S_LAUNCH(3) break;
        default: WV_H16S_LAUNCH(4) break;
    }
#undef WV_H16S_LAUNCH
#undef WV_H16S_GO
    return hipGetLastError();
}

}  // extern "C"
