// wv_hnsw.hip -- HNSW search (knnSearchByVector) with one wavefront per query.
//
// Restates adapters/repos/db/vector/hnsw/search.go:
//   knnSearchByVector (:460-550): entry point, greedy ef=1 descent over the
//   upper layers, then the layer-0 beam search with ef and the allow list;
//   searchLayerByVector (:160-327).
//
// Graph layout in HBM (a fixed-degree CSR re-layout):
//   levels[N] int8 (-1 = nil node), layer0[N][deg0] u32 (pad 0xFFFFFFFF),
//   upper_row[N] u32, upper[n_upper][max_level][degU] u32, vectors[N][ldx] f32.
//
// Exactness.  The reference processes the neighbours of a popped candidate one
// by one; a neighbour is accepted when d < worst || |results| < ef, and worst
// only moves when an allowed, untombstoned neighbour enters the results.  On
// tie-free distances that sequential loop ends in the same state as
//   R' = the ef smallest of R u {eligible neighbours},
//   S' = S u {ineligible neighbours with d <= worst(R')} (all of them while R'
//        is not full),
// where R holds the results (a candidate is exactly an unexpanded member of R)
// and S holds the traversed-but-ineligible candidates (filtered-out or
// tombstoned, search.go:282-298).  Candidates with d > worst can never be
// expanded (the loop breaks on them, :213-215), so they are not stored.  The
// wave therefore computes all neighbour distances in parallel (bit-identical
// to the reference distancer), sorts them, and merges the batch into R and S.
// The visited list (:256-264) is a lossy LDS cache: a node it forgets is
// re-evaluated, and re-evaluating a visited node cannot change R or S (its
// key is already in R/S, was evicted with d > worst, or it was expanded from S,
// which the exact set X records), so pruning with any subset of the visited
// set is exact.
#include "wv_device.h"
#include "wv_h16_dev.h"
#include "wv_params.h"

#include <float.h>
#include <cstdlib>

namespace wv {


constexpr int BATCH = 128;
constexpr int MAX_LOCAL_TOMB = 4;
// rows per 8-lane group in one distance round trip (exact_dist_rows)
#ifndef WV_HNSW_RPG
#define WV_HNSW_RPG 4
#endif
// rows per 8-lane group on the side-register path (24 rows a trip: at 4 it
// spilled ~25 VGPRs at 3 waves per SIMD; 3 measured fastest of 2 / 3 / 4 on
// the C1 graph with 1 % tombstones and 10 / 50 % allow lists,
// profiles/r06/side_rpg_wps_ab.log)
#ifndef WV_HNSW_SIDE_RPG
#define WV_HNSW_SIDE_RPG 3
#endif

// Diagnostic build only (-DWV_HNSW_STAMPS, tools/hnsw_latency.sh): per-phase
// shader-clock cycles of the expansion loop, summed over the queries of a
// launch -- pop, neighbour-id/level load, visited filter, distances, merge --
// plus the whole query's cycles and wall ticks (100 MHz).  Empty otherwise.
struct Stamps {
#ifdef WV_HNSW_STAMPS
    uint64_t acc[5] = {0, 0, 0, 0, 0};
    uint64_t t = 0;
    __device__ __forceinline__ void start() { t = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void lap(int i) {
        const uint64_t n = __builtin_amdgcn_s_memtime();
        acc[i] += n - t;
        t = n;
    }
#else
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void lap(int) {}
#endif
};
#ifdef WV_HNSW_STAMPS
__device__ unsigned long long wv_hnsw_stamps[16];
extern "C" void wv_hnsw_stamps_read(unsigned long long* out, int reset) {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(wv_hnsw_stamps), sizeof(wv_hnsw_stamps));
    if (reset) {
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(wv_hnsw_stamps), z, sizeof(z));
    }
}
#endif

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct WaveState {
    float* qv;
    float* Rd; uint32_t* Ri;
    float* Rd2; uint32_t* Ri2;
    float* Sd; uint32_t* Si;
    float* Sd2; uint32_t* Si2;
    float* Bd; uint32_t* Bi;    // raw batch (distance by batch slot)
    float* Cd; uint32_t* Ci;    // sorted batch
    uint16_t* vc;   // visited cache (HnswParams.vc_tbits)
    uint32_t* xs;
    uint32_t* ltomb;
    uint32_t* ew;   // side path: the batch's eligibility words (LDS-DMA targets, 4 x 64)
    unsigned long long* ub;   // this query's exact visited bitmap (diagnostic counts; nullable)
    volatile int* wg_nb;      // workgroup-per-query launch: the batch size the helpers read (-1: done)
};

// the diagnostic count of a batch's layer-0 evaluations: nodes first
// evaluated now (their bit set by this wave); every evaluation otherwise
__device__ __forceinline__ uint32_t eval_count(const WaveState& w, int level, int nb, bool v0, uint32_t id0, bool v1,
                                               uint32_t id1) {
    if (level != 0 || !w.ub) return (uint32_t)nb;
    bool f0 = false, f1 = false;
    if (v0) {
        const unsigned long long b = 1ull << (id0 & 63);
        f0 = !(atomicOr(w.ub + (id0 >> 6), b) & b);
    }
    if (v1) {
        const unsigned long long b = 1ull << (id1 & 63);
        f1 = !(atomicOr(w.ub + (id1 >> 6), b) & b);
    }
    return (uint32_t)(__popcll(__ballot(f0)) + __popcll(__ballot(f1)));
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) { return x * 2654435761u; }

// visited-cache slot and tag of a node id (HnswParams.vc_tbits)
__device__ __forceinline__ uint32_t vc_hash(const HnswParams& p, uint32_t id) {
    return hash32(id) & ((1u << (p.vc_log2 + p.vc_tbits)) - 1u);
}
__device__ __forceinline__ uint32_t vc_slot(const HnswParams& p, uint32_t h) { return h >> p.vc_tbits; }
__device__ __forceinline__ uint16_t vc_tag(const HnswParams& p, uint32_t h) {
    return (uint16_t)(h & ((1u << p.vc_tbits) - 1u));
}
constexpr uint16_t VC_EMPTY = 0xFFFF;

// lower bound: number of entries of a sorted (d,id) array with key < (d,id)
__device__ __forceinline__ int lower_bound(const float* ad, const uint32_t* ai, int n, float d, uint32_t id) {
    int lo = 0, len = n;
    while (len > 0) {
        const int half = len >> 1;
        const int mid = lo + half;
        if (key_less(ad[mid], ai[mid], d, id)) {
            lo = mid + 1;
            len = len - half - 1;
        } else {
            len = half;
        }
    }
    return lo;
}

template <int METRIC, bool PQ = false>
__device__ __forceinline__ void search_layer(const HnswParams& p, WaveState& w_io, int level, int ef, uint32_t ep,
                             float epd, const uint64_t* allow, int& Rl_out, int& Sh_out, int& Sl_out, int& status,
                             int nlt, uint32_t& n_dist, uint32_t& n_exp, Stamps& ts) {
    // the state lives in registers for the whole layer (LDS pointers and the
    // R / S lengths are wave-uniform); written back once at the end
    WaveState w = w_io;
    const int lane = threadIdx.x & 63;
    const int VC = 1 << p.vc_log2;
    const int XS = 1 << p.xs_log2;
    for (int i = lane; i < VC; i += 64) w.vc[i] = VC_EMPTY;
    for (int i = lane; i < XS; i += 64) w.xs[i] = WV_NIL;
    wave_sync();

    auto eligible = [&](uint32_t id) -> bool {
        if (p.tomb && bit_test(p.tomb, p.tomb_nbits, id)) return false;
        for (int t = 0; t < nlt; ++t)
            if (w.ltomb[t] == id) return false;
        if (level == 0 && allow && !bit_test(allow, p.allow_nbits, id)) return false;
        return true;
    };

    // insertViableEntrypointsAsCandidatesAndResults (search.go:329-353)
    if (lane == 0) {
        const uint32_t he = vc_hash(p, ep);
        w.vc[vc_slot(p, he)] = vc_tag(p, he);
    }
    const bool ep_ok = eligible(ep);
    if (lane == 0) {
        float* dd = ep_ok ? w.Rd : w.Sd;
        uint32_t* di = ep_ok ? w.Ri : w.Si;
        dd[0] = epd;
        di[0] = ep;
    }
    int Rl = ep_ok ? 1 : 0, Sh = 0, Sl = ep_ok ? 0 : 1;
    wave_sync();
    // currentWorstResultDistanceToFloat (:355-377)
    float worst = Rl > 0 ? w.Rd[Rl - 1] : FLT_MAX;

    const uint32_t* nbr_base;
    int deg;
    ts.start();
    for (;;) {
        // A full side set or expanded-set table makes the state inexact (an
        // expanded side candidate that X cannot record would be re-inserted
        // and expanded again, forever): stop, the query is answered by the
        // exact fallback (status != 0).
        if (status) break;
        // ---- pop the best live candidate: first unexpanded R entry vs S head ----
        int ridx = Rl;
        for (int base = 0; base < Rl; base += 64) {
            const int i = base + lane;
            const bool unexp = i < Rl && !(w.Ri[i] & WV_FLAG);
            const uint64_t m = __ballot(unexp);
            if (m) { ridx = base + __builtin_ctzll(m); break; }
        }
        const bool haveR = ridx < Rl;
        const bool haveS = Sl > 0;
        if (!haveR && !haveS) break;
        float cd; uint32_t cid; bool fromR;
        if (haveR && (!haveS || key_less(w.Rd[ridx], w.Ri[ridx], w.Sd[Sh], w.Si[Sh]))) {
            cd = w.Rd[ridx]; cid = w.Ri[ridx] & WV_IDMASK; fromR = true;
        } else {
            cd = w.Sd[Sh]; cid = w.Si[Sh]; fromR = false;
        }
        if (cd > worst) break;  // :213-215
        wave_sync();
        if (fromR) {
            if (lane == 0) w.Ri[ridx] = cid | WV_FLAG;
        } else {
            Sh++; Sl--;
            // record the expansion in X (exact open-addressing set)
            if (lane == 0) {
                uint32_t h = hash32(cid) >> (32 - p.xs_log2);
                int probes = 0;
                while (w.xs[h] != WV_NIL && w.xs[h] != cid && probes < XS) { h = (h + 1) & (XS - 1); probes++; }
                if (probes >= XS) status |= 2;
                else w.xs[h] = cid;
            }
            status = __shfl(status, 0, 64);
        }
        wave_sync();
        ts.lap(0);
        // :217-234 nil node / level check.  Every layer-0 row exists (nil
        // nodes hold pads), so there the first neighbour ids are fetched in
        // the same memory round trip as the level.
        uint32_t pre0 = WV_NIL, pre1 = WV_NIL;
        if (level == 0) {
            nbr_base = p.layer0 + (uint64_t)cid * p.deg0;
            deg = p.deg0;
            if (lane < deg) pre0 = nbr_base[lane];
            if (64 + lane < deg) pre1 = nbr_base[64 + lane];
            if (p.levels[cid] < 0) continue;
        } else {
            if (p.levels[cid] < level) continue;
            const uint32_t row = p.upper_row[cid];
            nbr_base = p.upper + ((uint64_t)row * p.upper_levels + (level - 1)) * p.degU;
            deg = p.degU;
        }
        n_exp++;
        ts.lap(1);

        for (int c0 = 0; c0 < deg; c0 += BATCH) {
            // ---- neighbour ids, visited-cache filter, compaction ----
            uint32_t id0 = WV_NIL, id1 = WV_NIL;
            if (level == 0 && c0 == 0) {
                id0 = pre0;
                id1 = pre1;
            } else {
                if (c0 + lane < deg) id0 = nbr_base[c0 + lane];
                if (c0 + 64 + lane < deg) id1 = nbr_base[c0 + 64 + lane];
            }
            bool v0 = id0 != WV_NIL && id0 < p.N;
            bool v1 = id1 != WV_NIL && id1 < p.N;
            const uint32_t e0 = vc_hash(p, id0), e1 = vc_hash(p, id1);
            const uint32_t h0 = v0 ? vc_slot(p, e0) : 0, h1 = v1 ? vc_slot(p, e1) : 0;
            const uint16_t t0 = vc_tag(p, e0), t1 = vc_tag(p, e1);
            if (v0 && w.vc[h0] == t0) v0 = false;
            if (v1 && w.vc[h1] == t1) v1 = false;
            wave_sync();
            if (v0) w.vc[h0] = t0;
            if (v1) w.vc[h1] = t1;
            const uint64_t m0 = __ballot(v0), m1 = __ballot(v1);
            const int n0 = __popcll(m0);
            const int nb = n0 + __popcll(m1);
            if (v0) w.Bi[mbcnt64(m0)] = id0;
            if (v1) w.Bi[n0 + mbcnt64(m1)] = id1;
            wave_sync();
            ts.lap(2);
            if (nb == 0) continue;

            // ---- exact distances, 8 lanes per row (search.go:265-271); on a
            // compressed index one lane per row from the codes (:196-199) ----
            if (PQ) {
                for (int base = 0; base < nb; base += 64)
                    if (base + lane < nb) w.Bd[base + lane] = pq_dist_row<METRIC>(w.qv, p.pq, w.Bi[base + lane]);
            } else {
                for (int base = 0; base < nb; base += 8 * WV_HNSW_RPG)
                    exact_dist_rows<METRIC, WV_HNSW_RPG>(w.qv, p.X, p.ldx, p.D, w.Bi + base, nb - base, w.Bd + base,
                                                         lane);
            }
            n_dist += eval_count(w, level, nb, v0, id0, v1, id1);
            wave_sync();
            ts.lap(3);

            // ---- keep test + dedupe (lanes hold batch slots lane, lane+64) ----
            // Only a neighbour the reference pushes into the candidate heap
            // matters: d < worst || |results| < ef (search.go:282).  worst only
            // falls while R is full, so the pre-batch worst keeps a superset;
            // the merge below settles the rest.  Late in a search most
            // neighbours fail here and the batch ends without any sorting.
            uint32_t cls[2]; float bd[2]; uint32_t bi[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = lane + 64 * h;
                cls[h] = 2; bd[h] = FLT_MAX; bi[h] = WV_NIL;
                if (e < nb) {
                    const uint32_t id = w.Bi[e];
                    const float d = w.Bd[e];
                    if (d < worst || Rl < ef) {
                        const bool el = eligible(id);
                        bool dup;
                        if (el) {
                            const int pos = lower_bound(w.Rd, w.Ri, Rl, d, id);
                            dup = pos < Rl && w.Rd[pos] == d && (w.Ri[pos] & WV_IDMASK) == id;
                        } else {
                            const int pos = lower_bound(w.Sd + Sh, w.Si + Sh, Sl, d, id);
                            dup = pos < Sl && w.Sd[Sh + pos] == d && w.Si[Sh + pos] == id;
                            if (!dup) {
                                uint32_t hh = hash32(id) >> (32 - p.xs_log2);
                                for (int pr = 0; pr < XS; ++pr) {
                                    const uint32_t v = w.xs[hh];
                                    if (v == id) { dup = true; break; }
                                    if (v == WV_NIL) break;
                                    hh = (hh + 1) & (XS - 1);
                                }
                            }
                        }
                        if (!dup) { cls[h] = el ? 0 : 1; bd[h] = d; bi[h] = id; }
                    }
                }
            }
            const uint64_t me0 = __ballot(cls[0] == 0), me1 = __ballot(cls[1] == 0);
            const uint64_t ms0 = __ballot(cls[0] == 1), ms1 = __ballot(cls[1] == 1);
            const int ne = __popcll(me0) + __popcll(me1);
            const int ns = __popcll(ms0) + __popcll(ms1);
            if (ne + ns == 0) {
                wave_sync();
                ts.lap(4);
                continue;
            }
            // compact the kept keys into the (consumed) raw batch: eligible
            // [0, ne), ineligible [ne, ne + ns)
            wave_sync();
            if (cls[0] == 0) { const int u = mbcnt64(me0); w.Bd[u] = bd[0]; w.Bi[u] = bi[0]; }
            if (cls[1] == 0) { const int u = __popcll(me0) + mbcnt64(me1); w.Bd[u] = bd[1]; w.Bi[u] = bi[1]; }
            if (cls[0] == 1) { const int u = ne + mbcnt64(ms0); w.Bd[u] = bd[0]; w.Bi[u] = bi[0]; }
            if (cls[1] == 1) { const int u = ne + __popcll(ms0) + mbcnt64(ms1); w.Bd[u] = bd[1]; w.Bi[u] = bi[1]; }
            wave_sync();
            // rank sort inside each class by (d, id); equal keys (a neighbour
            // listed twice) keep their batch order
            for (int u = lane; u < ne + ns; u += 64) {
                const float d = w.Bd[u];
                const uint32_t id = w.Bi[u];
                const int lo = u < ne ? 0 : ne, hi = u < ne ? ne : ne + ns;
                int r = lo;
                for (int i = lo; i < hi; ++i) {
                    const float di = w.Bd[i];
                    const uint32_t ii = w.Bi[i];
                    r += key_less(di, ii, d, id) || (i < u && di == d && ii == id);
                }
                w.Cd[r] = d;
                w.Ci[r] = id;
            }
            wave_sync();

            // ---- merge eligible [0, ne) into R (cap ef) ----
            if (ne > 0) {
                const int newRl = min(ef, Rl + ne);
                for (int i = lane; i < Rl; i += 64) {
                    const float d = w.Rd[i];
                    const uint32_t id = w.Ri[i];
                    const int pos = i + lower_bound(w.Cd, w.Ci, ne, d, id);
                    if (pos < newRl) { w.Rd2[pos] = d; w.Ri2[pos] = id; }
                }
                for (int j = lane; j < ne; j += 64) {
                    const float d = w.Cd[j];
                    const uint32_t id = w.Ci[j];
                    const int pos = j + lower_bound(w.Rd, w.Ri, Rl, d, id);
                    if (pos < newRl) { w.Rd2[pos] = d; w.Ri2[pos] = id; }
                }
                wave_sync();
                float* td = w.Rd; w.Rd = w.Rd2; w.Rd2 = td;
                uint32_t* ti = w.Ri; w.Ri = w.Ri2; w.Ri2 = ti;
                Rl = newRl;
                worst = w.Rd[Rl - 1];
            }
            // ---- side candidates: keep live ones, prune S by worst ----
            int nsk = ns;
            if (Rl >= ef) {
                // live iff d <= worst; the ineligible run [ne, ne+ns) is sorted
                nsk = lower_bound(w.Cd + ne, w.Ci + ne, ns, worst, 0xFFFFFFFFu) ;
                // entries equal to worst with any id are live: lower_bound with id max
                // counts keys < (worst, max id) -> all d < worst and d == worst
                const int sl_live = lower_bound(w.Sd + Sh, w.Si + Sh, Sl, worst, 0xFFFFFFFFu);
                Sl = sl_live;
            }
            if (nsk > 0) {
                int newSl = Sl + nsk;
                if (newSl > p.sc) { newSl = p.sc; status |= 1; }
                for (int i = lane; i < Sl; i += 64) {
                    const float d = w.Sd[Sh + i];
                    const uint32_t id = w.Si[Sh + i];
                    const int pos = i + lower_bound(w.Cd + ne, w.Ci + ne, nsk, d, id);
                    if (pos < newSl) { w.Sd2[pos] = d; w.Si2[pos] = id; }
                }
                for (int j = lane; j < nsk; j += 64) {
                    const float d = w.Cd[ne + j];
                    const uint32_t id = w.Ci[ne + j];
                    const int pos = j + lower_bound(w.Sd + Sh, w.Si + Sh, Sl, d, id);
                    if (pos < newSl) { w.Sd2[pos] = d; w.Si2[pos] = id; }
                }
                wave_sync();
                float* td = w.Sd; w.Sd = w.Sd2; w.Sd2 = td;
                uint32_t* ti = w.Si; w.Si = w.Si2; w.Si2 = ti;
                Sh = 0;
                Sl = newSl;
            }
            wave_sync();
            ts.lap(4);
        }
    }
    Rl_out = Rl;
    Sh_out = Sh;
    Sl_out = Sl;
    w_io = w;
}


// wave-wide shift by one lane toward higher lanes (lane 0 keeps its value)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ float wave_shr1(float v) { return __uint_as_float(wave_shr1(__float_as_uint(v))); }

// The unfiltered search with ef <= 64 NR (no allow list, tombstones or nil
// nodes: every node is eligible, so S stays empty): the results R live in
// registers, entry i in lane i % 64 of register i / 64 (distance rd, id ri,
// WV_FLAG once expanded).  The pop is a ballot; a neighbour that passes the
// keep test (d < worst || |R| < ef, search.go:282) is inserted by one ballot
// per register (its rank), a duplicate check on the entry at that rank and a
// one-lane DPP shift of the tail (lane 63 of a register carried into lane 0
// of the next).  Inserting the
// kept neighbours one by one ends in the same R as the LDS path's sorted batch
// merge (the ef smallest keys of R and the kept neighbours, duplicates once),
// so the expansion order and the results are the same, bit for bit.
// (e is wave-uniform: the register is picked by scalar compares)
template <int NR>
__device__ __forceinline__ float reg_entry_d(const float (&rd)[NR], int e) {
    float v = rd[0];
#pragma unroll
    for (int r = 1; r < NR; ++r)
        if ((e >> 6) == r) v = rd[r];
    return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), e & 63));
}
template <int NR>
__device__ __forceinline__ uint32_t reg_entry_i(const uint32_t (&ri)[NR], int e) {
    uint32_t v = ri[0];
#pragma unroll
    for (int r = 1; r < NR; ++r)
        if ((e >> 6) == r) v = ri[r];
    return (uint32_t)__builtin_amdgcn_readlane(v, e & 63);
}

// Distances of a batch in a workgroup-per-query launch: wave v computes rows
// 32 v .. 32 v + 31 (all of them at once, one memory round trip: a lone
// wave's two trips of 32 rows were 66 % of an expansion, and one CU's
// gathers are bound by the bytes it has in flight).  Wave 0 publishes nb; the
// helpers (wg_helper) wait at the same two barriers.
//
// Barrier invariant (wv_hnsw_wg_kernel): wave 0 reaches __syncthreads only
// inside wg_dist (exactly two per call) and once after knn_one_reg returns
// (the -1 "done" barrier); the helpers pair each with their loop's two.  So
// knn_one_reg / search_layer_reg must never return early past a pending
// wg_dist pair nor add a barrier of their own on the wg path: every path out
// of them ends at the kernel's final barrier.  (test_gpu_parity.py
// test_hnsw_workgroup_launch_edge_graphs: 1- and 2-node graphs, k = ef = 1.)
template <int METRIC>
__device__ __forceinline__ void wg_dist(const HnswParams& p, const WaveState& w, int nb, int lane) {
    if (lane == 0) *w.wg_nb = nb;
    __syncthreads();
    exact_dist_rows<METRIC, 4, true>(w.qv, p.X, p.ldx, p.D, w.Bi, min(nb, 32), w.Bd, lane);
    __syncthreads();
}
template <int METRIC>
__device__ void wg_helper(const HnswParams& p, const WaveState& w, int wave, int lane) {
    for (;;) {
        __syncthreads();
        const int nb = *w.wg_nb;
        if (nb < 0) break;
        const int base = 32 * wave;
        if (base < nb)
            exact_dist_rows<METRIC, 4, true>(w.qv, p.X, p.ldx, p.D, w.Bi + base, min(nb - base, 32), w.Bd + base, lane);
        __syncthreads();
    }
}

template <int METRIC, bool PQ, int NR>
__device__ __forceinline__ void search_layer_reg(const HnswParams& p, WaveState& w, int level, int ef, uint32_t ep,
                                                 float epd, float (&rd)[NR], uint32_t (&ri)[NR], int& Rl,
                                                 uint32_t& n_dist, uint32_t& n_exp, Stamps& ts) {
    static_assert(NR == 1 || NR == 2 || NR == 4, "64, 128 or 256 results per wave");
    const int lane = threadIdx.x & 63;
    const int VC = 1 << p.vc_log2;
    for (int i = lane; i < VC; i += 64) w.vc[i] = VC_EMPTY;
    wave_sync();
    if (lane == 0) {
        const uint32_t he = vc_hash(p, ep);
        w.vc[vc_slot(p, he)] = vc_tag(p, he);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        rd[r] = lane == 0 && r == 0 ? epd : FLT_MAX;
        ri[r] = lane == 0 && r == 0 ? ep : WV_NIL;
    }
    Rl = 1;
    float worst = epd;
    wave_sync();
    const uint32_t* nbr_base;
    int deg;
    ts.start();
    for (;;) {
        // ---- pop the best unexpanded result ----
        int ridx = -1;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint64_t um = __ballot(64 * r + lane < Rl && !(ri[r] & WV_FLAG));
            if (ridx < 0 && um) ridx = 64 * r + __builtin_ctzll(um);
        }
        if (ridx < 0) break;
        const float cd = reg_entry_d<NR>(rd, ridx);
        const uint32_t cid = reg_entry_i<NR>(ri, ridx) & WV_IDMASK;
        if (cd > worst) break;   // :213-215
#pragma unroll
        for (int r = 0; r < NR; ++r)
            if (64 * r + lane == ridx) ri[r] |= WV_FLAG;
        ts.lap(0);
        uint32_t pre0 = WV_NIL, pre1 = WV_NIL;
        if (level == 0) {
            nbr_base = p.layer0 + (uint64_t)cid * p.deg0;
            deg = p.deg0;
            if (lane < deg) pre0 = nbr_base[lane];
            if (64 + lane < deg) pre1 = nbr_base[64 + lane];
            if (p.levels[cid] < 0) continue;
        } else {
            if (p.levels[cid] < level) continue;
            const uint32_t row = p.upper_row[cid];
            nbr_base = p.upper + ((uint64_t)row * p.upper_levels + (level - 1)) * p.degU;
            deg = p.degU;
        }
        n_exp++;
        ts.lap(1);
        for (int c0 = 0; c0 < deg; c0 += BATCH) {
            uint32_t id0 = WV_NIL, id1 = WV_NIL;
            if (level == 0 && c0 == 0) {
                id0 = pre0;
                id1 = pre1;
            } else {
                if (c0 + lane < deg) id0 = nbr_base[c0 + lane];
                if (c0 + 64 + lane < deg) id1 = nbr_base[c0 + 64 + lane];
            }
            bool v0 = id0 != WV_NIL && id0 < p.N;
            bool v1 = id1 != WV_NIL && id1 < p.N;
            const uint32_t e0 = vc_hash(p, id0), e1 = vc_hash(p, id1);
            const uint32_t h0 = v0 ? vc_slot(p, e0) : 0, h1 = v1 ? vc_slot(p, e1) : 0;
            const uint16_t t0 = vc_tag(p, e0), t1 = vc_tag(p, e1);
            if (v0 && w.vc[h0] == t0) v0 = false;
            if (v1 && w.vc[h1] == t1) v1 = false;
            wave_sync();
            if (v0) w.vc[h0] = t0;
            if (v1) w.vc[h1] = t1;
            const uint64_t m0 = __ballot(v0), m1 = __ballot(v1);
            const int n0 = __popcll(m0);
            const int nb = n0 + __popcll(m1);
            if (v0) w.Bi[mbcnt64(m0)] = id0;
            if (v1) w.Bi[n0 + mbcnt64(m1)] = id1;
            wave_sync();
            ts.lap(2);
            if (nb == 0) continue;
            if (PQ) {
                for (int base = 0; base < nb; base += 64)
                    if (base + lane < nb) w.Bd[base + lane] = pq_dist_row<METRIC>(w.qv, p.pq, w.Bi[base + lane]);
            } else if (p.wg_helpers) {
                wg_dist<METRIC>(p, w, nb, lane);
            } else {
                for (int base = 0; base < nb; base += 8 * WV_HNSW_RPG)
                    exact_dist_rows<METRIC, WV_HNSW_RPG, true>(w.qv, p.X, p.ldx, p.D, w.Bi + base, nb - base, w.Bd + base,
                                                         lane);
            }
            n_dist += eval_count(w, level, nb, v0, id0, v1, id1);
            wave_sync();
            ts.lap(3);
            // ---- keep test against the batch's starting R (as the LDS path's
            // merge), then one insertion per kept neighbour, in batch order; a
            // kept key ranked past ef falls out like the merge's tail ----
            float bd[2];
            uint32_t bi[2];
            uint64_t kmask[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = lane + 64 * h;
                bd[h] = e < nb ? w.Bd[e] : FLT_MAX;
                bi[h] = e < nb ? w.Bi[e] : WV_NIL;
                kmask[h] = __ballot(e < nb && (bd[h] < worst || Rl < ef));
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint64_t km = kmask[h];
                while (km) {
                    const int src = __builtin_ctzll(km);
                    km &= km - 1;
                    const float d = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(bd[h]), src));
                    const uint32_t id = (uint32_t)__builtin_amdgcn_readlane(bi[h], src);
                    int pos = 0;
#pragma unroll
                    for (int r = 0; r < NR; ++r)
                        pos += __popcll(__ballot((64 * r + lane < Rl) & key_less_nb(rd[r], ri[r] & WV_IDMASK, d, id)));
                    if (pos >= ef) continue;
                    if (pos < Rl && reg_entry_d<NR>(rd, pos) == d && (reg_entry_i<NR>(ri, pos) & WV_IDMASK) == id)
                        continue;   // already a result (a neighbour the visited cache forgot)
                    float sd[NR];
                    uint32_t si[NR];
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        sd[r] = wave_shr1(rd[r]);
                        si[r] = wave_shr1(ri[r]);
                        if (r > 0) {   // (lane 63 of the register below moves to lane 0)
                            const float cdv = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rd[r - 1]), 63));
                            const uint32_t civ = (uint32_t)__builtin_amdgcn_readlane(ri[r - 1], 63);
                            if (lane == 0) { sd[r] = cdv; si[r] = civ; }
                        }
                    }
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        const int e = 64 * r + lane;
                        if (e > pos) { rd[r] = sd[r]; ri[r] = si[r]; }
                        if (e == pos) { rd[r] = d; ri[r] = id; }
                    }
                    Rl = min(Rl + 1, ef);
                    worst = reg_entry_d<NR>(rd, Rl - 1);
                }
            }
            ts.lap(4);
        }
    }
}

template <int METRIC, bool PQ, int NR>
__device__ __forceinline__ void knn_one_reg(const HnswParams& p, WaveState& w, int q) {
    const int lane = threadIdx.x & 63;
    const int g = lane & 7;
    for (int i = lane; i < p.dpad; i += 64) w.qv[i] = i < p.D ? p.Q[(uint64_t)q * p.ldq + i] : 0.f;
    wave_sync();
    uint32_t n_dist = 0, n_exp = 0;
    Stamps ts;
#ifdef WV_HNSW_STAMPS
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t ep = p.entrypoint;
    float epd = PQ ? pq_dist_row<METRIC>(w.qv, p.pq, ep)
                   : exact_dist_group8<METRIC>(w.qv, p.X + (uint64_t)ep * p.ldx, p.D, g);
    epd = __shfl(epd, 0, 64);
    n_dist++;
    float rd[NR];
    uint32_t ri[NR];
    int Rl;
    for (int level = p.max_level; level >= 1; --level) {
        search_layer_reg<METRIC, PQ, NR>(p, w, level, 1, ep, epd, rd, ri, Rl, n_dist, n_exp, ts);
        // (no nil nodes on this path: the closest result is the next entry)
        ep = (uint32_t)__builtin_amdgcn_readlane(ri[0], 0) & WV_IDMASK;
        epd = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rd[0]), 0));
    }
    search_layer_reg<METRIC, PQ, NR>(p, w, 0, p.ef, ep, epd, rd, ri, Rl, n_dist, n_exp, ts);
    const int n = min(Rl, p.k);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = 64 * r + lane;
        if (e < n) {
            p.out_ids[(uint64_t)q * p.k + e] = p.id_base + (ri[r] & WV_IDMASK);
            p.out_d[(uint64_t)q * p.k + e] = rd[r];
        }
    }
    if (lane == 0) {
        p.out_n[q] = n;
        p.status[q] = 0;
        if (p.counters) { p.counters[2 * q] = n_dist; p.counters[2 * q + 1] = n_exp; }
#ifdef WV_HNSW_STAMPS
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < 5; ++i) atomicAdd(&wv_hnsw_stamps[i], (unsigned long long)ts.acc[i]);
        atomicAdd(&wv_hnsw_stamps[5], (unsigned long long)(c1 - c0));
        atomicAdd(&wv_hnsw_stamps[6], (unsigned long long)(w1 - w0));
        atomicAdd(&wv_hnsw_stamps[7], (unsigned long long)n_exp);
        atomicAdd(&wv_hnsw_stamps[8], 1ull);
        atomicAdd(&wv_hnsw_stamps[9], (unsigned long long)n_dist);
#endif
    }
}

template <int METRIC, bool PQ>
__device__ __forceinline__ void knn_one(const HnswParams& p, WaveState& w, int q) {
    const int lane = threadIdx.x & 63;
    const int g = lane & 7;
    // query -> LDS
    for (int i = lane; i < p.dpad; i += 64) w.qv[i] = i < p.D ? p.Q[(uint64_t)q * p.ldq + i] : 0.f;
    wave_sync();
    const uint64_t* allow = p.allow ? p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0) : nullptr;
    int status = 0;
    uint32_t n_dist = 0, n_exp = 0;
    int nlt = 0;
    Stamps ts;
#ifdef WV_HNSW_STAMPS
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
#endif

    // entry point distance (search.go:467-476)
    uint32_t ep = p.entrypoint;
    float epd = PQ ? pq_dist_row<METRIC>(w.qv, p.pq, ep)   // index.go:493-511
                   : exact_dist_group8<METRIC>(w.qv, p.X + (uint64_t)ep * p.ldx, p.D, g);
    epd = __shfl(epd, 0, 64);
    n_dist++;
    int Rl, Sh, Sl;
    // greedy descent, levels max..1 with ef = 1 (:479-521)
    for (int level = p.max_level; level >= 1; --level) {
        search_layer<METRIC, PQ>(p, w, level, 1, ep, epd, nullptr, Rl, Sh, Sl, status, nlt, n_dist, n_exp, ts);
        if (Rl > 0) {
            const uint32_t cid = w.Ri[0] & WV_IDMASK;
            if (p.levels[cid] < 0) {
                // nil node in the results: tombstoned by the reference (:496-507)
                if (nlt < MAX_LOCAL_TOMB) {
                    if (lane == 0) w.ltomb[nlt] = cid;
                    nlt++;
                }
                wave_sync();
            } else {
                ep = cid;
                epd = w.Rd[0];
            }
        }
    }
    // layer 0 with ef and the allow list (:523-528)
    search_layer<METRIC, PQ>(p, w, 0, p.ef, ep, epd, allow, Rl, Sh, Sl, status, nlt, n_dist, n_exp, ts);
    const int n = min(Rl, p.k);
    for (int i = lane; i < n; i += 64) {
        p.out_ids[(uint64_t)q * p.k + i] = p.id_base + (w.Ri[i] & WV_IDMASK);
        p.out_d[(uint64_t)q * p.k + i] = w.Rd[i];
    }
    if (lane == 0) {
        p.out_n[q] = n;
        p.status[q] = status;
        if (p.counters) { p.counters[2 * q] = n_dist; p.counters[2 * q + 1] = n_exp; }
#ifdef WV_HNSW_STAMPS
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < 5; ++i) atomicAdd(&wv_hnsw_stamps[i], (unsigned long long)ts.acc[i]);
        atomicAdd(&wv_hnsw_stamps[5], (unsigned long long)(c1 - c0));
        atomicAdd(&wv_hnsw_stamps[6], (unsigned long long)(w1 - w0));
        atomicAdd(&wv_hnsw_stamps[7], (unsigned long long)n_exp);
        atomicAdd(&wv_hnsw_stamps[8], 1ull);
        atomicAdd(&wv_hnsw_stamps[9], (unsigned long long)n_dist);
#endif
    }
}

// LDS of a register-results wave (hnsw_reg_per_wave_words): query, batch,
// visited cache, local tombstones
__device__ __forceinline__ void reg_wave_state(const HnswParams& p, float* cur, WaveState& w) {
    w.qv = cur; cur += p.dpad;
    w.Bd = cur; cur += BATCH; w.Bi = reinterpret_cast<uint32_t*>(cur); cur += BATCH;
    w.ltomb = reinterpret_cast<uint32_t*>(cur); cur += MAX_LOCAL_TOMB;
    w.vc = reinterpret_cast<uint16_t*>(cur);
}

// One instantiation per (metric, raw / PQ, LDS results / 64 / 128 / 256 register
// results): each gets its own register allocation (one kernel holding all six
// inlined searches spilled 431 SGPRs into VGPR lanes); the host launches the
// matching one.
template <int METRIC, bool PQ, int NR>
__global__ __launch_bounds__(256) void wv_hnsw_kernel(HnswParams p) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6;
    const int q = blockIdx.x * (blockDim.x >> 6) + wave;
    if (q >= p.nq) return;
    if (p.redo && p.redo[q] == 0) return;   // (second pass: this query completed)
    float* base = lds + (uint64_t)wave * p.per_wave_words;
    WaveState w;
    if constexpr (NR > 0) {   // register results: no R, S, sorted batch or X in LDS
        reg_wave_state(p, base, w);
        w.ub = p.uniq ? p.uniq + (uint64_t)q * p.uniq_words : nullptr;
        knn_one_reg<METRIC, PQ, NR>(p, w, q);
    } else {
        float* cur = base;
        w.qv = cur; cur += p.dpad;
        w.Rd = cur; cur += p.efc; w.Ri = reinterpret_cast<uint32_t*>(cur); cur += p.efc;
        w.Rd2 = cur; cur += p.efc; w.Ri2 = reinterpret_cast<uint32_t*>(cur); cur += p.efc;
        w.Sd = cur; cur += p.sc; w.Si = reinterpret_cast<uint32_t*>(cur); cur += p.sc;
        w.Sd2 = cur; cur += p.sc; w.Si2 = reinterpret_cast<uint32_t*>(cur); cur += p.sc;
        w.Bd = cur; cur += BATCH; w.Bi = reinterpret_cast<uint32_t*>(cur); cur += BATCH;
        w.Cd = cur; cur += BATCH; w.Ci = reinterpret_cast<uint32_t*>(cur); cur += BATCH;
        w.vc = reinterpret_cast<uint16_t*>(cur); cur += ((1 << p.vc_log2) + 1) / 2;
        w.xs = reinterpret_cast<uint32_t*>(cur); cur += (1 << p.xs_log2);
        w.ltomb = reinterpret_cast<uint32_t*>(cur); cur += MAX_LOCAL_TOMB;
        w.ub = p.uniq ? p.uniq + (uint64_t)q * p.uniq_words : nullptr;
        knn_one<METRIC, PQ>(p, w, q);
    }
}

// Small unfiltered batches (wv_search_batch under ~64 queries: the batcher's
// single callers): one 4-wave workgroup per query, wave 0 running the search
// of wv_hnsw_kernel's register path and waves 1..3 its distance batches
// (wg_dist).  Same expansion order and results, bit for bit.
template <int METRIC, int NR>
__global__ __launch_bounds__(256) void wv_hnsw_wg_kernel(HnswParams p) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x;
    if (q >= p.nq) return;
    WaveState w;
    reg_wave_state(p, lds, w);
    w.wg_nb = reinterpret_cast<volatile int*>(lds + p.per_wave_words);
    w.ub = p.uniq ? p.uniq + (uint64_t)q * p.uniq_words : nullptr;
    if (wave == 0) {
        knn_one_reg<METRIC, false, NR>(p, w, q);
        if (lane == 0) *w.wg_nb = -1;
        __syncthreads();
    } else {
        wg_helper<METRIC>(p, w, wave, lane);
    }
}

// ===========================================================================
// Side-register path (round 6): filtered, tombstoned or nil-node searches with
// ef <= 128.  The results R live in registers as on the unfiltered register
// path (search_layer_reg); the side candidates S -- traversed but ineligible
// (filtered out at layer 0, tombstoned, or a nil node the descent tombstoned:
// search.go:282-298, :496-507) -- live unsorted in an LDS array of
// side_rows x 64 entries, appended batch by batch, with the minimum key and
// its position kept wave-uniform: a side pop moves the last entry into the
// popped one's place and rescans (n / 64 LDS reads per lane and one DPP
// reduction).
//
// Layer 0 (EV): the visited list is exact -- a per-query bitmap in HBM behind
// the LDS cache: a neighbour the cache misses is claimed by an atomic OR
// (search.go:256-264), so every node is evaluated and queued at most once, as
// in the reference (a selective list traverses ~15-25k nodes a query, far past
// any LDS cache: the lossy cache alone re-evaluated 1.5x and filled S with
// copies).  S never holds a copy, so no expanded set is needed.  S keeps its
// smallest keys in LDS and the rest in a per-query spill in HBM: every LDS key
// is <= the bound U < every spilled key, so the LDS minimum is S's minimum
// while LDS is not empty; a full LDS array first drops its dead entries
// (d > worst once R is full: never expandable, :213-215), then moves the keys
// above a sampled median to the spill (U drops to it); an empty LDS array
// with a live spill takes back the spill's smallest keys (U rises).  Only a
// spill past spill_cap ends in status != 0 (the exact fallback).
//
// Upper levels (!EV, ef = 1, tombstones / nil nodes only): the lossy LDS
// cache, the expanded set X (exact, open addressing) and, when S is full, the
// smallest dropped key: exact while every pop is below it and the search ends
// with it above worst; otherwise status != 0.

// one step of a (d, id) minimum by DPP (no LDS): lanes whose source is out
// of range or masked take the identity
template <int CTRL, int RM>
__device__ __forceinline__ void kmin_step(float& d, uint32_t& i) {
    const float od = __uint_as_float((uint32_t)__builtin_amdgcn_update_dpp(
        (int)__float_as_uint(FLT_MAX), (int)__float_as_uint(d), CTRL, RM, 0xF, false));
    const uint32_t oi = (uint32_t)__builtin_amdgcn_update_dpp((int)WV_NIL, (int)i, CTRL, RM, 0xF, false);
    const bool lt = key_less_nb(od, oi, d, i);
    d = lt ? od : d;
    i = lt ? oi : i;
}
// (d, id) minimum over the wave (row_shr 1/2/4/8 within rows, row_bcast
// 15/31 across them, lane 63 read out): every lane returns it
__device__ __forceinline__ void wave_min_key(float& d, uint32_t& i) {
    kmin_step<0x111, 0xF>(d, i);
    kmin_step<0x112, 0xF>(d, i);
    kmin_step<0x114, 0xF>(d, i);
    kmin_step<0x118, 0xF>(d, i);
    kmin_step<0x142, 0xA>(d, i);
    kmin_step<0x143, 0xC>(d, i);
    d = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(d), 63));
    i = (uint32_t)__builtin_amdgcn_readlane((int)i, 63);
}

// the key of rank r among the wave's 64 distinct (d, id) keys (one per lane)
__device__ __forceinline__ void wave_rank_key(float d, uint32_t i, int r, float& od, uint32_t& oi) {
    int rank = 0;
    for (int t = 0; t < 64; ++t) {
        const float td = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(d), t));
        const uint32_t ti = (uint32_t)__builtin_amdgcn_readlane((int)i, t);
        rank += key_less_nb(td, ti, d, i) ? 1 : 0;
    }
    const uint64_t m = __ballot(rank == r);
    const int src = m ? __builtin_ctzll(m) : 0;
    od = __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(d), src));
    oi = (uint32_t)__builtin_amdgcn_readlane((int)i, src);
}

template <int METRIC, int NR, int RPG, bool EV>
__device__ __forceinline__ void search_layer_side(const HnswParams& p, WaveState& w, int level, int ef, uint32_t ep,
                                                  float epd, const uint64_t* allow, int nlt, uint32_t* vb,
                                                  uint32_t* sp, float (&rd)[NR], uint32_t (&ri)[NR], int& Rl,
                                                  int& status, uint32_t& n_dist, uint32_t& n_exp, uint32_t& n_miss) {
    static_assert(NR == 1 || NR == 2, "64 or 128 results per wave");
    const int lane = threadIdx.x & 63;
    const int VC = 1 << p.vc_log2;
    const int XS = EV ? 0 : 1 << p.xs_log2;
    const int SC = 64 * p.side_rows;
    float* Sd = w.Sd;
    uint32_t* Si = w.Si;
    for (int i = lane; i < VC; i += 64) w.vc[i] = VC_EMPTY;
    if (!EV)
        for (int i = lane; i < XS; i += 64) w.xs[i] = WV_NIL;
    wave_sync();
    if (lane == 0) {
        const uint32_t he = vc_hash(p, ep);
        w.vc[vc_slot(p, he)] = vc_tag(p, he);
        if (EV) atomicOr(vb + (ep >> 5), 1u << (ep & 31));   // visitedList.Visit(ep) (:338)
    }
    auto eligible = [&](uint32_t id) -> bool {
        if (p.tomb && bit_test(p.tomb, p.tomb_nbits, id)) return false;
        for (int t = 0; t < nlt; ++t)
            if (w.ltomb[t] == id) return false;
        if (level == 0 && allow && !bit_test(allow, p.allow_nbits, id)) return false;
        return true;
    };
    // insertViableEntrypointsAsCandidatesAndResults (search.go:329-353)
    const bool ep_ok = eligible(ep);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        rd[r] = ep_ok && lane == 0 && r == 0 ? epd : FLT_MAX;
        ri[r] = ep_ok && lane == 0 && r == 0 ? ep : WV_NIL;
    }
    Rl = ep_ok ? 1 : 0;
    // currentWorstResultDistanceToFloat (:355-377)
    float worst = ep_ok ? epd : FLT_MAX;
    // S in LDS: n entries, minimum (smd, smi) at spos.  !EV: xd/xi the
    // smallest dropped key.  EV: gcnt spilled entries in sp, every one keyed
    // above (ud, ui) >= every LDS key (while gcnt > 0)
    int n = 0, spos = 0, gcnt = 0;
    float smd = FLT_MAX, xd = FLT_MAX, ud = FLT_MAX;
    uint32_t smi = WV_NIL, xi = WV_NIL, ui = WV_NIL;
    if (!ep_ok) {
        if (lane == 0) { Sd[0] = epd; Si[0] = ep; }
        n = 1; smd = epd; smi = ep;
    }
    // rescan S for its minimum (after a pop or a shed)
    auto rescan = [&]() {
        float bd_ = FLT_MAX;
        uint32_t bi_ = WV_NIL;
        int bp = 0;
        for (int j = lane; j < n; j += 64) {
            const float d = Sd[j];
            const uint32_t id = Si[j];
            const bool lt = key_less_nb(d, id, bd_, bi_);
            bd_ = lt ? d : bd_;
            bi_ = lt ? id : bi_;
            bp = lt ? j : bp;
        }
        float md = bd_;
        uint32_t mi = bi_;
        wave_min_key(md, mi);
        const uint64_t wm = __ballot(bd_ == md && bi_ == mi);
        spos = wm ? __builtin_amdgcn_readlane(bp, __builtin_ctzll(wm)) : 0;
        smd = md;
        smi = mi;
    };
    auto dead = [&](float d) { return Rl >= ef && d > worst; };
    // EV: drop the spill's dead entries in place (before it would overflow;
    // a chunk's writes land at or below its reads)
    auto compact_spill = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        int m = 0;
        for (int j0 = 0; j0 < gcnt; j0 += 64) {
            const int j = j0 + lane;
            const float d = j < gcnt ? __uint_as_float(sp[2 * j]) : FLT_MAX;
            const uint32_t id = j < gcnt ? sp[2 * j + 1] : WV_NIL;
            const bool live = j < gcnt && !dead(d);
            const uint64_t lm = __ballot(live);
            if (live) { sp[2 * (m + mbcnt64(lm))] = __float_as_uint(d); sp[2 * (m + mbcnt64(lm)) + 1] = id; }
            m += __popcll(lm);
        }
        gcnt = m;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    };
    // EV: move the LDS keys above a sampled median (n >= 64) to the spill and
    // drop the dead ones; U falls to that median
    auto split = [&]() {
        const int idx = (int)(((uint32_t)lane * (uint32_t)n) >> 6);
        float md;
        uint32_t mi;
        wave_rank_key(Sd[idx], Si[idx], 31, md, mi);
        if (gcnt + n > p.spill_cap) compact_spill();
        int k = 0;
        for (int j0 = 0; j0 < n; j0 += 64) {
            const int j = j0 + lane;
            const float d = j < n ? Sd[j] : FLT_MAX;
            const uint32_t id = j < n ? Si[j] : WV_NIL;
            const bool live = j < n && !dead(d);
            const bool stay = live && !key_less_nb(md, mi, d, id);
            const bool mv = live && !stay;
            const uint64_t lm = __ballot(stay), sm = __ballot(mv);
            wave_sync();
            if (stay) { Sd[k + mbcnt64(lm)] = d; Si[k + mbcnt64(lm)] = id; }
            if (mv) {
                const int g = gcnt + mbcnt64(sm);
                if (g < p.spill_cap) { sp[2 * g] = __float_as_uint(d); sp[2 * g + 1] = id; }
            }
            k += __popcll(lm);
            gcnt += __popcll(sm);
            wave_sync();
        }
        if (gcnt > p.spill_cap) status |= 2;
        n = k;
        ud = md;
        ui = mi;
        rescan();
    };
    // EV: LDS is empty and the spill is not -- take back its smallest live keys
    auto refill = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // (the wave's own spill stores)
        // drop the dead, compact the spill in place (a chunk's writes land at
        // or below its reads) and copy the live ones to LDS while they fit
        int m = 0;
        for (int j0 = 0; j0 < gcnt; j0 += 64) {
            const int j = j0 + lane;
            const float d = j < gcnt ? __uint_as_float(sp[2 * j]) : FLT_MAX;
            const uint32_t id = j < gcnt ? sp[2 * j + 1] : WV_NIL;
            const bool live = j < gcnt && !dead(d);
            const uint64_t lm = __ballot(live);
            const int o = m + mbcnt64(lm);
            if (live) {
                sp[2 * o] = __float_as_uint(d);
                sp[2 * o + 1] = id;
                if (o < SC) { Sd[o] = d; Si[o] = id; }
            }
            m += __popcll(lm);
        }
        gcnt = m;
        wave_sync();
        if (m <= SC) {   // all of it fits: the spill is empty again
            n = m;
            gcnt = 0;
            if (n) rescan();
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        // a bound whose keys fill about half the array: 64 keys sampled
        // evenly among the spilled keys at or below the current bound (into
        // the idle batch arrays), the one of the target rank taken, its keys
        // counted exactly; a bound that still admits too many narrows the
        // next round's sample to its own keys (each round ~64x fewer)
        float bd = FLT_MAX;
        uint32_t bi = WV_NIL;
        bool found = false;
        int cq = m;   // keys at or below (bd, bi)
        for (int round = 0; round < 4 && !found; ++round) {
            const int stride = max(1, cq / 64);
            int t = 0;
            for (int j0 = 0; j0 < m; j0 += 64) {
                const int j = j0 + lane;
                const float d = j < m ? __uint_as_float(sp[2 * j]) : FLT_MAX;
                const uint32_t id = j < m ? sp[2 * j + 1] : WV_NIL;
                const bool qual = j < m && (round == 0 || !key_less_nb(bd, bi, d, id));
                const uint64_t qm = __ballot(qual);
                const int ti = t + mbcnt64(qm);
                if (qual && ti % stride == 0 && ti / stride < 64) { w.Bd[ti / stride] = d; w.Bi[ti / stride] = id; }
                t += __popcll(qm);
            }
            wave_sync();
            const int ns_ = min(64, (cq + stride - 1) / stride);
            const float sd_ = lane < ns_ ? w.Bd[lane] : FLT_MAX;
            const uint32_t si_ = lane < ns_ ? w.Bi[lane] : (WV_NIL - 1 - (uint32_t)lane);   // (distinct fillers, ranked last)
            wave_sync();
            const int r = min(ns_ - 1, max(0, (ns_ * (SC / 2)) / cq - 1));
            float nd;
            uint32_t ni;
            wave_rank_key(sd_, si_, r, nd, ni);
            int c = 0;
            for (int j0 = 0; j0 < m; j0 += 64) {
                const int j = j0 + lane;
                const bool in = j < m && !key_less_nb(nd, ni, __uint_as_float(sp[2 * j]), sp[2 * j + 1]);
                c += __popcll(__ballot(in));
            }
            bd = nd;
            bi = ni;
            cq = c;
            found = c <= SC;
        }
        if (!found) { status |= 2; return; }
        int k = 0, g = 0;
        for (int j0 = 0; j0 < m; j0 += 64) {
            const int j = j0 + lane;
            const float d = j < m ? __uint_as_float(sp[2 * j]) : FLT_MAX;
            const uint32_t id = j < m ? sp[2 * j + 1] : WV_NIL;
            const bool in = j < m && !key_less_nb(bd, bi, d, id);
            const bool out = j < m && !in;
            const uint64_t lm = __ballot(in), om = __ballot(out);
            if (in) { Sd[k + mbcnt64(lm)] = d; Si[k + mbcnt64(lm)] = id; }
            if (out) { sp[2 * (g + mbcnt64(om))] = __float_as_uint(d); sp[2 * (g + mbcnt64(om)) + 1] = id; }
            k += __popcll(lm);
            g += __popcll(om);
        }
        wave_sync();
        n = k;
        gcnt = g;
        ud = bd;
        ui = bi;
        rescan();
    };
    wave_sync();
    const uint32_t* nbr_base;
    int deg;
    for (;;) {
        // ---- pop: the first unexpanded result vs the side minimum ----
        int ridx = -1;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint64_t um = __ballot(64 * r + lane < Rl && !(ri[r] & WV_FLAG));
            if (ridx < 0 && um) ridx = 64 * r + __builtin_ctzll(um);
        }
        if (EV && n == 0 && gcnt > 0) {
            // S's minimum is in the spill (above U): a result candidate at or
            // below U comes first; otherwise take the spill's smallest back
            bool r_first = false;
            if (ridx >= 0)
                r_first = !key_less(ud, ui, reg_entry_d<NR>(rd, ridx), reg_entry_i<NR>(ri, ridx) & WV_IDMASK);
            if (!r_first) {
                refill();
                if (status) break;
                continue;
            }
        }
        if (ridx < 0 && n == 0) {   // candidates exhausted
            if (!EV && xi != WV_NIL) status |= 1;   // (a dropped one was still to be expanded)
            break;
        }
        float cd = smd;
        uint32_t cid = smi;
        bool fromR = false;
        if (ridx >= 0) {
            const float rdv = reg_entry_d<NR>(rd, ridx);
            const uint32_t riv = reg_entry_i<NR>(ri, ridx) & WV_IDMASK;
            if (n == 0 || key_less(rdv, riv, smd, smi)) { cd = rdv; cid = riv; fromR = true; }
        }
        if (cd > worst) {   // :213-215
            if (!EV && xi != WV_NIL && !(xd > worst)) status |= 1;
            break;
        }
        if (!EV && xi != WV_NIL && key_less(xd, xi, cd, cid)) { status |= 1; break; }
        if (fromR) {
#pragma unroll
            for (int r = 0; r < NR; ++r)
                if (64 * r + lane == ridx) ri[r] |= WV_FLAG;
        } else {
            // remove it: the last entry takes its place
            --n;
            if (lane == 0 && spos != n) { Sd[spos] = Sd[n]; Si[spos] = Si[n]; }
            wave_sync();
            rescan();
            if (!EV) {
                // X: expanded once (search.go:256-264 by way of the exact set)
                const uint32_t h0 = hash32(cid) >> (32 - p.xs_log2);
                bool dup = false, placed = false;
                for (int b = 0; b < XS; b += 64) {
                    const uint32_t slot = (h0 + b + lane) & (XS - 1);
                    const uint32_t v = w.xs[slot];
                    const uint64_t fm = __ballot(v == cid), em = __ballot(v == WV_NIL);
                    const int fe = em ? __builtin_ctzll(em) : 64;
                    if (fm && __builtin_ctzll(fm) < fe) { dup = true; break; }
                    if (em) {
                        if (lane == fe) w.xs[slot] = cid;
                        placed = true;
                        break;
                    }
                }
                if (dup) continue;
                if (!placed) { status |= 2; break; }
            }
        }
        uint32_t pre0 = WV_NIL, pre1 = WV_NIL;
        if (level == 0) {
            nbr_base = p.layer0 + (uint64_t)cid * p.deg0;
            deg = p.deg0;
            if (lane < deg) pre0 = nbr_base[lane];
            if (64 + lane < deg) pre1 = nbr_base[64 + lane];
            if (p.levels[cid] < 0) continue;   // :217-234
        } else {
            if (p.levels[cid] < level) continue;
            const uint32_t row = p.upper_row[cid];
            nbr_base = p.upper + ((uint64_t)row * p.upper_levels + (level - 1)) * p.degU;
            deg = p.degU;
        }
        n_exp++;
        for (int c0 = 0; c0 < deg; c0 += BATCH) {
            uint32_t id0 = WV_NIL, id1 = WV_NIL;
            if (level == 0 && c0 == 0) {
                id0 = pre0;
                id1 = pre1;
            } else {
                if (c0 + lane < deg) id0 = nbr_base[c0 + lane];
                if (c0 + 64 + lane < deg) id1 = nbr_base[c0 + 64 + lane];
            }
            bool v0 = id0 != WV_NIL && id0 < p.N;
            bool v1 = id1 != WV_NIL && id1 < p.N;
            const uint32_t e0 = vc_hash(p, id0), e1 = vc_hash(p, id1);
            const uint32_t h0 = v0 ? vc_slot(p, e0) : 0, h1 = v1 ? vc_slot(p, e1) : 0;
            const uint16_t t0 = vc_tag(p, e0), t1 = vc_tag(p, e1);
            if (v0 && w.vc[h0] == t0) v0 = false;
            if (v1 && w.vc[h1] == t1) v1 = false;
            wave_sync();
            if (v0) w.vc[h0] = t0;
            if (v1) w.vc[h1] = t1;
            // eligibility words (tombstones, the allow list at layer 0): LDS-
            // DMA loads issued now, beside the claims / row loads, read after
            // the distances -- no VGPRs held across them and no branch on
            // them before (that would wait: one more round trip an expansion)
            const uint32_t eb = __builtin_amdgcn_readfirstlane(lds_addr(w.ew));
            const bool use_al = level == 0 && allow;
            if (p.tomb) {
                if (v0 && id0 < p.tomb_nbits) glds4(reinterpret_cast<const uint32_t*>(p.tomb) + (id0 >> 5), eb);
                if (v1 && id1 < p.tomb_nbits) glds4(reinterpret_cast<const uint32_t*>(p.tomb) + (id1 >> 5), eb + 256);
            }
            if (use_al) {
                if (v0 && id0 < p.allow_nbits) glds4(reinterpret_cast<const uint32_t*>(allow) + (id0 >> 5), eb + 512);
                if (v1 && id1 < p.allow_nbits) glds4(reinterpret_cast<const uint32_t*>(allow) + (id1 >> 5), eb + 768);
            }
            // (EV spec, an A/B switch: the rows of every cache miss are
            // loaded beside the claims, the ones already visited dropped
            // after -- one round trip less, more rows)
            const bool spec = EV && p.ev_spec;
            bool f0 = true, f1 = true;
            if (EV) {
                // the cache's misses claim their bit: a node another expansion
                // evaluated (the cache forgot it) is skipped, as the exact
                // visited list skips it
                n_miss += (uint32_t)(__popcll(__ballot(v0)) + __popcll(__ballot(v1)));
                if (v0) {
                    const uint32_t b = 1u << (id0 & 31);
                    f0 = !(atomicOr(vb + (id0 >> 5), b) & b);
                }
                if (v1) {
                    const uint32_t b = 1u << (id1 & 31);
                    f1 = !(atomicOr(vb + (id1 >> 5), b) & b);
                }
                if (!spec) {
                    v0 = v0 && f0;
                    v1 = v1 && f1;
                }
            }
            const uint64_t m0 = __ballot(v0), m1 = __ballot(v1);
            const int n0 = __popcll(m0);
            const int nb = n0 + __popcll(m1);
            if (v0) w.Bi[mbcnt64(m0)] = id0;
            if (v1) w.Bi[n0 + mbcnt64(m1)] = id1;
            wave_sync();
            if (nb == 0) continue;
            if (p.wg_helpers) {
                wg_dist<METRIC>(p, w, nb, lane);
            } else {
                for (int base = 0; base < nb; base += 8 * RPG)
                    exact_dist_rows<METRIC, RPG, true>(w.qv, p.X, p.ldx, p.D, w.Bi + base, nb - base, w.Bd + base,
                                                       lane);
            }
            n_dist += (uint32_t)nb;
            wave_sync();
            float bd_spec[2] = {FLT_MAX, FLT_MAX};
            if (spec) {   // (distances by batch slot, then only the claimed ones go on)
                bd_spec[0] = v0 ? w.Bd[mbcnt64(m0)] : FLT_MAX;
                bd_spec[1] = v1 ? w.Bd[n0 + mbcnt64(m1)] : FLT_MAX;
                v0 = v0 && f0;
                v1 = v1 && f1;
            }
            // ---- keep test against the batch's starting state (search.go:282),
            // on the neighbours' own lanes (batch order = lane order, id0s
            // first): eligible keys into R one by one, ineligible ones to S ----
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the eligibility words landed)
            auto el_of = [&](bool v, uint32_t id, int h) -> bool {
                const uint32_t tw = p.tomb && id < p.tomb_nbits ? w.ew[64 * h + lane] : 0u;
                const uint32_t aw = !use_al ? ~0u : id < p.allow_nbits ? w.ew[128 + 64 * h + lane] : 0u;
                bool e = v && !((tw >> (id & 31)) & 1u) && ((aw >> (id & 31)) & 1u);
                for (int t = 0; t < nlt; ++t) e = e && w.ltomb[t] != id;
                return e;
            };
            const bool el0 = el_of(v0, id0, 0), el1 = el_of(v1, id1, 1);
            float bd[2];
            uint32_t bi[2];
            uint64_t kmask[2], smask[2];
            bd[0] = spec ? bd_spec[0] : v0 ? w.Bd[mbcnt64(m0)] : FLT_MAX;
            bd[1] = spec ? bd_spec[1] : v1 ? w.Bd[n0 + mbcnt64(m1)] : FLT_MAX;
            bi[0] = id0;
            bi[1] = id1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const bool keep = (h ? v1 : v0) && (bd[h] < worst || Rl < ef);
                const bool el = h ? el1 : el0;
                kmask[h] = __ballot(keep && el);
                smask[h] = __ballot(keep && !el);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint64_t km = kmask[h];
                while (km) {
                    const int src = __builtin_ctzll(km);
                    km &= km - 1;
                    const float d = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(bd[h]), src));
                    const uint32_t id = (uint32_t)__builtin_amdgcn_readlane(bi[h], src);
                    int pos = 0;
#pragma unroll
                    for (int r = 0; r < NR; ++r)
                        pos += __popcll(__ballot((64 * r + lane < Rl) & key_less_nb(rd[r], ri[r] & WV_IDMASK, d, id)));
                    if (pos >= ef) continue;
                    if (pos < Rl && reg_entry_d<NR>(rd, pos) == d && (reg_entry_i<NR>(ri, pos) & WV_IDMASK) == id)
                        continue;   // already a result (a neighbour the visited cache forgot)
                    float sd[NR];
                    uint32_t si[NR];
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        sd[r] = wave_shr1(rd[r]);
                        si[r] = wave_shr1(ri[r]);
                        if (r > 0) {
                            const float cdv = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rd[r - 1]), 63));
                            const uint32_t civ = (uint32_t)__builtin_amdgcn_readlane(ri[r - 1], 63);
                            if (lane == 0) { sd[r] = cdv; si[r] = civ; }
                        }
                    }
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        const int e = 64 * r + lane;
                        if (e > pos) { rd[r] = sd[r]; ri[r] = si[r]; }
                        if (e == pos) { rd[r] = d; ri[r] = id; }
                    }
                    Rl = min(Rl + 1, ef);
                    worst = reg_entry_d<NR>(rd, Rl - 1);
                }
            }
            // ---- the ineligible keys to S (EV: the ones already dead against
            // the batch's final worst are never expandable: not queued) ----
            if (EV) {
                smask[0] &= __ballot(!dead(bd[0]));
                smask[1] &= __ballot(!dead(bd[1]));
            }
            if ((smask[0] | smask[1]) == 0) continue;
            if (EV) {
                // each new key to LDS (at or below U) or to the spill; a full
                // array drops its dead, then splits
                uint64_t lmask[2];
                bool shed = false;
                for (;;) {
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        lmask[h] = smask[h] & __ballot(gcnt == 0 || !key_less_nb(ud, ui, bd[h], bi[h]));
                    const int nl = __popcll(lmask[0]) + __popcll(lmask[1]);
                    if (n + nl <= SC) break;
                    if (!shed && Rl >= ef) {
                        int k = 0;
                        for (int j0 = 0; j0 < n; j0 += 64) {
                            const int j = j0 + lane;
                            const float d = j < n ? Sd[j] : FLT_MAX;
                            const uint32_t id = j < n ? Si[j] : WV_NIL;
                            const bool live = j < n && !dead(d);
                            const uint64_t lm = __ballot(live);
                            wave_sync();
                            if (live) { Sd[k + mbcnt64(lm)] = d; Si[k + mbcnt64(lm)] = id; }
                            k += __popcll(lm);
                            wave_sync();
                        }
                        n = k;
                        rescan();
                        shed = true;
                        continue;
                    }
                    split();
                    if (status) break;
                }
                if (status) break;
                const uint64_t g0 = smask[0] & ~lmask[0], g1 = smask[1] & ~lmask[1];
                if (g0 | g1) {
                    const int gn0 = __popcll(g0);
                    if (gcnt + gn0 + __popcll(g1) > p.spill_cap) compact_spill();
                    if ((g0 >> lane) & 1) {
                        const int g = gcnt + mbcnt64(g0);
                        if (g < p.spill_cap) { sp[2 * g] = __float_as_uint(bd[0]); sp[2 * g + 1] = bi[0]; }
                    }
                    if ((g1 >> lane) & 1) {
                        const int g = gcnt + gn0 + mbcnt64(g1);
                        if (g < p.spill_cap) { sp[2 * g] = __float_as_uint(bd[1]); sp[2 * g + 1] = bi[1]; }
                    }
                    gcnt += gn0 + __popcll(g1);
                    if (gcnt > p.spill_cap) { status |= 2; break; }
                }
                smask[0] = lmask[0];
                smask[1] = lmask[1];
                if ((smask[0] | smask[1]) == 0) continue;
            }
            const int ns0 = __popcll(smask[0]);
            const int ns = ns0 + __popcll(smask[1]);
            if (!EV && n + ns > SC && Rl >= ef) {
                // shed the dead (d > worst), in place: a chunk's reads come
                // before its writes, which land at or below them
                int k = 0;
                for (int j0 = 0; j0 < n; j0 += 64) {
                    const int j = j0 + lane;
                    const float d = j < n ? Sd[j] : FLT_MAX;
                    const uint32_t id = j < n ? Si[j] : WV_NIL;
                    const bool live = j < n && !(d > worst);
                    const uint64_t lm = __ballot(live);
                    wave_sync();
                    if (live) { Sd[k + mbcnt64(lm)] = d; Si[k + mbcnt64(lm)] = id; }
                    k += __popcll(lm);
                    wave_sync();
                }
                n = k;
                rescan();
            }
            const int fit = min(ns, SC - n);
            float nd_ = FLT_MAX, xd_ = FLT_MAX;
            uint32_t ni_ = WV_NIL, xi_ = WV_NIL;
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if ((smask[h] >> lane) & 1) {
                    const int r = (h ? ns0 : 0) + mbcnt64(smask[h]);
                    if (r < fit) {
                        Sd[n + r] = bd[h];
                        Si[n + r] = bi[h];
                        if (key_less(bd[h], bi[h], nd_, ni_)) { nd_ = bd[h]; ni_ = bi[h]; }
                    } else if (key_less(bd[h], bi[h], xd_, xi_)) {
                        xd_ = bd[h]; xi_ = bi[h];
                    }
                }
            wave_min_key(nd_, ni_);
            if (n == 0 || key_less(nd_, ni_, smd, smi)) {
                smd = nd_;
                smi = ni_;
                const uint64_t pm0 = __ballot(((smask[0] >> lane) & 1) && bd[0] == nd_ && bi[0] == ni_);
                const uint64_t pm1 = __ballot(((smask[1] >> lane) & 1) && bd[1] == nd_ && bi[1] == ni_);
                spos = pm0 ? n + __popcll(smask[0] & ((1ull << __builtin_ctzll(pm0)) - 1))
                           : n + ns0 + __popcll(smask[1] & ((1ull << __builtin_ctzll(pm1)) - 1));
            }
            if (!EV && fit < ns) {
                wave_min_key(xd_, xi_);
                if (key_less(xd_, xi_, xd, xi)) { xd = xd_; xi = xi_; }
            }
            n += fit;
            wave_sync();
        }
        if (status) break;
    }
}

template <int METRIC, int NR, int RPG, bool EV0>
__device__ __forceinline__ int knn_one_side(const HnswParams& p, WaveState& w, int q) {
    const int lane = threadIdx.x & 63;
    const int g = lane & 7;
    for (int i = lane; i < p.dpad; i += 64) w.qv[i] = i < p.D ? p.Q[(uint64_t)q * p.ldq + i] : 0.f;
    wave_sync();
    const uint64_t* allow = p.allow ? p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0) : nullptr;
    uint32_t* vb = EV0 ? p.vbits + (uint64_t)q * p.vwords : nullptr;
    if (EV0 && !p.vb_host_clear) {
        // this query's layer-0 visited bitmap starts empty (cleared here,
        // overlapped with the other waves' searches; the fence orders the
        // clear before the claims)
        uint4* v4 = reinterpret_cast<uint4*>(vb);
        const uint64_t n4 = p.vwords / 4;
        for (uint64_t i = lane; i < n4; i += 64) v4[i] = make_uint4(0u, 0u, 0u, 0u);
        for (uint64_t i = 4 * n4 + lane; i < p.vwords; i += 64) vb[i] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    uint32_t* sp = p.spill + 2 * (uint64_t)q * p.spill_cap;
    int status = 0, nlt = 0;
    uint32_t n_dist = 0, n_exp = 0, n_miss = 0;
    uint32_t ep = p.entrypoint;
    float epd = __shfl(exact_dist_group8<METRIC>(w.qv, p.X + (uint64_t)ep * p.ldx, p.D, g), 0, 64);
    n_dist++;
    float rd[NR];
    uint32_t ri[NR];
    int Rl = 0;
    // greedy descent, levels max..1 with ef = 1 (search.go:479-521): a nil
    // result is tombstoned for the rest of the search (:496-507)
    for (int level = p.max_level; level >= 1 && !status; --level) {
        search_layer_side<METRIC, NR, RPG, false>(p, w, level, 1, ep, epd, nullptr, nlt, vb, sp, rd, ri, Rl, status,
                                                  n_dist, n_exp, n_miss);
        if (Rl > 0) {
            const uint32_t cid = (uint32_t)__builtin_amdgcn_readlane(ri[0], 0) & WV_IDMASK;
            if (p.levels[cid] < 0) {
                if (nlt < MAX_LOCAL_TOMB) {
                    if (lane == 0) w.ltomb[nlt] = cid;
                    nlt++;
                }
                wave_sync();
            } else {
                ep = cid;
                epd = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(rd[0]), 0));
            }
        }
    }
    if (!status)
        search_layer_side<METRIC, NR, RPG, EV0>(p, w, 0, p.ef, ep, epd, allow, nlt, vb, sp, rd, ri, Rl, status, n_dist,
                                                n_exp, n_miss);
    const int n = status ? 0 : min(Rl, p.k);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int e = 64 * r + lane;
        if (e < n) {
            p.out_ids[(uint64_t)q * p.k + e] = p.id_base + (ri[r] & WV_IDMASK);
            p.out_d[(uint64_t)q * p.k + e] = rd[r];
        }
    }
    if (lane == 0) {
        p.out_n[q] = n;
        p.status[q] = status;
        if (p.counters) { p.counters[2 * q] = n_dist; p.counters[2 * q + 1] = n_exp; }
        if (status && p.side_acc) atomicAdd(p.side_acc + (EV0 ? 3 : 4), 1ull);
        if (EV0 && p.side_acc) atomicAdd(p.side_acc + 5, (unsigned long long)n_miss);   // (cache misses claimed)
    }
    return status;
}

// LDS per wave: query, batch, side array, X, local tombstones, visited cache
__device__ __forceinline__ void side_wave_state(const HnswParams& p, float* cur, WaveState& w) {
    w.qv = cur; cur += p.dpad;
    w.Bd = cur; cur += BATCH; w.Bi = reinterpret_cast<uint32_t*>(cur); cur += BATCH;
    w.Sd = cur; cur += 64 * p.side_rows; w.Si = reinterpret_cast<uint32_t*>(cur); cur += 64 * p.side_rows;
    w.xs = reinterpret_cast<uint32_t*>(cur); cur += (1 << p.xs_log2);
    w.ltomb = reinterpret_cast<uint32_t*>(cur); cur += MAX_LOCAL_TOMB;
    w.ew = reinterpret_cast<uint32_t*>(cur); cur += 256;
    w.vc = reinterpret_cast<uint16_t*>(cur);
}

// WPS: waves per SIMD the register allocation targets.  EV0: layer 0 with the
// exact visited bitmap (selective lists); otherwise the lossy cache + X, and
// a query whose side state overflows is re-run with EV0 (p.redo).
template <int METRIC, int NR, int RPG, int WPS, bool EV0>
__global__ __launch_bounds__(256, WPS) void wv_hnsw_side_kernel(HnswParams p) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6;
    const int q = blockIdx.x * (blockDim.x >> 6) + wave;
    if (q >= p.nq) return;
    if (p.redo && p.redo[q] == 0) return;   // (second pass: this query completed)
    WaveState w{};
    side_wave_state(p, lds + (uint64_t)wave * p.per_wave_words, w);
    knn_one_side<METRIC, NR, RPG, EV0>(p, w, q);
}

// Small batches (the batcher's callers): one 4-wave workgroup per query, wave
// 0 running the side search and waves 1..3 its distance batches (wg_dist,
// the barrier invariant above it).  Same expansion order and results.
template <int METRIC, int NR, bool EV0>
__global__ __launch_bounds__(256) void wv_hnsw_side_wg_kernel(HnswParams p) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x;
    if (q >= p.nq) return;
    if (p.redo && p.redo[q] == 0) return;   // (uniform over the workgroup)
    WaveState w{};
    side_wave_state(p, lds, w);
    w.wg_nb = reinterpret_cast<volatile int*>(lds + p.per_wave_words);
    if (wave == 0) {
        // (a lossy first pass that overflowed re-runs in a second launch: an
        // in-kernel re-run with the exact visited bitmap doubled the code and
        // took a lone tombstoned query 399 -> 509 us)
        knn_one_side<METRIC, NR, 4, EV0>(p, w, q);
        if (lane == 0) *w.wg_nb = -1;
        __syncthreads();
    } else {
        wg_helper<METRIC>(p, w, wave, lane);
    }
}

// ===========================================================================
// GPU graph construction -- insert.go:103-217 in batches.
// A batch of new nodes is inserted against the graph of every node before it:
//   1. wv_build_search_kernel (one wave per node): findBestEntrypointForNode
//      (ef = 1 descent above the node's level, index.go:371-408), then
//      searchLayerByVector with efConstruction at each level <= min(level, top)
//      (neighbor_connections.go:71-84); the next level starts from the closest
//      result (the last of the selected neighbours, :119-128).
//   2. wv_build_select_kernel (one wave per node and level):
//      selectNeighborsHeuristic to M (heuristic.go:23-135), the node's own list
//      (setConnectionsAtLevel, farthest first as popped from the max-heap) and
//      one reverse-link request per neighbour.
//   3. requests sorted by (level, neighbour), stable, so each neighbour sees
//      its new links in batch order; wv_build_link_kernel (one wave per
//      neighbour): connectNeighborAtLevel (:134-209) -- append while below
//      capacity (2M at layer 0, M above), else re-prune the list plus the new
//      node with the heuristic.
// Members of one batch do not see each other (the graph they search is the
// one before the batch); batches grow with the graph (a fixed fraction).

template <int METRIC>
__device__ __forceinline__ void build_search_one(const BuildParams& b, WaveState& w, int slot) {
    Stamps ts;   // (not sampled in the build)
    const HnswParams& p = b.h;
    const int lane = threadIdx.x & 63;
    const int g = lane & 7;
    const uint64_t id = b.first + (uint64_t)slot;
    const int target = b.target[slot];
    for (int i = lane; i < p.dpad; i += 64) w.qv[i] = i < p.D ? p.X[id * p.ldx + i] : 0.f;
    wave_sync();
    int status = 0, nlt = 0;
    uint32_t n_dist = 0, n_exp = 0;
    uint32_t ep = p.entrypoint;
    float epd = __shfl(exact_dist_group8<METRIC>(w.qv, p.X + (uint64_t)ep * p.ldx, p.D, g), 0, 64);
    int Rl, Sh, Sl;
    for (int level = p.max_level; level > target; --level) {
        search_layer<METRIC>(p, w, level, 1, ep, epd, nullptr, Rl, Sh, Sl, status, nlt, n_dist, n_exp, ts);
        if (Rl > 0) { ep = w.Ri[0] & WV_IDMASK; epd = w.Rd[0]; }
    }
    for (int level = min(target, p.max_level); level >= 0; --level) {
        search_layer<METRIC>(p, w, level, p.ef, ep, epd, nullptr, Rl, Sh, Sl, status, nlt, n_dist, n_exp, ts);
        const uint64_t o = ((uint64_t)slot * b.lb + level) * p.ef;
        for (int i = lane; i < Rl; i += 64) {
            b.cand_i[o + i] = w.Ri[i] & WV_IDMASK;
            b.cand_d[o + i] = w.Rd[i];
        }
        if (lane == 0) b.cand_n[(uint64_t)slot * b.lb + level] = Rl;
        if (Rl > 0) { ep = w.Ri[0] & WV_IDMASK; epd = w.Rd[0]; }
        wave_sync();
    }
}

__global__ __launch_bounds__(256) void wv_build_search_kernel(BuildParams b) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6;
    const int slot = blockIdx.x * (blockDim.x >> 6) + wave;
    if (slot >= b.nb) return;
    const HnswParams& p = b.h;
    float* cur = lds + (uint64_t)wave * p.per_wave_words;
    WaveState w;
    w.ub = nullptr;
    w.qv = cur; cur += p.dpad;
    w.Rd = cur; cur += p.efc; w.Ri = reinterpret_cast<uint32_t*>(cur); cur += p.efc;
    w.Rd2 = cur; cur += p.efc; w.Ri2 = reinterpret_cast<uint32_t*>(cur); cur += p.efc;
    w.Sd = cur; cur += p.sc; w.Si = reinterpret_cast<uint32_t*>(cur); cur += p.sc;
    w.Sd2 = cur; cur += p.sc; w.Si2 = reinterpret_cast<uint32_t*>(cur); cur += p.sc;
    w.Bd = cur; cur += BATCH; w.Bi = reinterpret_cast<uint32_t*>(cur); cur += BATCH;
    w.Cd = cur; cur += BATCH; w.Ci = reinterpret_cast<uint32_t*>(cur); cur += BATCH;
    w.vc = reinterpret_cast<uint16_t*>(cur); cur += ((1 << p.vc_log2) + 1) / 2;
    w.xs = reinterpret_cast<uint32_t*>(cur); cur += (1 << p.xs_log2);
    w.ltomb = reinterpret_cast<uint32_t*>(cur);
    if (p.metric == WV_METRIC_L2) build_search_one<WV_METRIC_L2>(b, w, slot);
    else if (p.metric == WV_METRIC_DOT) build_search_one<WV_METRIC_DOT>(b, w, slot);
    else build_search_one<WV_METRIC_COSINE>(b, w, slot);
}

// selectNeighborsHeuristic (heuristic.go:23-135) over n candidates sorted
// ascending (ci/cd in LDS): keep a candidate unless an already kept one is
// closer to it than the query is (SingleDist(cand, kept) < dist(cand, query));
// at most mx kept, in ascending order, into sel.  Returns the count.
template <int METRIC>
__device__ int heuristic_select(const HnswParams& p, const uint32_t* ci, const float* cd, int n, int mx,
                                uint32_t* sel) {
    const int lane = threadIdx.x & 63;
    const int g = lane & 7, grp = lane >> 3;
    if (n < mx) {   // input.Len() < max: every candidate stays
        for (int i = lane; i < n; i += 64) sel[i] = ci[i];
        wave_sync();
        return n;
    }
    int ns = 0;
    for (int i = 0; i < n && ns < mx; ++i) {
        const uint32_t c = ci[i];
        const float dq = cd[i];
        const float* cv = p.X + (uint64_t)c * p.ldx;
        bool bad = false;
        for (int j0 = 0; j0 < ns; j0 += 8) {
            const int j = j0 + grp;
            float pd = FLT_MAX;
            if (j < ns) pd = exact_dist_group8<METRIC>(cv, p.X + (uint64_t)sel[j] * p.ldx, p.D, g);
            bad = bad || (j < ns && pd < dq);
            if (__any(bad)) break;
        }
        if (!__any(bad)) {
            if (lane == 0) sel[ns] = c;
            ns++;
            wave_sync();
        }
    }
    return ns;
}

template <int METRIC>
__device__ void build_select_one(const BuildParams& b, int slot, int level, uint32_t* ci, float* cd, uint32_t* sel) {
    const HnswParams& p = b.h;
    const int lane = threadIdx.x & 63;
    const int target = b.target[slot];
    const uint64_t id = b.first + (uint64_t)slot;
    const uint64_t rq = ((uint64_t)slot * b.lb + level) * b.M;
    for (int i = lane; i < b.M; i += 64) b.req_key[rq + i] = ~0ull;
    if (level > min(target, p.max_level)) return;
    const int n = b.cand_n[(uint64_t)slot * b.lb + level];
    const uint64_t o = ((uint64_t)slot * b.lb + level) * p.ef;
    for (int i = lane; i < n; i += 64) { ci[i] = b.cand_i[o + i]; cd[i] = b.cand_d[o + i]; }
    wave_sync();
    const int ns = heuristic_select<METRIC>(p, ci, cd, n, b.M, sel);
    // own list, farthest first (popped from the results max-heap, :101-111)
    uint32_t* row;
    if (level == 0) row = const_cast<uint32_t*>(p.layer0) + id * (uint64_t)p.deg0;
    else row = const_cast<uint32_t*>(p.upper) + ((uint64_t)p.upper_row[id] * p.upper_levels + (level - 1)) * p.degU;
    for (int i = lane; i < ns; i += 64) {
        row[i] = sel[ns - 1 - i];
        b.req_key[rq + i] = ((uint64_t)level << 32) | sel[i];
        b.req_node[rq + i] = (uint32_t)id;
    }
    if (lane == 0) {
        if (level == 0) b.counts0[id] = ns;
        else b.countsU[(uint64_t)p.upper_row[id] * p.upper_levels + (level - 1)] = ns;
    }
}

__global__ __launch_bounds__(64) void wv_build_select_kernel(BuildParams b) {
    extern __shared__ float lds[];
    const int slot = blockIdx.x / b.lb, level = blockIdx.x % b.lb;
    if (slot >= b.nb) return;
    uint32_t* ci = reinterpret_cast<uint32_t*>(lds);
    float* cd = lds + b.h.ef;
    uint32_t* sel = reinterpret_cast<uint32_t*>(lds + 2 * b.h.ef);
    if (b.h.metric == WV_METRIC_L2) build_select_one<WV_METRIC_L2>(b, slot, level, ci, cd, sel);
    else if (b.h.metric == WV_METRIC_DOT) build_select_one<WV_METRIC_DOT>(b, slot, level, ci, cd, sel);
    else build_select_one<WV_METRIC_COSINE>(b, slot, level, ci, cd, sel);
}

// connectNeighborAtLevel for every new link of one neighbour, in batch order.
template <int METRIC>
__device__ void build_link_one(const BuildParams& b, int r, uint32_t* ci, float* cd, uint32_t* ui, float* ud,
                               uint32_t* sel, uint32_t* rowl) {
    const HnswParams& p = b.h;
    const int lane = threadIdx.x & 63;
    const int g = lane & 7, grp = lane >> 3;
    const uint64_t key = b.run_key[r];
    if (key == ~0ull) return;
    const int level = (int)(key >> 32);
    const uint32_t nb = (uint32_t)key;
    const int maxc = level == 0 ? b.M0 : b.M;
    uint32_t* row;
    uint32_t* cnt;
    if (level == 0) {
        row = const_cast<uint32_t*>(p.layer0) + (uint64_t)nb * p.deg0;
        cnt = b.counts0 + nb;
    } else {
        const uint64_t u = (uint64_t)p.upper_row[nb] * p.upper_levels + (level - 1);
        row = const_cast<uint32_t*>(p.upper) + u * p.degU;
        cnt = b.countsU + u;
    }
    const float* nv = p.X + (uint64_t)nb * p.ldx;
    int c = (int)*cnt;
    // the neighbour's list lives in LDS while its new links are applied
    for (int i = lane; i < c; i += 64) rowl[i] = row[i];
    wave_sync();
    const uint32_t off = b.run_off[r], len = b.run_len[r];
    for (uint32_t t = 0; t < len; ++t) {
        const uint32_t x = b.sorted_node[off + t];
        if (c < maxc) {   // appendConnectionAtLevelNoLock (:151-157)
            if (lane == 0) rowl[c] = x;
            c++;
            wave_sync();
            continue;
        }
        // re-prune (:158-205): the list plus x, distances to the neighbour
        const int n = c + 1;
        for (int i = lane; i < n; i += 64) ui[i] = i < c ? rowl[i] : x;
        wave_sync();
        for (int i0 = 0; i0 < n; i0 += 8) {
            const int i = i0 + grp;
            float d = 0.f;
            if (i < n) d = exact_dist_group8<METRIC>(p.X + (uint64_t)ui[i] * p.ldx, nv, p.D, g);
            if (i < n && g == 0) ud[i] = d;
        }
        wave_sync();
        // ascending by (d, id): rank placement
        for (int u = lane; u < n; u += 64) {
            const float d = ud[u];
            const uint32_t id = ui[u];
            int rk = 0;
            for (int i = 0; i < n; ++i) rk += key_less(ud[i], ui[i], d, id) || (i < u && ud[i] == d && ui[i] == id);
            ci[rk] = id;
            cd[rk] = d;
        }
        wave_sync();
        const int ns = heuristic_select<METRIC>(p, ci, cd, n, maxc, sel);
        for (int i = lane; i < ns; i += 64) rowl[i] = sel[ns - 1 - i];   // farthest first (max-heap pops)
        c = ns;
        wave_sync();
    }
    for (int i = lane; i < maxc; i += 64) row[i] = i < c ? rowl[i] : WV_NIL;
    if (lane == 0) *cnt = c;
}

__global__ __launch_bounds__(64) void wv_build_link_kernel(BuildParams b) {
    extern __shared__ float lds[];
    const int r = blockIdx.x;
    if (r >= b.n_runs) return;
    const int cap = b.M0 + 1;
    uint32_t* ci = reinterpret_cast<uint32_t*>(lds);
    float* cd = lds + cap;
    uint32_t* ui = reinterpret_cast<uint32_t*>(lds + 2 * cap);
    float* ud = lds + 3 * cap;
    uint32_t* sel = reinterpret_cast<uint32_t*>(lds + 4 * cap);
    uint32_t* rowl = reinterpret_cast<uint32_t*>(lds + 5 * cap);
    if (b.h.metric == WV_METRIC_L2) build_link_one<WV_METRIC_L2>(b, r, ci, cd, ui, ud, sel, rowl);
    else if (b.h.metric == WV_METRIC_DOT) build_link_one<WV_METRIC_DOT>(b, r, ci, cd, ui, ud, sel, rowl);
    else build_link_one<WV_METRIC_COSINE>(b, r, ci, cd, ui, ud, sel, rowl);
}

int hnsw_side_per_wave_words(int dpad, int side_rows, int vc_log2, int xs_log2) {
    return dpad + 2 * BATCH + 128 * side_rows + (1 << xs_log2) + MAX_LOCAL_TOMB + 256 + ((1 << vc_log2) + 1) / 2;
}

int hnsw_reg_per_wave_words(int dpad, int vc_log2) {
    return dpad + 2 * BATCH + MAX_LOCAL_TOMB + ((1 << vc_log2) + 1) / 2;
}

int hnsw_per_wave_words(int dpad, int efc, int sc, int vc_log2, int xs_log2) {
    return dpad + 4 * efc + 4 * sc + 4 * BATCH + ((1 << vc_log2) + 1) / 2 + (1 << xs_log2) + MAX_LOCAL_TOMB;
}

}  // namespace wv

extern "C" {

int wv_hnsw_per_wave_words(int dpad, int efc, int sc, int vc_log2, int xs_log2) {
    return wv::hnsw_per_wave_words(dpad, efc, sc, vc_log2, xs_log2);
}

int wv_hnsw_reg_per_wave_words(int dpad, int vc_log2) { return wv::hnsw_reg_per_wave_words(dpad, vc_log2); }

int wv_hnsw_side_per_wave_words(int dpad, int side_rows, int vc_log2, int xs_log2) {
    return wv::hnsw_side_per_wave_words(dpad, side_rows, vc_log2, xs_log2);
}

// side-register path (filtered / tombstoned / nil nodes, ef <= 128, no PQ);
// ev: layer 0 with the exact visited bitmap; wg: a workgroup per query
hipError_t wv_launch_hnsw_side(const wv::HnswParams* p, int waves_per_block, int ev, hipStream_t s) {
    if (p->nq == 0) return hipSuccess;
    const int nr = p->efc == 64 ? 1 : p->efc == 128 ? 2 : 0;
    if (nr == 0 || p->pq.codes || p->side_rows < 4 || (ev && (!p->vbits || !p->spill))) return hipErrorInvalidValue;
    if (p->wg_helpers) {
        const size_t lds = (size_t)p->per_wave_words * sizeof(float) + 16;
#define WV_HNSW_SIDE_WG(M, NRV, E) \
        hipLaunchKernelGGL((wv::wv_hnsw_side_wg_kernel<M, NRV, E>), dim3(p->nq), dim3(256), lds, s, *p)
#define WV_HNSW_SIDE_WG_M(M)                                                                                        \
        do {                                                                                                        \
            if (nr == 1) { if (ev) WV_HNSW_SIDE_WG(M, 1, true); else WV_HNSW_SIDE_WG(M, 1, false); }                \
            else { if (ev) WV_HNSW_SIDE_WG(M, 2, true); else WV_HNSW_SIDE_WG(M, 2, false); }                        \
        } while (0)
        if (p->metric == WV_METRIC_L2) WV_HNSW_SIDE_WG_M(WV_METRIC_L2);
        else if (p->metric == WV_METRIC_DOT) WV_HNSW_SIDE_WG_M(WV_METRIC_DOT);
        else WV_HNSW_SIDE_WG_M(WV_METRIC_COSINE);
#undef WV_HNSW_SIDE_WG_M
#undef WV_HNSW_SIDE_WG
        return hipGetLastError();
    }
    const size_t lds = (size_t)waves_per_block * p->per_wave_words * sizeof(float);
    const unsigned blocks = (unsigned)((p->nq + waves_per_block - 1) / waves_per_block);
#define WV_HNSW_SIDE_W(M, NRV, W)                                                                                   \
    do {                                                                                                            \
        if (ev) hipLaunchKernelGGL((wv::wv_hnsw_side_kernel<M, NRV, WV_HNSW_SIDE_RPG, W, true>), dim3(blocks),      \
                                   dim3(64 * waves_per_block), lds, s, *p);                                         \
        else hipLaunchKernelGGL((wv::wv_hnsw_side_kernel<M, NRV, WV_HNSW_SIDE_RPG, W, false>), dim3(blocks),        \
                                dim3(64 * waves_per_block), lds, s, *p);                                            \
    } while (0)
#define WV_HNSW_SIDE(M)                                                                                             \
    do {                                                                                                            \
        if (nr == 1 && wps == 3) WV_HNSW_SIDE_W(M, 1, 3);                                                           \
        else if (nr == 1) WV_HNSW_SIDE_W(M, 1, 2);                                                                  \
        else if (wps == 3) WV_HNSW_SIDE_W(M, 2, 3);                                                                 \
        else WV_HNSW_SIDE_W(M, 2, 2);                                                                               \
    } while (0)
    // 12 waves per CU need <= 168 VGPRs (spilling a few) and <= 13 KiB of LDS
    // per wave; otherwise the LDS caps it at 8 anyway
    int wps = (size_t)p->per_wave_words * 4 <= 13 * 1024 ? 3 : 2;
    if (const char* e = std::getenv("WV_HNSW_SIDE_WPS")) wps = std::atoi(e) == 3 ? 3 : 2;
    if (p->metric == WV_METRIC_L2) WV_HNSW_SIDE(WV_METRIC_L2);
    else if (p->metric == WV_METRIC_DOT) WV_HNSW_SIDE(WV_METRIC_DOT);
    else WV_HNSW_SIDE(WV_METRIC_COSINE);
#undef WV_HNSW_SIDE
#undef WV_HNSW_SIDE_W
    return hipGetLastError();
}

hipError_t wv_launch_build_search(const wv::BuildParams* b, int waves_per_block, hipStream_t s) {
    const size_t lds = (size_t)waves_per_block * b->h.per_wave_words * sizeof(float);
    const unsigned blocks = (unsigned)((b->nb + waves_per_block - 1) / waves_per_block);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_build_search_kernel, dim3(blocks), dim3(64 * waves_per_block), lds, s, *b);
    return hipGetLastError();
}

hipError_t wv_launch_build_select(const wv::BuildParams* b, hipStream_t s) {
    const size_t lds = (2 * (size_t)b->h.ef + b->M) * sizeof(float);
    if (b->nb == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_build_select_kernel, dim3((unsigned)(b->nb * b->lb)), dim3(64), lds, s, *b);
    return hipGetLastError();
}

hipError_t wv_launch_build_link(const wv::BuildParams* b, hipStream_t s) {
    const size_t lds = 6 * ((size_t)b->M0 + 1) * sizeof(float);
    if (b->n_runs == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_build_link_kernel, dim3((unsigned)b->n_runs), dim3(64), lds, s, *b);
    return hipGetLastError();
}

// workgroup-per-query launch of an unfiltered register-path search (no PQ)
hipError_t wv_launch_hnsw_wg(const wv::HnswParams* p, hipStream_t s) {
    if (p->nq == 0) return hipSuccess;
    const int nr = p->sc == 0 && !p->allow ? (p->efc == 64 ? 1 : p->efc == 128 ? 2 : p->efc <= 256 ? 4 : 0) : 0;
    if (nr == 0 || p->pq.codes || !p->wg_helpers) return hipErrorInvalidValue;
    const size_t lds = (size_t)p->per_wave_words * sizeof(float) + 16;
#define WV_HNSW_WG(M)                                                                                              \
    do {                                                                                                           \
        if (nr == 1) hipLaunchKernelGGL((wv::wv_hnsw_wg_kernel<M, 1>), dim3(p->nq), dim3(256), lds, s, *p);       \
        else if (nr == 2) hipLaunchKernelGGL((wv::wv_hnsw_wg_kernel<M, 2>), dim3(p->nq), dim3(256), lds, s, *p);  \
        else hipLaunchKernelGGL((wv::wv_hnsw_wg_kernel<M, 4>), dim3(p->nq), dim3(256), lds, s, *p);               \
    } while (0)
    if (p->metric == WV_METRIC_L2) WV_HNSW_WG(WV_METRIC_L2);
    else if (p->metric == WV_METRIC_DOT) WV_HNSW_WG(WV_METRIC_DOT);
    else WV_HNSW_WG(WV_METRIC_COSINE);
#undef WV_HNSW_WG
    return hipGetLastError();
}

hipError_t wv_launch_hnsw(const wv::HnswParams* p, int waves_per_block, hipStream_t s) {
    const size_t lds = (size_t)waves_per_block * p->per_wave_words * sizeof(float);
    const unsigned blocks = (unsigned)((p->nq + waves_per_block - 1) / waves_per_block);
    if (blocks == 0) return hipSuccess;
    // results in registers: unfiltered (no side set) with ef <= 64 (one
    // register) or ef <= 128 (two)
    const int nr = p->sc == 0 && !p->allow ? (p->efc == 64 ? 1 : p->efc == 128 ? 2 : p->efc <= 256 ? 4 : 0) : 0;
#define WV_HNSW_LAUNCH(M, PQ)                                                                                        \
    do {                                                                                                             \
        if (nr == 1) hipLaunchKernelGGL((wv::wv_hnsw_kernel<M, PQ, 1>), dim3(blocks), dim3(64 * waves_per_block),   \
                                        lds, s, *p);                                                                 \
        else if (nr == 2) hipLaunchKernelGGL((wv::wv_hnsw_kernel<M, PQ, 2>), dim3(blocks),                          \
                                             dim3(64 * waves_per_block), lds, s, *p);                                \
        else if (nr == 4) hipLaunchKernelGGL((wv::wv_hnsw_kernel<M, PQ, 4>), dim3(blocks),                          \
                                             dim3(64 * waves_per_block), lds, s, *p);                                \
        else hipLaunchKernelGGL((wv::wv_hnsw_kernel<M, PQ, 0>), dim3(blocks), dim3(64 * waves_per_block), lds, s,   \
                                *p);                                                                                 \
    } while (0)
    // a compressed index (PQ codes) is its own instantiation: the raw-vector
    // kernel keeps its registers and schedule
    if (p->pq.codes) {
        if (p->metric == WV_METRIC_L2) WV_HNSW_LAUNCH(WV_METRIC_L2, true);
        else if (p->metric == WV_METRIC_DOT) WV_HNSW_LAUNCH(WV_METRIC_DOT, true);
        else WV_HNSW_LAUNCH(WV_METRIC_COSINE, true);
    } else {
        if (p->metric == WV_METRIC_L2) WV_HNSW_LAUNCH(WV_METRIC_L2, false);
        else if (p->metric == WV_METRIC_DOT) WV_HNSW_LAUNCH(WV_METRIC_DOT, false);
        else WV_HNSW_LAUNCH(WV_METRIC_COSINE, false);
    }
#undef WV_HNSW_LAUNCH
    return hipGetLastError();
}

}  // extern "C"
