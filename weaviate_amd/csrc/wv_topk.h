// wv_topk.h -- per-lane candidate lists of the brute-force key passes
// (wv_bf.hip, wv_h16.hip): the tile minimum, and the rare extraction of keys
// that beat a lane's list tail.
#pragma once
#include "wv_device.h"
#include "wv_params.h"

#include <type_traits>

namespace wv {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// v_min3_f32 without the IEEE canonicalisation hipcc wraps around fminf of
// MFMA results (a NaN key never wins a comparison either way)
#ifdef WV_BF_DBG_ITERS
// ablation builds only: wave-level counts of tiles (0), extract-loop rounds
// (1), lanes that ran a round (2) and extraction calls (3); counted by the
// first active lane (the loops are divergent)
__device__ unsigned long long wv_dbg_counts[4];
#define WV_DBG_COUNT(i)                                                                        \
    {                                                                                          \
        const uint64_t dbg_b = __ballot(1);                                                    \
        if (__lane_id() == __builtin_ctzll(dbg_b)) {                                           \
            atomicAdd(&wv_dbg_counts[i], 1ull);                                                \
            if ((i) == 1) atomicAdd(&wv_dbg_counts[2], (unsigned long long)__popcll(dbg_b));   \
        }                                                                                      \
    }
extern "C" __attribute__((weak)) void wv_dbg_read(unsigned long long* out) { hipMemcpyFromSymbol(out, HIP_SYMBOL(wv_dbg_counts), 32); }
#else
#define WV_DBG_COUNT(i)
#endif

__device__ __forceinline__ float min3_raw(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Split pass candidate extraction (rare: a lane runs it only when its tile
// minimum M beats its list tail; the wave runs it while any lane does, so it
// is kept branch-free).  A0 / A1 hold this lane's 32 keys of one query column
// (row offsets (r & 3) + 8 (r >> 2) and 32 + the same); each round takes the
// minimum, masks it to +inf and inserts it.  Insertion compares keys only:
// a key equal to the tail is dropped, which the finalize's certificate (all
// dropped keys >= the smallest tail) still covers, and the reported ids and
// distances come from the exact re-rank.  PT is the lane-pair partner's tail
// (a valid rejection threshold, see the caller).
__device__ __forceinline__ void split_extract(float& M, floatx16& A0, floatx16& A1, float (&ld)[BF_KP],
                                              uint32_t (&li)[BF_KP], float pt, uint32_t rb0,
                                              const uint32_t* __restrict__ rowidx = nullptr) {
    const float INF = __builtin_inff();
    while (M <= fminf(ld[BF_KP - 1], pt)) {
        WV_DBG_COUNT(1)
        // position of M: a descending scan, so among equal keys the lowest row wins
        uint32_t sel = 0;
#pragma unroll
        for (int r = 15; r >= 0; --r) sel = A1[r] == M ? 16u + r : sel;
#pragma unroll
        for (int r = 15; r >= 0; --r) sel = A0[r] == M ? (uint32_t)r : sel;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            A0[r] = sel == (uint32_t)r ? INF : A0[r];
            A1[r] = sel == 16u + r ? INF : A1[r];
        }
        uint32_t rb = rb0;   // opaque: the row ids stay in this rare loop
        asm volatile("" : "+v"(rb));
        if (!(M < ld[BF_KP - 1])) break;
        uint32_t id = rb + (sel & 3u) + 8u * ((sel >> 2) & 3u) + 32u * (sel >> 4);
        if (rowidx) id = rowidx[id];   // corpus id; the map is increasing
        float d = M;
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            const bool lt = d < ld[i];
            const float td = ld[i];
            const uint32_t ti = li[i];
            ld[i] = lt ? d : td;
            li[i] = lt ? id : ti;
            d = lt ? td : d;
            id = lt ? ti : id;
        }
        M = INF;
#pragma unroll
        for (int r = 0; r < 16; ++r) M = min3_raw(M, A0[r], A1[r]);
    }
}


// split_extract over one 32 x 32 accumulator's 16 keys of a lane (rows
// rb + (r & 3) + 8 (r >> 2)): the f16 pass extracts per half tile.  The keys
// are compared with fminf (the file is built with -fno-honor-nans: v_min3
// without canonicalisation; a NaN key -- only possible after an f16 overflow,
// whose residual makes eps infinite -- never certifies anything).
__device__ __forceinline__ void split_extract16(float& M, floatx16& A, float (&ld)[BF_KP], uint32_t (&li)[BF_KP],
                                                float pt, uint32_t rb) {
    const float INF = __builtin_inff();
    while (M <= fminf(ld[BF_KP - 1], pt)) {
        WV_DBG_COUNT(1)
        uint32_t sel = 0;
#pragma unroll
        for (int r = 15; r >= 0; --r) sel = A[r] == M ? (uint32_t)r : sel;
#pragma unroll
        for (int r = 0; r < 16; ++r) A[r] = sel == (uint32_t)r ? INF : A[r];
        uint32_t rbo = rb;   // opaque: the row ids stay in this rare loop
        asm volatile("" : "+v"(rbo));
        if (!(M < ld[BF_KP - 1])) break;
        uint32_t id = rbo + (sel & 3u) + 8u * (sel >> 2);
        float d = M;
#pragma unroll
        for (int i = 0; i < BF_KP; ++i) {
            const bool lt = d < ld[i];
            const float td = ld[i];
            const uint32_t ti = li[i];
            ld[i] = lt ? d : td;
            li[i] = lt ? id : ti;
            d = lt ? td : d;
            id = lt ? ti : id;
        }
        float m0 = fminf(fminf(A[0], A[1]), A[2]), m1 = fminf(fminf(A[3], A[4]), A[5]);
        float m2 = fminf(fminf(A[6], A[7]), A[8]), m3 = fminf(fminf(A[9], A[10]), A[11]);
        m0 = fminf(fminf(m0, A[12]), A[13]);
        m1 = fminf(fminf(m1, A[14]), A[15]);
        M = fminf(fminf(m0, m1), fminf(m2, m3));
    }
}

// Candidate insertion by key position (the f16 passes' rare path, round 4):
// for each of the lane's NK keys (rows rb + (r & 3) + 8 (r >> 2), + 32 for
// the second accumulator) the wave tests key <= thr by ballot; only positions
// where some lane hits run the insertion, for every hitting lane at once.  So
// an event costs NK compares + one insertion per hit position, instead of a
// wave-serial round (scan for the minimum's position, mask it, insert,
// re-reduce) per key that serves ~1 lane.  thr is the lane's threshold at the
// event's start; a key that no longer beats the list's tail when its turn
// comes is dropped by the insertion itself (key-only compares: a key equal to
// the tail does not enter -- the certificate covers it, see split_extract).
__device__ __forceinline__ void list_insert(float d, uint32_t id, float (&ld)[BF_KP], uint32_t (&li)[BF_KP]) {
#pragma unroll
    for (int i = 0; i < BF_KP; ++i) {
        const bool lt = d < ld[i];
        const float td = ld[i];
        const uint32_t ti = li[i];
        ld[i] = lt ? d : td;
        li[i] = lt ? id : ti;
        d = lt ? td : d;
        id = lt ? ti : id;
    }
}
__device__ __forceinline__ void ballot_extract(const floatx16& A, float thr, float (&ld)[BF_KP], uint32_t (&li)[BF_KP],
                                               uint32_t rb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const bool c = A[r] <= thr;
        if (__any(c)) {
            WV_DBG_COUNT(1)
            uint32_t id = rb;   // opaque: the row ids stay in this rare path
            asm volatile("" : "+v"(id));
            if (c) list_insert(A[r], id + (uint32_t)((r & 3) + 8 * (r >> 2)), ld, li);
        }
    }
}

// A column whose smallest key m is under its threshold (x, per lane): m goes
// in straight from its position (a select chain, no per-key branch); the
// column's other keys are scanned only when one of them is also under the
// lane's threshold after the insertion (rare).  The list ends as after
// ballot_extract(A, thr): a key between the new and the old tail falls off
// the list either way.  A's entry at m's position is cleared to +inf.
__device__ __forceinline__ void min_extract(float m, bool x, floatx16& A, float pt, float (&ld)[BF_KP],
                                            uint32_t (&li)[BF_KP], uint32_t rb) {
    int pos = 15;
#pragma unroll
    for (int r = 14; r >= 0; --r) pos = A[r] == m ? r : pos;
    uint32_t id = rb;   // opaque: the row ids stay in this rare path
    asm volatile("" : "+v"(id));
    if (x) list_insert(m, id + (uint32_t)((pos & 3) + 8 * (pos >> 2)), ld, li);
    const float thr2 = x ? fminf(ld[BF_KP - 1], pt) : -__builtin_inff();
    float m2 = __builtin_inff();
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        A[r] = r == pos ? __builtin_inff() : A[r];
        A[r + 1] = r + 1 == pos ? __builtin_inff() : A[r + 1];
        m2 = fminf(fminf(m2, A[r]), A[r + 1]);
    }
    if (__builtin_expect(__any(m2 <= thr2), 0)) ballot_extract(A, thr2, ld, li, rb);
}

// Certificate eps of the f16 key pass (true units): |key + offset - reference
// distance| <= eps for every row, offset = |q|^2 (L2), 0 (dot), 1 (cosine).
// Accumulation and reference-order terms 6 (D + 4) 2^-24 (|q| + max|x|)^2
// (L2) / |q| max|x| (dot, cosine), plus the f16 rounding of the corpus
// (ex_max |b~|) and of the query (max|x| qres), b = -2q (L2) or -q.
__device__ __forceinline__ float h16_eps(int metric, int D, float qnorm, float xnorm_max, float ex_max, float qres) {
    const float u = 5.9604645e-08f;
    const float D4 = (float)(D + 4);
    float eps;
    if (metric == WV_METRIC_L2) {
        const float qn = sqrtf(qnorm);
        const float s = qn + xnorm_max;
        eps = 6.f * D4 * u * s * s + ex_max * (2.f * qn + qres) + xnorm_max * qres;
    } else {
        eps = 6.f * D4 * u * qnorm * xnorm_max + 4.f * u + ex_max * (qnorm + qres) + xnorm_max * qres;
    }
    return eps * 1.0001f;
}

// Finalize sort keys: (dist, id) as one u64 whose unsigned order is
// key_less's (dist's bits made monotonic -- -0 folded into +0 first, as the
// float compare ties them -- then the id's 31 bits; nil ids come back as nil:
// no row id reaches 2^31 - 1).  One v_cmp_lt_u64 per compare: key_less's
// short-circuit form compiled to exec-mask branches in these sorts, ~10x
// their shuffle cost at one wave per SIMD (in-kernel stamps).
__device__ __forceinline__ uint64_t fin_key(float d, uint32_t id) {
    uint32_t u = __float_as_uint(d + 0.0f);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((uint64_t)u << 32) | (uint64_t)(id & WV_IDMASK);
}
__device__ __forceinline__ void fin_unkey(uint64_t k, float& d, uint32_t& id) {
    uint32_t u = (uint32_t)(k >> 32);
    u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    d = __uint_as_float(u);
    const uint32_t lo = (uint32_t)k;
    id = lo == WV_IDMASK ? WV_NIL : lo;
}

// A wave-wide bitonic sort of 256 fin_key keys, element i = 64 j + lane in
// register j: strides >= 64 inside the lane, smaller ones by shuffles; the
// smallest FIN_KF end in lanes 0 .. FIN_KF - 1 of j = 0.
__device__ __forceinline__ void bitonic256_wave(uint64_t (&kk)[4], int lane) {
#pragma unroll
    for (int k = 2; k <= 256; k <<= 1) {
#pragma unroll
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            if (jj >= 64) {
                // (register pairs named by literal indices: a runtime
                // j ^ (jj / 64) made the arrays dynamically indexed)
                auto cas = [&](auto jc, auto pc) {
                    constexpr int j = decltype(jc)::value, pj = decltype(pc)::value;
                    const bool up = ((64 * j + lane) & k) == 0;   // element j is the lower index
                    // (operands selected, then one compare: a ternary of two
                    // compares compiled to exec-mask branches)
                    const uint64_t a = up ? kk[pj] : kk[j], b = up ? kk[j] : kk[pj];
                    const bool sw = a < b;
                    const uint64_t t = kk[j];
                    kk[j] = sw ? kk[pj] : kk[j];
                    kk[pj] = sw ? t : kk[pj];
                };
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                using I2 = std::integral_constant<int, 2>;
                using I3 = std::integral_constant<int, 3>;
                if (jj == 64) { cas(I0{}, I1{}); cas(I2{}, I3{}); }
                else { cas(I0{}, I2{}); cas(I1{}, I3{}); }
            } else {
                const bool lower = (lane & jj) == 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t plo = (uint32_t)__shfl_xor((int)(uint32_t)kk[j], jj, 64);
                    const uint32_t phi = (uint32_t)__shfl_xor((int)(uint32_t)(kk[j] >> 32), jj, 64);
                    const uint64_t pk = ((uint64_t)phi << 32) | plo;
                    const bool up = ((64 * j + lane) & k) == 0;
                    // the lower index of an ascending pair keeps the min
                    const bool c = lower == up;
                    const uint64_t a = c ? pk : kk[j], b = c ? kk[j] : pk;
                    const bool take = a < b;
                    kk[j] = take ? pk : kk[j];
                }
            }
        }
    }
}

}  // namespace wv
