// wv_params.h -- kernel parameter blocks shared by the kernels and the host API.
#pragma once
#include <stdint.h>

namespace wv {

constexpr int BF_BQ = 128;   // queries per workgroup tile
constexpr int BF_BN = 128;   // base rows per workgroup tile
constexpr int BF_BK = 32;    // k-chunk staged through LDS
constexpr int BF_LDT = 36;   // LDS row: 32 k + 4 pad floats (odd 16-byte stride: conflict-free b128)
constexpr int BF_KP = 8;     // candidates kept per producer lane (register list)
constexpr int BF_PROD = 4;   // producers per query: 2 base-row waves x 2 lane halves
constexpr int FIN_KF = 32;   // candidates re-ranked exactly per query
constexpr int BF_FAST_KMAX = 32;   // k served by the MFMA + finalize pipeline
// larger k (searches with limit > 32, SearchByVectorDistance's deepening): the
// f16 key pass with at least 2k lists per query, merged by the wide finalize
constexpr int BF_WIDE_KMAX = 256;
constexpr int FINW_NE = 8192;      // list entries one wide-finalize workgroup sorts in LDS
constexpr int FINW_KF = 1024;      // candidates it re-ranks exactly at most
constexpr int HNSW_EF_MAX = 512;   // largest ef the LDS beam holds

struct BfParams {
    const float* X;         // base rows [N][ldx]
    const float* Q;         // queries [nq][ldq]
    const float* xnorm;     // |x|^2 per row (L2 only)
    const uint64_t* tomb;   // excluded ids (tombstones, nil nodes, missing rows)
    const uint64_t* allow;  // allow bits (nullable)
    const uint32_t* rowidx; // compacted rows (nullable): tile row r = corpus row rowidx[r], N = their count
    uint64_t tomb_nbits, allow_nbits, allow_stride;  // stride in words (0 = shared)
    uint64_t N;
    int nq, D, ldx, ldq, metric;
    // flattened schedule (bf_schedule): the (query block, base tile) units are
    // numbered qb * ntiles + tile and cut into n_blocks equal contiguous runs
    int n_qblocks, n_slots;
    uint64_t ntiles, units_per_block;
    float* out_d;           // [nq][n_slots][BF_PROD*BF_KP]
    uint32_t* out_id;
    int split;              // X and Q are split images (split_hi_index): wv_bf_split_kernel
    int bq;                 // queries per block (BF_BQ; the split kernel runs 2 * BF_BQ)
    int prod;               // producers (lists) per query per slot: BF_PROD
    int locality;           // bit 1: XCD-contiguous block ids; bit 2: aligned tile rotation
};

// MFMA-native bf16 hi/lo image (split key pass): 32-row group g, 32-k chunk c,
// k-step s (16 k), part (hi = 0, lo = +512): a 1 KiB block of 64 lanes x 8
// bf16 where lane (h << 5 | r) holds row 32 g + r, k = 32 c + 16 s + 8 h ..
// +7 -- the A/B operand of v_mfma_f32_32x32x16_bf16.  nk = stride / 32; an
// image of R rows (R a multiple of 32) takes R * stride * 4 bytes, as fp32.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t split_hi_index(uint64_t row, int k, int nk) {
    const uint64_t g = row >> 5;
    const int r = (int)(row & 31), c = k >> 5, kk = k & 31, s = kk >> 4, h = (kk >> 3) & 1, e = kk & 7;
    return ((((g * nk + c) * 2 + s) * 2) * 64 + (h * 32 + r)) * 8 + e;
}

// Equal-work schedule for wv_bf_mfma_kernel: exactly n_blocks workgroups
// (a multiple of the resident slots) so no partial last wave of workgroups.
// A block's run of units crosses at most a few query blocks; the lists it
// produces for query block qb go to slot (block - first block of qb).
struct BfSchedule {
    int n_blocks, n_slots, bq;
    uint64_t ntiles, units_per_block;
};
inline BfSchedule bf_schedule(int nq, uint64_t N, int target_blocks, int bq = BF_BQ, int tile_rows = BF_BN) {
    BfSchedule s{};
    s.bq = bq;
    const uint64_t nqb = (uint64_t)(nq + bq - 1) / bq;
    s.ntiles = (N + tile_rows - 1) / tile_rows;
    const uint64_t total = nqb * s.ntiles;
    uint64_t nb = target_blocks > 0 ? (uint64_t)target_blocks : 1;
    if (nb > total) nb = total;
    s.units_per_block = (total + nb - 1) / nb;
    s.n_blocks = (int)((total + s.units_per_block - 1) / s.units_per_block);
    // slots touched by one query block: ceil(ntiles / U) + 1 at most
    s.n_slots = (int)((s.ntiles + s.units_per_block - 1) / s.units_per_block) + 1;
    return s;
}
// The same schedule with every query block cut at the same tile offsets (S
// slots of U tiles; the unit grid per query block is S U >= the corpus's tiles,
// the padding units empty), so that the blocks of all query blocks that scan a
// tile start and run together -- with the XCD block order (run_h16), in one
// XCD's L2.  Used where it costs no work: S = target / nqb slots, U no larger
// than the flat schedule's run (else n_blocks = 0: use bf_schedule).
inline BfSchedule bf_schedule_aligned(int nq, uint64_t N, int target_blocks, int bq, int tile_rows,
                                      bool any_cost = false) {
    BfSchedule s{};
    s.bq = bq;
    const uint64_t nqb = (uint64_t)(nq + bq - 1) / bq;
    const uint64_t nt = (N + tile_rows - 1) / tile_rows;
    const uint64_t S = nqb ? (uint64_t)(target_blocks > 0 ? target_blocks : 1) / nqb : 0;
    if (nqb < 2 || S < 1 || nt < S) return s;
    const uint64_t U = (nt + S - 1) / S;
    const uint64_t flat = (nqb * nt + (uint64_t)target_blocks - 1) / (uint64_t)target_blocks;
    if (U > flat + flat / 64 && !any_cost) return s;
    s.units_per_block = U;
    s.ntiles = S * U;
    s.n_blocks = (int)(nqb * S);
    s.n_slots = (int)S + 1;
    return s;
}
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int bf_first_block(uint64_t qb, uint64_t ntiles, uint64_t upb) { return (int)(qb * ntiles / upb); }
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int bf_slots_of(uint64_t qb, uint64_t ntiles, uint64_t upb) {
    return (int)(((qb + 1) * ntiles - 1) / upb) - bf_first_block(qb, ntiles, upb) + 1;
}

// ---- f16 key pass (wv_bf_h16_kernel, wv_h16.hip) ---------------------------
// One f16 product per fp32 product: keys k~ = s * (|x|^2 + sum f16(s_x x) *
// f16(s_q b)) / (s_x s_q) up to the certified error (BfFinParams.h16), b = -2q
// (L2) or -q; s = s_x * s_q (powers of two).  Corpus image: f16 rows in the
// MFMA-native A layout of h16_index, 64-row tiles of 2 * ns KiB contiguous.
constexpr int H_BN = 64;      // corpus rows per tile
constexpr int H_WAVES = 8;    // waves per workgroup (one 512-thread workgroup per CU)
constexpr int H_BQ = 512;     // queries per block: 64 per wave, held in registers as B operands
constexpr int H_PROD = 2;     // lists per query per slot (the two lane halves)
constexpr int H_NS_MAX = 8;   // 16-k steps: D <= 128
constexpr int H_SAMPLE = 16;  // seed pre-pass: every H_SAMPLE-th tile

#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t h16_index(uint64_t row, int k, int ns) {
    const uint64_t block = (row >> 5) * (uint64_t)ns + (uint64_t)(k >> 4);   // (32-row group, 16-k step)
    const uint64_t lane = (uint64_t)(((k >> 3) & 1) * 32) + (row & 31);
    return (block * 64 + lane) * 8 + (uint64_t)(k & 7);
}

// The wide-D (D > 128) corpus image: 16-row groups of ns * 512 B, each a
// sequence of 1 KiB panels (32 k, i.e. 64 B, of the group's 16 rows, row
// after row).  A run of 16 consecutive rows' panel is one contiguous 1 KiB
// piece (an unfiltered scan's LDS-DMA), and any single row's panel is 64
// contiguous bytes (a compacted scan's per-lane fill, no gathered copy).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint64_t h16w_index(uint64_t row, int k, int ns) {
    return (row >> 4) * (uint64_t)ns * 256 + (uint64_t)(k >> 5) * 512 + (row & 15) * 32 + (uint64_t)(k & 31);
}

struct H16Params {
    const void* X;            // corpus image (h16_index), rows padded to whole tiles (zeros)
    const void* Q;            // query image (h16_index over query rows), padded to whole H_BQ blocks
    const float* xns;         // s * |x|^2 per row (L2 only), padded to whole tiles
    const uint64_t* excl;     // excluded rows (tombstones, nil nodes, no vector): one word per tile
    const uint64_t* allow;    // shared allow bits (nullable): at least one word per tile
    const float* tau;         // [nq] seed threshold in true key units (nullable): keys above it are dropped
    const float* qscale;      // device scalar s_q (read at launch)
    float sx;                 // corpus scale s_x
    uint64_t N;               // rows
    int nq, metric;
    int n_qblocks, n_slots;
    uint64_t ntiles, units_per_block;   // ntiles: tiles scanned (the sample's when tile_stride > 1)
    uint64_t ntiles_real;     // the wide-D pass: the corpus's tiles (ntiles, the unit grid per query block, may pad it)
    int tile_stride;          // corpus tile = tile_base + scanned tile * tile_stride (seed pre-pass)
    uint64_t tile_base;       // (the D <= 128 pass; 0 elsewhere)
    int out_slots;            // list slots per query in out_d / out_id (0: n_slots)
    uint64_t clean_tiles;     // corpus tiles [0, clean_tiles) have no excluded row (no allow list either): no mask
    int locality;             // bit 1: XCD-contiguous workgroup ids
    const int* block_order;   // optional: XCD-contiguous position -> block (run_h16's block_order)
    float* out_d;             // [nq][n_slots][H_PROD][BF_KP] scaled keys
    uint32_t* out_id;
    // running per-query threshold shared by every slot (k <= 2 BF_KP): each
    // lane pair publishes an upper bound of the query's k-th key (k of its own
    // list entries) + 2 eps, atomicMin'ed into gtau (order-preserving keys of
    // scaled units, h16_key_enc); keys above it are dropped everywhere
    unsigned int* gtau;       // [nq] (nullable)
    int kth;                  // k (0: no running threshold)
    const float* marg;        // [nq] 2 eps in scaled key units, rounded up (wv_h16_margin_kernel)
    // cross-slot threshold (xslot, 32x32x16 pass): each slot stores its lists'
    // heads in gslot[q][2 slot + lane half] at a few points of its segment and
    // reads the others', whose k-th smallest + 2 eps bounds the k-th key
    float* gslot;             // [nq][2 n_slots] (xslot)
    int xslot;                // 1: use gslot instead of the gtau publish
    int ns;                   // 16-k steps of the images (the wide-D kernel: a multiple of HW_KC)
    int wide_rows;            // the wide-D kernel's rows per wave: 128 (256-row tiles) or 64 (128-row tiles)
    // the wide-D kernel (round 5): X is h16w_index (row r's 64 B panels per
    // 16-row group) and its operand blocks are filled per lane; rowidx
    // (nullable): scan rows rowidx[0 .. N) (a compacted allow list, ascending,
    // padded to whole 256-row tiles) instead of rows 0 .. N -- no gathered image
    const uint32_t* rowidx;
    // (nullable, wide-D kernel) the row count as the device computed it (a
    // compacted list's length, never read back by the host): the schedule is
    // then n_slots - 1 slots per query block of U = ceil(tiles / slots) tiles
    // each, fixed at kernel start; the host passes ntiles = n_slots - 1 and
    // units_per_block = 1 (the same grid, slots and block order)
    const uint32_t* n_dev;
};

// ---- f16 key pass for D > 128 (wv_bf_h16w_kernel, wv_h16.hip) --------------
// Both operands stream through LDS in 64-k chunks (3 stages): 128 corpus rows
// x 256 queries per 512-thread workgroup, 64 x 64 per wave; the tile epilogue
// (mask, minima, extraction) runs once per D / 64 chunks.
constexpr int HW_BN = 256;    // corpus rows per tile (wide_rows 128; 128 at wide_rows 64)
constexpr int HW_BQ = 256;    // queries per block
constexpr int HW_KC = 4;      // 16-k steps per chunk
constexpr int HW_PROD = 4;    // lists per query per slot: 2 row halves x 2 lane halves
constexpr int HW_NS_MAX = 64; // D <= 1024

// order-preserving uint keys of floats (a < b <=> enc(a) < enc(b)); +inf and
// above (0xFF800000..) decode to +inf
#if defined(__HIPCC__)
__host__ __device__
#endif
inline unsigned int h16_key_enc(float f) {
    union { float f; unsigned int u; } v;
    v.f = f;
    return (v.u & 0x80000000u) ? ~v.u : (v.u | 0x80000000u);
}
#if defined(__HIPCC__)
__host__ __device__
#endif
inline float h16_key_dec(unsigned int k) {
    if (k >= 0xFF800000u) return __builtin_inff();
    union { float f; unsigned int u; } v;
    v.u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    return v.f;
}

struct H16SeedParams {
    const float* minima;      // [nq][n_slots][H_PROD] pre-pass running minima (scaled keys)
    int n_slots;
    uint64_t ntiles, units_per_block;   // the pre-pass schedule
    int nq, k, metric, D;
    const float* qscale;
    float sx;
    const float* qnorm;       // |q|^2 (L2) or |q|
    float xnorm_max, ex_max;
    const float* qres;
    float* tau;               // [nq] out: threshold in true key units (+inf: none)
    unsigned int* gtau;       // [nq] out (nullable): h16_key_enc(tau * s), the running threshold's start
    int bq;                   // queries per block of the pre-pass
    int prod;                 // minima per query per slot (0: H_PROD)
    // list mode (ids != nullptr; tau holds the minima pre-pass's thresholds,
    // which the result never exceeds): `minima` are the list pre-pass's lists
    // ([nq][n_slots][prod] entries, prod = H_PROD BF_KP), the key of each a
    // distinct row; their 2 BF_KP smallest also go to the main pass's lists as
    // one more slot (slot bf_slots_of(qb) of out_ntiles / out_upb, out_slots
    // per query): even ranks to its first list, odd ranks to its second
    const uint32_t* ids;
    float* out_d;
    uint32_t* out_id;
    int out_slots;
    uint64_t out_ntiles, out_upb;
};

struct BfFinParams {
    const float* X;
    const float* Q;
    const float* cand_d;
    const uint32_t* cand_id;
    const float* qnorm;     // |q|^2 (L2) or |q| (dot, cosine)
    float xnorm_max;        // max |x| over the corpus (rounded up)
    int n_slots;            // list slots per query (BfParams.n_slots)
    int extra_slot;         // 1: one more slot of lists after a query block's slots (the seed pre-pass's)
    uint64_t ntiles, units_per_block;
    int nq, D, ldx, ldq, metric, k;
    uint64_t id_base;       // global id of local id 0
    uint64_t* out_ids;      // [nq][k]
    float* out_d;
    int32_t* out_n;
    int32_t* fail;          // per query: 1 = uncertified
    float* fail_thr;        // per query: exact d_k of the re-ranked set (upper bound of the true d_k)
    int split;              // approximate keys came from the bf16x3 pass (wider eps)
    int bq;                 // queries per block of the key pass (BfParams.bq)
    int prod;               // producers per query per slot (BfParams.prod)
    int kp;                 // entries per list (0: BF_KP)
    int finw_ne;            // wide finalize: LDS entry capacity (a power of two >= FINW_KF; 0: FINW_NE)
    // f16 key pass (h16 = 1): keys are scaled by s = sx * qscale[0]; eps adds
    // ex_max * |B| + xnorm_max * qres[q] (the f16 rounding of corpus and query)
    int h16;
    const float* qscale;    // device scalar s_q
    float sx;
    float ex_max;           // max_x |x - f16(s_x x) / s_x| (rounded up)
    const float* qres;      // [nq] |b - f16(s_q b) / s_q| (rounded up)
    const float* tau_in;    // [nq] seed threshold the key pass dropped keys above (nullable)
    float* tau_out;         // seed pre-pass: [nq] threshold in true key units, no results written
    // (nullable, finalize_one) the candidates' ids are positions in this
    // ascending row list (a compacted allow list): the selected positions are
    // mapped to rows before the re-rank -- the map is increasing, so every
    // (key, id) order on positions is the order on rows.  Positions at or
    // past the list's length (rowidx_n, or *rowidx_ndev when set) map to nil.
    const uint32_t* rowidx;
    uint64_t rowidx_n;
    const uint32_t* rowidx_ndev;
};

// Certificate fallback: exact distances of every row for a batch of failed
// queries, keeping the rows with d <= thr[f] (thr = an upper bound of the
// true k-th distance), then a per-query sort of the survivors.
constexpr int FB_CAP = 2048;       // survivors kept per failed query
struct FbParams {
    const float* X;
    const float* Q;          // all queries [nq][ldq]
    const int32_t* qidx;     // [nf] query index of each failed query
    const float* thr;        // [nq] threshold per query
    const uint64_t* tomb;
    const uint64_t* allow;
    uint64_t tomb_nbits, allow_nbits, allow_stride;
    uint64_t N;
    int nf, D, ldx, ldq, metric, k;
    uint64_t id_base;
    float* cand_d;           // [nf][FB_CAP]
    uint32_t* cand_id;
    uint32_t* cand_n;        // [nf] (may exceed FB_CAP: overflow)
    uint64_t* out_ids;       // [nq][k]
    float* out_d;
    int32_t* out_n;
    int32_t* overflow;       // [nf] 1 = more than FB_CAP survivors
    // device-resolved fallback (no host round trip): the failed queries are
    // listed on the device (qidx, *d_nf <= nf); the filter / select kernels
    // loop over them, and an overflowed query is answered by a full scan into
    // scratch[slot][N] plus a radix select (fbd kernels, wv_bf.hip)
    const int32_t* d_nf;
    float* scratch;
    int n_scr;
    unsigned long long* fb_total;   // += number of listed queries (batch stats; nullable)
};
constexpr int FBD_SCR = 8;   // full-scan slots of the device fallback

struct ScanParams {
    const float* X;
    const float* q;          // one query (device)
    const uint64_t* tomb;
    const uint64_t* allow;
    uint64_t tomb_nbits, allow_nbits;
    uint64_t N;
    int D, ldx, metric;
    float* dist;             // [N]
    uint32_t* ids;           // [N] iota
};

// Product-quantized rows (ssdhelpers/product_quantization.go): codes[row]
// holds m codes (u8 when ks <= 256, else u16) at a row stride of `stride`
// bytes; cent[m][ks][ds] = kms[i].Centroid(c).  codes == nullptr: raw vectors.
struct PqParams {
    const uint8_t* codes;
    const float* cent;
    uint64_t stride;
    int m, ks, ds, wide;
};

struct HnswParams {
    const float* X;
    const int8_t* levels;
    const uint32_t* layer0;
    const uint32_t* upper_row;
    const uint32_t* upper;
    const uint64_t* tomb;
    const uint64_t* allow;
    const float* Q;
    uint64_t N, tomb_nbits, allow_nbits, allow_stride, id_base;
    uint32_t entrypoint;
    int D, ldx, ldq, metric, deg0, degU, max_level;
    int upper_levels;    // level stride of `upper` (>= max_level)
    int nq, k, ef;
    int efc, sc, vc_log2, xs_log2, dpad, per_wave_words;
    // visited cache (round 5): 2^vc_log2 16-bit slots; node id -> h = id *
    // 2654435761 mod 2^(vc_log2 + vc_tbits) (a bijection on ids below that
    // power of two, which covers N), slot = h >> vc_tbits, tag = the low
    // vc_tbits <= 15 bits (0xFFFF: empty) -- an exact membership test per
    // slot in half the LDS of a 32-bit id
    int vc_tbits;
    uint64_t* out_ids;   // [nq][k]
    float* out_d;
    int32_t* out_n;
    int32_t* status;     // bit0 side overflow, bit1 expanded-set / spill overflow
    uint32_t* counters;  // [nq][2]: distance evaluations, expansions (nullable)
    PqParams pq;         // compressed index: distances from codes (search.go:171-199)
    // diagnostic (WV_HNSW_UNIQUE_COUNTS): one exact visited bitmap per query
    // ([nq][uniq_words], zeroed): layer-0 evaluations are counted once per
    // node, as the reference's exact visited list does (search.go:256-264) --
    // the lossy LDS cache's re-evaluations are not -- so the count equals the
    // restatement's E on the same traversal (nullable: off)
    unsigned long long* uniq;
    uint64_t uniq_words;
    // a second pass (nullable): only the queries whose entry here is non-zero
    // (the first pass's status: its side state overflowed) search again
    const int32_t* redo;
    // (round 5) workgroup per query (wv_hnsw_wg_kernel, small unfiltered
    // batches): wave 0 searches, waves 1..3 compute rows 32 v .. 32 v + 31 of
    // every distance batch -- one memory round trip for up to 128 rows
    int wg_helpers;
    // (round 6) side-register path (wv_hnsw_side_kernel: filtered,
    // tombstoned or nil-node searches with ef <= 128): results in registers,
    // the side candidates' smallest keys in a side_rows x 64-entry LDS array,
    // the rest in a per-query spill in HBM (spill_cap (d, id) pairs), and an
    // exact layer-0 visited bitmap per query in HBM ([nq][vwords] u32, zeroed
    // before the launch: search.go:256-264 exactly, so nothing is evaluated or
    // queued twice).  The upper levels keep the LDS cache + expanded set
    // (2^xs_log2 slots).
    int side_rows;
    uint32_t* vbits;
    uint64_t vwords;
    uint32_t* spill;
    int spill_cap;
    int vb_host_clear;   // the host zeroed vbits (A/B switch; default: each wave clears its own)
    // batch stats (nullable): [3] += queries whose side state overflowed an
    // exact-visited search (the exact fallback answers them), [4] += queries
    // a lossy first pass handed to the exact-visited search
    unsigned long long* side_acc;
    int ev_spec;   // (A/B, WV_HNSW_EV_SPEC) exact-visited rows loaded beside the claims
};

// SearchByVectorDistance's threshold pass (wv_sbd.hip): per query, the
// allowed rows within the target distance, with their sort keys and counts
struct SbdParams {
    const float* X;
    const float* Q;           // [nq][dpad] (normalized if cosine)
    const float* target;      // [nq]
    const uint64_t* excl;     // tombstones, nil nodes, missing rows
    const uint64_t* allow;    // nullable; [nq][allow_stride] or shared
    uint64_t excl_nbits, allow_nbits, allow_stride, N;
    int D, ldx, dpad, metric, nq;
    uint64_t rows_per_block;
    int cap;                  // list entries per query
    unsigned long long* keys; // [nq][cap]: (orderable d) << 32 | row
    unsigned int* cnt;        // [nq][3]: |Q|, A (d <= target), n (rows searchable)
};

// Flat search over PQ codes (flat_search.go:19-74 on a compressed index):
// distances of a chunk of queries against a row list, keyed for a stable
// segmented sort by (dist, row).
struct PqScanParams {
    PqParams pq;
    const float* Q;          // [nq][ldq] prepared queries (normalized for cosine)
    const uint32_t* rows;    // [nr] ascending row ids (nullable: rows 0..nr-1)
    const uint64_t* excl;    // excluded rows (tombstones, nil nodes, rows without a code)
    const uint64_t* allow;   // allow bits (nullable)
    uint64_t excl_nbits, allow_nbits, allow_stride;
    uint64_t nr;
    int q0, nqc, ldq, metric;
    float* key;              // [nqc][nr] sort key: the distance (+0 for -0), +inf = excluded
    float* dist;             // [nqc][nr] the distance as computed
    uint32_t* val;           // [nqc][nr] j
};

// GPU graph construction: one batch of new nodes
// [first, first + nb), inserted against the graph of the h.N nodes before it.
struct BuildParams {
    HnswParams h;             // graph + search state: h.N inserted rows, h.entrypoint, h.max_level current top
    uint64_t first;
    int nb;                   // batch size
    int lb;                   // level slots per node in the candidate buffers (max target + 1)
    int M;                    // maximumConnections: selected per level, upper-layer capacity
    int M0;                   // maximumConnectionsLayerZero = 2M: layer-0 capacity
    const int8_t* target;     // [nb] drawn level of each batch node
    uint32_t* cand_i;         // [nb][lb][efc] efConstruction results per level, ascending
    float* cand_d;
    int32_t* cand_n;          // [nb][lb]
    uint32_t* counts0;        // [cap] layer-0 list lengths
    uint32_t* countsU;        // [n_upper][upper_levels]
    uint64_t* req_key;        // [nb][lb][M] reverse-link requests: level << 32 | neighbour (~0 = none)
    uint32_t* req_node;       //   ... the new node that links to it
    const uint64_t* run_key;  // link phase: one run of equal keys per wave
    const uint32_t* run_off;
    const uint32_t* run_len;
    const uint32_t* sorted_node;
    int n_runs;
};

}  // namespace wv
