/*
 * wv_oracle.h -- CPU restatement of Weaviate's vector-index search path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * product path (weaviate_amd/csrc) and the CPU baseline timed by bench.py's
 * cpu_baseline leg.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path never links or calls it.
 *
 * Parity pinning: the reference hot path is Go + Go assembly and there is no
 * Go toolchain in the build image, so the reference cannot be compiled or run
 * here (recorded in DESIGN.md).  This restatement is pinned against every
 * known-answer vector the reference's own tests hold for the path (copied as
 * data into tests/golden/reference_kats.json) and cross-checks its scalar
 * emulation of the AVX2 assembly against an instruction-by-instruction
 * _mm256 intrinsics mirror of the same assembly.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * adapters/repos/db/vector/hnsw/ unless stated).
 */
#ifndef WV_ORACLE_H
#define WV_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { WVO_L2 = 0, WVO_DOT = 1, WVO_COSINE = 2 };

/* ---- distancers (distancer/ and distancer/asm/) -------------------- */
/* asm-order distance (the path taken on AVX2 hosts): l2_amd64.s / dot_amd64.s */
float wvo_distance(int metric, const float *a, const float *b, int n);
/* same, via _mm256 intrinsics mirroring the assembly instruction by instruction */
float wvo_distance_avx2(int metric, const float *a, const float *b, int n);
/* pure-Go fallback order (non-AVX2 hosts): l2.go:16-25, dot_product.go:23-31 */
float wvo_distance_purego(int metric, const float *a, const float *b, int n);
/* raw asm.L2 / asm.Dot kernels */
float wvo_asm_l2(const float *x, const float *y, int n);
float wvo_asm_dot(const float *x, const float *y, int n);
/* distancer/normalize.go:16-32 */
void wvo_normalize(const float *in, float *out, int n);
void wvo_normalize_rows(const float *in, float *out, uint64_t rows, int dim);

/* ---- binary heap clone (priorityqueue/queue.go) for the heap-order KAT -- */
/* Runs a script of ops on a fresh Min (is_max=0) or Max (is_max=1) queue.
 * op[i] = 0: Insert(ids[i], dists[i]); op[i] = 1: Pop() -> appended to out. */
int wvo_pq_script(int is_max, int nops, const int *op, const uint64_t *ids,
                  const float *dists, uint64_t *out_ids, float *out_d);

/* ---- search-time ef (search.go:30-62) ----------------------------------- */
int wvo_search_time_ef(int64_t ef, int64_t ef_min, int64_t ef_max,
                       int64_t ef_factor, int k);

/* ---- index ---------------------------------------------------------------- */
typedef struct wvo_index wvo_index;

typedef struct {
    uint64_t dist_evals;   /* E: distance evaluations (excl. redundant recomputes) */
    uint64_t expansions;   /* X: candidate pops that read a neighbour list       */
    uint64_t nbr_slots;    /* neighbour-list entries scanned                      */
    uint64_t visited;      /* visited-set insertions                              */
    uint64_t max_cand;     /* high-water mark of the candidate heap               */
    uint64_t layer0_visited_max; /* max visited count of one layer-0 search      */
    uint64_t ties;         /* decisions taken between equal distances (heap order) */
    /* diagnostics of the side candidates (traversed but ineligible: filtered
     * out or tombstoned, search.go:282-298), collected only after
     * wvo_set_side_diag(1): the high-water mark of the live ones (distance
     * <= worst, or all of them while the results are not full) over one
     * layer-0 search, and how many were expanded (total / max per search) */
    uint64_t side_live_max;
    uint64_t side_exp;
    uint64_t side_exp_max;
} wvo_stats;

void wvo_set_side_diag(int on);

wvo_index *wvo_create(int dim, int metric, int max_connections,
                      int ef_construction, uint64_t capacity, uint64_t seed);
void wvo_destroy(wvo_index *h);
void wvo_set_search_config(wvo_index *h, int64_t ef, int64_t ef_min,
                           int64_t ef_max, int64_t ef_factor,
                           int64_t flat_search_cutoff, int forbid_flat);
/* Store the vector for id without inserting a graph node (object store stand-
 * in: VectorForIDThunk).  Cosine vectors are normalized as on read
 * (vector_cache.go:110-112). */
int wvo_set_vector(wvo_index *h, uint64_t id, const float *vec);
/* the object store lost id's object: later reads of its vector fail */
int wvo_clear_vector(wvo_index *h, uint64_t id);
/* Add (insert.go:43-65 / 103-217).  Levels are drawn from a counter-based
 * generator keyed by (seed, id) so the graph does not depend on thread
 * interleaving of the level draws. */
int wvo_add(wvo_index *h, uint64_t id, const float *vec);
/* concurrent Add of n vectors with ids first_id.. (threads<=1: sequential) */
int wvo_add_batch(wvo_index *h, uint64_t first_id, const float *vecs,
                  uint64_t n, int threads);
/* override the level draw for the next wvo_add (test hook, like randFunc) */
void wvo_set_next_level(wvo_index *h, int level);
int wvo_add_tombstone(wvo_index *h, uint64_t id);
int wvo_remove_tombstone(wvo_index *h, uint64_t id);

/* graph import (debug.go:108-175 NewFromJSONDump*) */
int wvo_import_node(wvo_index *h, uint64_t id, int level,
                    const uint64_t *conns, const int *counts /* level+1 */);
int wvo_import_csr(wvo_index *h, uint64_t n, const float *vecs, const int8_t *levels, const uint32_t *layer0,
                   int deg0, const uint32_t *upper_row, const uint32_t *upper, int degU, int max_level,
                   uint64_t entrypoint);
/* commit log written during builds (commitlog/logger.go record layouts) */
void wvo_log_enable(wvo_index *h, int on);
uint64_t wvo_log_size(wvo_index *h);
uint64_t wvo_log_copy(wvo_index *h, uint8_t *out, uint64_t cap);
void wvo_set_entrypoint(wvo_index *h, uint64_t ep, int max_level);

/* graph export for the GPU CSR upload */
void wvo_graph_info(wvo_index *h, uint64_t *n_slots, uint64_t *entrypoint,
                    int *max_level, uint64_t *n_upper_nodes);
/* levels[n_slots] (-1 for nil nodes), layer0[n_slots*deg0] padded with
 * 0xFFFFFFFF, counts0[n_slots] */
int wvo_export_layer0(wvo_index *h, int deg0, int8_t *levels, uint32_t *layer0,
                      uint32_t *counts0);
/* upper layers: for node with level L>=1 (in id order) row r:
 *   upper_row[id] = r (0xFFFFFFFF otherwise),
 *   upper[r][l-1][0..degU) neighbours at level l (padded), l = 1..L */
int wvo_export_upper(wvo_index *h, int degU, int max_level, uint32_t *upper_row,
                     uint32_t *upper, uint64_t n_rows);

/* ---- search entry points ------------------------------------------------ */
/* allow_bits: nullable bitmap over ids (bit i of word i/64); the AllowList of
 * helpers/allow_list.go:19-118 restated as a dense bitmap.  Results are written
 * ascending; *out_n receives the count. */
int wvo_search_by_vector(wvo_index *h, const float *q, int k,
                         const uint64_t *allow_bits, uint64_t allow_nbits,
                         uint64_t *out_ids, float *out_d, int *out_n,
                         wvo_stats *st);
int wvo_knn_search(wvo_index *h, const float *q, int k, int ef,
                   const uint64_t *allow_bits, uint64_t allow_nbits,
                   uint64_t *out_ids, float *out_d, int *out_n, wvo_stats *st);
int wvo_flat_search(wvo_index *h, const float *q, int k,
                    const uint64_t *allow_bits, uint64_t allow_nbits,
                    uint64_t *out_ids, float *out_d, int *out_n);
/* SearchByVectorDistance (search.go:90-158): outputs up to out_cap results */
int wvo_search_by_vector_distance(wvo_index *h, const float *q, float target,
                                  int64_t max_limit, const uint64_t *allow_bits,
                                  uint64_t allow_nbits, uint64_t *out_ids,
                                  float *out_d, int64_t out_cap,
                                  int64_t *out_n);
/* batched knnSearchByVector, queries split in contiguous chunks over threads
 * like ssdhelpers.Concurrently (ssdhelpers/utils.go:22-37).  mode 0 = knn
 * (hnsw), 1 = flat over allow list (exact). out_* are Q*k. */
int wvo_search_batch(wvo_index *h, const float *qs, int nq, int k, int ef,
                     const uint64_t *allow_bits, uint64_t allow_nbits, int mode,
                     int threads, uint64_t *out_ids, float *out_d, int *out_n,
                     wvo_stats *st);

/* ---- product quantization (ssdhelpers/product_quantization.go, kmeans.go) */
/* bits / bytes of NewProductQuantizer (:116-179) */
int wvo_pq_layout(int ks, int use_bits, int *bits, int *bytes);
/* ExtractCode / PutCode over one encoded vector (:191-258) */
int wvo_pq_extract(const uint8_t *enc, int n_codes, int ks, int use_bits, uint64_t *out);
int wvo_pq_put(const uint64_t *codes, int n_codes, int ks, int use_bits, uint8_t *enc);
/* DistanceBetweenCompressedAndUncompressedVectors (:284-291) = the LUT
 * distance (:56-75); cent[m][ks][dim/m] */
float wvo_pq_distance(int metric, const float *x, const uint8_t *enc, const float *cent, int m, int ks, int dim,
                      int use_bits);
/* Encode (:348-354) with KMeans encoders (kmeans.go:78-110): enc[n][m*bytes] */
int wvo_pq_encode_kmeans(const float *vecs, uint64_t n, int dim, int m, int ks, const float *cent, int use_bits,
                         uint8_t *enc);
/* Compress (hnsw/compress.go:39-89): all later searches use PQ distances */
int wvo_compress(wvo_index *h, int m, int ks, int use_bits, const float *cent, const uint8_t *codes,
                 const uint8_t *has, uint64_t n);

/* ---- standalone exact scan over raw arrays (no index) -------------------- */
/* flatSearch semantics (flat_search.go:19-74) over ids 0..n-1 of a row-major
 * base[n][dim]; tombstone/allow bitmaps nullable.  Cosine inputs must already
 * be normalized.  Parallel over queries. */
int wvo_flat_scan(int metric, const float *base, uint64_t n, int dim,
                  const float *qs, int nq, int k, const uint64_t *allow_bits,
                  const uint64_t *tomb_bits, int threads, uint64_t *out_ids,
                  float *out_d, int *out_n);

#ifdef __cplusplus
}
#endif
#endif
