/*
 * wvgpu.h -- C ABI of the MI355X vector-index engine (libwvgpu.so).
 *
 * This is the drop-in boundary a cgo package (adapters/repos/db/vector/gpu,
 * see INTEGRATION.md) binds.  It replaces, for the search path, the methods of
 * the reference's VectorIndex interface
 *   adapters/repos/db/vector_index.go:23-40
 *     SearchByVector(vector []float32, k int, allow helpers.AllowList)
 *         ([]uint64, []float32, error)                          -> wv_search_by_vector
 *     SearchByVectorDistance(vector []float32, dist float32, maxLimit int64,
 *         allow helpers.AllowList) ([]uint64, []float32, error)  -> wv_search_by_vector_distance
 * as implemented by the hnsw package
 *   adapters/repos/db/vector/hnsw/search.go:64-79 (SearchByVector)
 *   adapters/repos/db/vector/hnsw/search.go:90-158 (SearchByVectorDistance)
 *   adapters/repos/db/vector/hnsw/search.go:460-550 (knnSearchByVector)
 *   adapters/repos/db/vector/hnsw/flat_search.go:19-74 (flatSearch)
 * plus a batched entry point (wv_search_batch*) that a Go-side micro-batcher
 * uses to coalesce concurrent single-query calls.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Host pointers unless the name says
 *    _device.  The library copies inputs during the call and never retains a
 *    caller pointer after returning (cgo pointer rules).
 *  - Every function returns a wv_status; on failure wv_last_error() returns a
 *    thread-local message.  Nothing aborts or exits across the ABI.
 *  - Ids: the index holds local ids 0..capacity-1 (Weaviate docIDs are dense per
 *    shard, adapters/repos/db/indexcounter); results are returned as uint64
 *    ids = id_base + local id (id_base set at creation, for corpus sharding).
 *  - The AllowList (adapters/repos/db/helpers/allow_list.go:19-118) crosses
 *    the boundary as a dense little-endian uint64 bitmap: bit i of word i/64
 *    set <=> docID i allowed.  allow_bits == NULL means "no filter".
 *  - Results are ascending by distance; equal distances are ordered by id.
 *  - Thread safety: an index may be searched from many threads at once (calls
 *    on one index are serialised on its stream; wv_batcher coalesces
 *    concurrent single-query calls into batches).  Uploads (vectors, graph,
 *    tombstones, config) must not race with searches on the same index.
 */
#ifndef WVGPU_H
#define WVGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    WV_OK = 0,
    WV_EINVAL = 1,    /* bad argument */
    WV_EOOM = 2,      /* device allocation failed */
    WV_EDEVICE = 3,   /* HIP runtime / kernel launch failure */
    WV_ESTATE = 4,    /* index not ready for this call (e.g. no graph for HNSW) */
    WV_EDELETED = 5   /* entrypoint deleted (search.go:473-476) */
} wv_status;

/* distancer.Provider.Type() (distancer/provider.go:14-24) */
typedef enum { WV_L2_SQUARED = 0, WV_DOT = 1, WV_COSINE_DOT = 2 } wv_metric;

typedef enum {
    WV_MODE_AUTO = 0,   /* SearchByVector dispatch: flat if allow && !forbidFlat && |allow| < cutoff */
    WV_MODE_EXACT = 1,  /* flatSearch over the allow list (or every id) */
    WV_MODE_HNSW = 2    /* knnSearchByVector */
} wv_mode;

/* The subset of ent.UserConfig (entities/vectorindex/hnsw/config.go:53-185)
 * that the search path reads (index.go:79-87). */
typedef struct {
    int device;                 /* HIP device ordinal */
    int max_connections;        /* M; layer-0 degree 2M (index.go:223) */
    int64_t ef;                 /* -1 = dynamic */
    int64_t dynamic_ef_min;
    int64_t dynamic_ef_max;
    int64_t dynamic_ef_factor;
    int64_t flat_search_cutoff;
    int forbid_flat;
    uint64_t id_base;           /* global id of local id 0 */
} wv_config;

typedef struct wv_index wv_index;

/* Fill cfg with the reference defaults (config.go:33-50). */
void wv_config_default(wv_config *cfg);

int wv_index_create(int dim, int metric, const wv_config *cfg, uint64_t capacity, wv_index **out);
int wv_index_destroy(wv_index *ix);
int wv_index_update_config(wv_index *ix, const wv_config *cfg);

/* Upload n rows (row-major float32 [n][dim]) for local ids first_id..first_id+n-1.
 * Cosine vectors are normalized on the device exactly as Normalize does
 * (distancer/normalize.go:16-32). */
int wv_index_upload_vectors(wv_index *ix, const float *rows, uint64_t n, uint64_t first_id);
/* Same, from a device pointer (row stride ld floats). */
int wv_index_upload_vectors_device(wv_index *ix, const float *d_rows, uint64_t n, uint64_t first_id, int ld);

/* HNSW graph as a fixed-degree CSR snapshot of the reference graph
 * (vertex.go:18-24 connections[level]):
 *   levels[n]                 node level, -1 for nil nodes
 *   layer0[n*deg0]            layer-0 neighbours in stored order, pad 0xFFFFFFFF
 *   upper_row[n]              row of the node in `upper` (0xFFFFFFFF if level 0)
 *   upper[n_upper*max_level*degU]  neighbours at level l in row[l-1]; the
 *                             level stride is exactly max_level (lists above
 *                             max_level are never searched, search.go:479)
 * deg0 <= 256 and degU <= 256.  A nil entrypoint returns WV_EDELETED
 * (search.go:473-476); an entrypoint whose level is below max_level is legal
 * and is skipped at the layers above its level (search.go:226-233). */
int wv_index_upload_graph(wv_index *ix, uint64_t n, const int8_t *levels, const uint32_t *layer0, int deg0,
                          const uint32_t *upper_row, const uint32_t *upper, uint64_t n_upper, int degU,
                          int max_level, uint64_t entrypoint);

/* GPU graph construction: the graph of rows [0, n_rows),
 * built on the device with the reference's insert (insert.go:103-217): level
 * floor(-ln(U)/ln(M)) (U counter-based per id and seed, the same draw as the
 * CPU restatement), ef=1 descent, efConstruction search per level,
 * selectNeighborsHeuristic to M (heuristic.go:23-135), bidirectional links
 * re-pruned at 2M (layer 0) / M (connectNeighborAtLevel,
 * neighbor_connections.go:134-209).  Nodes are inserted in id order in
 * batches of max(1, inserted / batch_div) (at most 16384) that search the
 * graph of all earlier batches.  The result is the index's graph (as after
 * wv_index_upload_graph, M = cfg.max_connections). */
int wv_index_build_graph(wv_index *ix, int ef_construction, uint64_t seed, int batch_div);
/* The index's graph in the wv_index_upload_graph layout (nullable outputs). */
int wv_index_graph_info(wv_index *ix, uint64_t *n, int *deg0, int *degU, int *max_level, uint64_t *n_upper,
                        uint64_t *entrypoint);
int wv_index_download_graph(wv_index *ix, int8_t *levels, uint32_t *layer0, uint32_t *upper_row, uint32_t *upper);

/* Tombstones (delete.go:546-566) as a bitmap over local ids (replaces the set). */
int wv_index_set_tombstones(wv_index *ix, const uint64_t *bits, uint64_t nbits);

/* Incremental writes while serving.  wv_index_add mirrors
 * hnsw.Add (insert.go:43-65): rows for arbitrary local ids, normalized for
 * cosine; an id the uploaded graph does not hold joins the delta set, which
 * every HNSW search also scans exactly and merges by (dist, id) -- the row is
 * findable at once, as after the reference's insert -- until a later
 * wv_index_upload_graph snapshot contains it.  Tombstones are added / removed
 * one by one (delete.go:29-84 AddTombstone, tombstone cleanup). */
int wv_index_add(wv_index *ix, const uint64_t *ids, const float *rows, uint64_t n);
int wv_index_add_tombstones(wv_index *ix, const uint64_t *ids, uint64_t n);
int wv_index_remove_tombstones(wv_index *ix, const uint64_t *ids, uint64_t n);
int wv_index_delta_size(wv_index *ix, uint64_t *n);
/* Capacity growth in place, every row, code, tombstone and the graph kept
 * (hnsw grows its node array the same way: maintainance.go:31-100
 * growIndexToAccomodateNode).  Waits for the queued work first; must not
 * race with searches.  wv_index_capacity: the capacity and highest row + 1. */
int wv_index_reserve(wv_index *ix, uint64_t capacity);
int wv_index_capacity(const wv_index *ix, uint64_t *capacity, uint64_t *n_rows);

/* Product quantization (ssdhelpers/product_quantization.go,
 * hnsw/compress.go:39-89).  The fitted quantizer crosses as its centroid
 * table, centroid_table[segments][centroids][dims/segments] =
 * kms[i].Centroid(c) (KMeans centers, or the tile encoder's one-float
 * centroids), plus encoder = ssdhelpers.Encoder (0 tile, 1 kmeans).
 * Codes are uploaded in ProductQuantizer.Encode's layout (segments * bytes
 * per vector, big-endian, bit-packed when use_bits_encoding and bits < 8 *
 * bytes: wv_pq_code_len), or -- KMeans -- encoded on the device from the
 * resident vectors (KMeans.Nearest, kmeans.go:78-110).  With the index
 * compressed (h.compressed) every search ranks by the PQ distance
 * (DistanceBetweenCompressedAndUncompressedVectors :284-291 = the lookup-table
 * distance :56-75): flatSearch and knnSearchByVector alike, as the reference
 * does.  Rows written later are encoded on the device (KMeans, insert.go:91-95)
 * or wait for their codes (tile encoder). */
enum { WV_PQ_TILE = 0, WV_PQ_KMEANS = 1 };
int wv_pq_code_len(int segments, int centroids, int use_bits_encoding);
int wv_index_set_pq(wv_index *ix, int segments, int centroids, int use_bits_encoding, int encoder,
                    const float *centroid_table);
int wv_index_upload_pq_codes(wv_index *ix, const uint8_t *encoded, uint64_t n, uint64_t first_id);
int wv_index_pq_encode(wv_index *ix);
/* the device codes of rows first_id.., one uint16 per segment: out[n][segments] */
int wv_index_download_pq_codes(wv_index *ix, uint16_t *out, uint64_t first_id, uint64_t n);
/* compressed on/off (h.compressed); on requires a code for every row holding a vector */
int wv_index_set_compressed(wv_index *ix, int on);

/* searchTimeEF (search.go:30-62) for the current config; the same rule for a
 * config without an index (no device needed). */
int wv_search_time_ef(const wv_index *ix, int k);
int wv_config_search_time_ef(const wv_config *cfg, int k);

/* SearchByVector (search.go:64-79). out_ids/out_dists have room for k;
 * *out_n receives the count (0 for an empty index). */
int wv_search_by_vector(wv_index *ix, const float *vector, int k, const uint64_t *allow_bits,
                        uint64_t allow_nbits, uint64_t *out_ids, float *out_dists, int32_t *out_n);

/* SearchByVectorDistance (search.go:90-158).  max_limit < 0 means unlimited.
 * At most out_cap results are written; *out_n receives the full count. */
int wv_search_by_vector_distance(wv_index *ix, const float *vector, float target_distance,
                                 int64_t max_limit, const uint64_t *allow_bits, uint64_t allow_nbits,
                                 uint64_t *out_ids, float *out_dists, int64_t out_cap, int64_t *out_n);

/* SearchByVectorDistance for a batch of queries (each with its own target
 * distance; one max_limit; allow lists shared or per query as in
 * wv_search_batch).  Outputs [nq][out_cap]; out_n[q] = the number of results
 * (entries past out_cap are not written).  Round 1 runs as the batch's
 * SearchByVector where that is an HNSW search; every exact round (a flat
 * round 1, all deeper rounds) is one threshold pass + segmented sort on the
 * device, launched beside round 1 -- one device sync per batch instead of a
 * host loop of single-query searches. */
int wv_search_by_vector_distance_batch(wv_index *ix, const float *queries, int nq, const float *target_distances,
                                       int64_t max_limit, const uint64_t *allow_bits, uint64_t allow_nbits,
                                       uint64_t allow_stride_words, uint64_t *out_ids, float *out_dists,
                                       int64_t out_cap, int64_t *out_n);

/* Batched search of nq queries (row-major [nq][dim]).  ef <= 0 selects
 * searchTimeEF(k).  allow_bits may be NULL, one bitmap shared by the batch
 * (allow_stride_words == 0) or one bitmap per query.  out_* are [nq][k]. */
int wv_search_batch(wv_index *ix, const float *queries, int nq, int k, int ef, const uint64_t *allow_bits,
                    uint64_t allow_nbits, uint64_t allow_stride_words, int mode, uint64_t *out_ids,
                    float *out_dists, int32_t *out_n);

/* Device-resident variant: every pointer is device memory.  d_queries holds
 * nq rows at a stride of wv_index_query_ld(ix) floats (dim rounded up to 4;
 * the pad columns are ignored).  The work is queued on `stream` (a
 * hipStream_t, NULL = the index's own stream, then also ordered after the work
 * already queued on the legacy default stream, where a caller may have just
 * written d_queries) and ordered after every earlier call on the index; later
 * calls on the index are ordered after it.  The
 * results are complete when the stream reaches the end of the queued work.
 * Exact searches (k <= 256 on the f16 key pass, k <= 32 otherwise) without an
 * allow list or, for D > 128, with a shared one (compacted on the device), and
 * HNSW searches with or without allow lists queue everything, certificate
 * and side-set fallbacks included (resolved on the device), and return
 * without waiting for the GPU; AUTO's per-query flat/HNSW decision over allow
 * lists, the D <= 128 exact pass over a shared allow list (row compaction),
 * the exact scan for larger k and PQ-compressed fallbacks still read counts
 * back.
 * Batch stats and kernel times are read (one sync) only when asked for. */
int wv_search_batch_device(wv_index *ix, const float *d_queries, int nq, int k, int ef,
                           const uint64_t *d_allow_bits, uint64_t allow_nbits, uint64_t allow_stride_words,
                           int mode, uint64_t *d_out_ids, float *d_out_dists, int32_t *d_out_n, void *stream);
/* Row stride (floats) of the device query rows wv_search_batch_device reads. */
int wv_index_query_ld(const wv_index *ix);
/* Wait for every call queued on the index's own stream (a NULL `stream`). */
int wv_index_synchronize(wv_index *ix);

/* Merge per-shard results: for each query, the k best (dist, id) of the
 * n_shards lists d_in_*[shard][nq][k] (entries beyond d_in_n are ignored).
 * Used after the RCCL all-gather of corpus-shard results. */
int wv_merge_shards_device(const float *d_in_dists, const uint64_t *d_in_ids, const int32_t *d_in_n, int n_shards,
                           int nq, int k, float *d_out_dists, uint64_t *d_out_ids, int32_t *d_out_n, void *stream);

/* Statistics of the last batch on the index (nullable outputs): HNSW distance
 * evaluations and expansions summed over the batch, and the queries answered
 * by the certificate fallback.  Waits for the batch to finish. */
int wv_last_batch_stats(wv_index *ix, uint64_t *dist_evals, uint64_t *expansions, uint64_t *fallbacks);

/* The last batch's filtered-HNSW state (nullable outputs): the queries whose
 * side candidates outgrew the per-query spill (answered by the exact
 * fallback), the queries a light-filter first pass (lossy visited cache)
 * handed to the exact-visited pass, the visited-bitmap claims (atomics: the
 * LDS visited cache's misses at layer 0), and the side-register launch's LDS side
 * array (rows of 64 entries) and spill capacity (entries per query; 0 when no
 * filtered HNSW search ran).  Waits for the batch to finish.  A measurement
 * hook (no reference counterpart). */
int wv_last_side_stats(wv_index *ix, uint64_t *overflowed, uint64_t *redone, uint64_t *claims, int *side_rows,
                       int *spill_cap);

/* Kernel timing with HIP events on the launch stream (off by default).  When
 * enabled, every batch records the device time of its dominant kernels: the
 * MFMA brute-force kernel, the exact re-rank/finalize kernel and the HNSW
 * beam-search kernel.  wv_last_kernel_times / wv_last_seed_time wait for the
 * recorded batches and return the per-batch average (milliseconds) over the
 * batches since the previous read (or since timing was enabled). */
int wv_index_set_timing(wv_index *ix, int enable);
int wv_last_kernel_times(wv_index *ix, float *bf_mfma_ms, float *bf_finalize_ms, float *hnsw_ms);
/* The f16 key pass's seed pre-pass of the last batch (key pass over every
 * 16th tile + its finalize), milliseconds; 0 when it did not run. */
int wv_last_seed_time(wv_index *ix, float *seed_ms);

/* HNSW commit log -> CSR.  Replays the write-ahead log a
 * Weaviate shard persists (adapters/repos/db/vector/hnsw/commitlog/logger.go
 * record layouts) exactly as Deserializer.Do does at startup
 * (deserializer.go:80-158, startup.go:56-152), so a GPU mirror can serve an
 * existing shard without rebuilding its graph.  Never modifies the files: a
 * record torn at the end of a file is reported (info.truncated) and the state
 * keeps every complete record, as the reference does before truncating. */
typedef struct wv_graph wv_graph;
typedef struct {
    uint64_t n_slots;        /* highest live node id + 1 */
    uint64_t entrypoint;
    uint64_t n_upper;        /* nodes with level >= 1 */
    uint64_t n_tombstones;
    uint64_t valid_bytes;    /* bytes of complete records over all files */
    int max_level;           /* SetEntryPointMaxLevel's level */
    int max_node_level;      /* highest level field of a live node */
    int max_deg0, max_degU;  /* longest layer-0 / upper neighbour list */
    int compressed;          /* an AddPQ record was seen (wv_graph_get_pq: its quantizer) */
    int truncated;           /* a file ended inside a record */
} wv_graph_info;
/* one log held in memory */
int wv_graph_load_commitlog_buffer(const uint8_t *buf, uint64_t len, wv_graph **out);
/* log files in the given order */
int wv_graph_load_commitlogs(const char *const *paths, int n_paths, wv_graph **out);
/* <root>/<name>.hnsw.commitlog.d: files ordered by timestamp name
 * (commit_logger.go:121-166), temporaries and hidden files ignored, a
 * .condensed file whose original still exists skipped
 * (corrupt_commit_logs_fixer.go:43-70) */
int wv_graph_load_commitlog_dir(const char *dir, wv_graph **out);
int wv_graph_get_info(const wv_graph *g, wv_graph_info *info);
/* one node: *node_level = -1 for a nil node; up to cap links of `level` copied,
 * *n_links = the list length */
int wv_graph_node(const wv_graph *g, uint64_t id, int level, int *node_level, uint64_t *links, int cap, int *n_links);
/* The CSR of wv_index_upload_graph for n = info.n_slots nodes:
 * levels[n], layer0[n*deg0], upper_row[n], upper[info.n_upper*max(1,info.max_node_level)*degU],
 * tomb_bits[(n+63)/64] (nullable).  deg0 >= info.max_deg0, degU >= info.max_degU. */
int wv_graph_export_csr(wv_graph *g, int deg0, int degU, int8_t *levels, uint32_t *layer0, uint32_t *upper_row,
                        uint32_t *upper, uint64_t *tomb_bits);
/* The last AddPQ record's quantizer (deserializer.go ReadPQ :510-563): the
 * header, and for the KMeans encoder (encoder 1) the centroid table
 * [segments][centroids][dims/segments] of ReadKMeansEncoder :487-508 --
 * wv_index_set_pq's layout; copied when table_cap >= table_floats.  The tile
 * encoder (encoder 0) holds distribution parameters, not centres
 * (table_floats 0).  present = 0: the log is not compressed. */
typedef struct {
    int present, dims, segments, centroids, encoder, distribution, use_bits_encoding;
    uint64_t table_floats;
} wv_graph_pq;
int wv_graph_get_pq(const wv_graph *g, wv_graph_pq *pq, float *centroid_table, uint64_t table_cap);
int wv_graph_destroy(wv_graph *g);

/* Micro-batcher (SURVEY 8b "Threading"): SearchByVector is called once per
 * request from many threads (adapters/repos/db/index.go:988-1028 ->
 * shard_read.go:246-252).  wv_batcher_search blocks its caller while a
 * dispatcher thread coalesces up to max_batch waiting requests into one
 * wv_search_batch with per-query allow lists, then returns this caller's row:
 * the same result as wv_search_by_vector(ix, vector, k, allow_bits,
 * allow_nbits, ...).  Latency-first: one batch runs on the device at a time and
 * takes every request queued while the previous one ran, so a lone request
 * launches at once; max_wait_us > 0 lets the oldest request at an idle device
 * linger that long for company.  Two workers: one wakes a finished batch's
 * callers (each alone) while the other launches the next.  Destroy the
 * batcher before the index. */
typedef struct wv_batcher wv_batcher;
int wv_batcher_create(wv_index *ix, int dim, int max_batch, int max_wait_us, wv_batcher **out);
int wv_batcher_search(wv_batcher *b, const float *vector, int k, const uint64_t *allow_bits, uint64_t allow_nbits,
                      uint64_t *out_ids, float *out_dists, int32_t *out_n);
/* The same with the AllowList as strictly ascending ids (its Slice(),
 * helpers/allow_list.go:19-118): filtered == 0 means no list; filtered with
 * n_allow == 0 allows nothing.  The ids go straight into the batch's bitmap
 * row (no per-caller dense bitmap); a batch whose requests all carry the
 * same list sends it once. */
int wv_batcher_search_ids(wv_batcher *b, const float *vector, int k, int filtered, const uint64_t *allow_ids,
                          uint64_t n_allow, uint64_t *out_ids, float *out_dists, int32_t *out_n);
/* SearchByVectorDistance through the micro-batcher: concurrent callers with
 * the same maxLimit coalesce into one wv_search_by_vector_distance_batch.
 * out_cap entries at most are written; *out_n receives the full count. */
int wv_batcher_search_distance_ids(wv_batcher *b, const float *vector, float target_distance, int64_t max_limit,
                                   int filtered, const uint64_t *allow_ids, uint64_t n_allow, uint64_t *out_ids,
                                   float *out_dists, int64_t out_cap, int64_t *out_n);
int wv_batcher_stats(wv_batcher *b, uint64_t *requests, uint64_t *batches);
int wv_batcher_destroy(wv_batcher *b);

/* In-process multi-GPU group (adapters/repos/db/index.go:967-1044):
 * one wv_index per device, driven from one process (the Go server).
 *   WV_GROUP_SHARD    corpus split by id range (member i holds global ids
 *                     [base_i, base_i + cap_i), base_i a multiple of 64);
 *                     every member searches the batch over its shard, the
 *                     per-shard top-k lists are gathered on the first device
 *                     over RCCL (ncclCommInitAll, grouped ncclGather; device
 *                     copies when members share a device) and merged there.
 *   WV_GROUP_REPLICA  every member holds the whole corpus; a batch is split
 *                     into contiguous query ranges, one per member, no
 *                     collective.
 * The search has wv_search_batch's signature and result (global ids). */
typedef struct wv_group wv_group;
enum { WV_GROUP_SHARD = 0, WV_GROUP_REPLICA = 1 };
int wv_group_create(const int *devices, int n_devices, int dim, int metric, const wv_config *cfg, uint64_t capacity,
                    int layout, wv_group **out);
int wv_group_destroy(wv_group *g);
int wv_group_info(const wv_group *g, int *n_members, int *uses_rccl);
/* member i's index (for per-member uploads such as a graph), its id base and capacity */
int wv_group_member(wv_group *g, int i, wv_index **ix, uint64_t *id_base, uint64_t *capacity);
/* rows of global ids first_id.. routed to their shard (every replica) */
int wv_group_upload_vectors(wv_group *g, const float *rows, uint64_t n, uint64_t first_id);
/* every member builds the graph of its own rows (wv_index_build_graph), in parallel */
int wv_group_build_graph(wv_group *g, int ef_construction, uint64_t seed, int batch_div);
int wv_group_add(wv_group *g, const uint64_t *ids, const float *rows, uint64_t n);
int wv_group_add_tombstones(wv_group *g, const uint64_t *ids, uint64_t n);
int wv_group_remove_tombstones(wv_group *g, const uint64_t *ids, uint64_t n);
int wv_group_update_config(wv_group *g, const wv_config *cfg);
int wv_group_search_batch(wv_group *g, const float *queries, int nq, int k, int ef, const uint64_t *allow_bits,
                          uint64_t allow_nbits, uint64_t allow_stride_words, int mode, uint64_t *out_ids,
                          float *out_dists, int32_t *out_n);
/* SearchByVectorDistance over the group (wv_search_by_vector_distance_batch's
 * arguments): a shard group merges its members' answers by distance. */
int wv_group_search_by_vector_distance_batch(wv_group *g, const float *queries, int nq, const float *target_distances,
                                             int64_t max_limit, const uint64_t *allow_bits, uint64_t allow_nbits,
                                             uint64_t allow_stride_words, uint64_t *out_ids, float *out_dists,
                                             int64_t out_cap, int64_t *out_n);
/* the micro-batcher over a group (wv_batcher_search / _stats / _destroy as above) */
int wv_batcher_create_group(wv_group *g, int dim, int max_batch, int max_wait_us, wv_batcher **out);

/* GPU mirror of one shard's hnsw index -- the whole lifecycle the cgo
 * decorator (go/vector/gpu/gpu.go) drives, kept native so that the replay
 * harness (tests/native/mirror_replay.cpp) tests the code Go calls:
 *   startup   wv_mirror_post_startup{,_async}: the shard's commit log
 *             (<RootPath>/<ID>.hnsw.commitlog.d, replayed as restoreFromDisk,
 *             startup.go:56-152) becomes the mirror's graph, its rows come
 *             from the shard's VectorForIDThunk (shard.go:165,
 *             shard_read.go:145-161) as PostStartup's cache prefill does
 *             (startup.go:169-205); a node whose object is gone is skipped
 *             as search.go's handleDeletedNode path skips it (a nil node).
 *             The async form returns at once and builds on a background
 *             thread while the CPU index serves (the reference prefills its
 *             cache in a goroutine the same way, startup.go:174-203); writes
 *             that arrive meanwhile are kept and replayed when the new index
 *             is installed.  A PQ-compressed log (AddPQ record, KMeans
 *             encoder) is served compressed: the quantizer comes from the log,
 *             the codes are encoded on the device (compress.go:39-99,
 *             kmeans.go:78-110); a tile-encoded one stays on the CPU index;
 *   writes    wv_mirror_add (hnsw.Add, insert.go:43-65: the dimension is
 *             learnt from the first vector, capacity grows as
 *             growIndexToAccomodateNode does, maintainance.go:22-24,69-100),
 *             wv_mirror_delete (delete.go:29-84);
 *   reads     wv_mirror_search (SearchByVector through the micro-batcher, the
 *             allow list crossing as ascending ids, allow_list.go:19-118),
 *             wv_mirror_search_by_distance;
 *   compaction rows added since the last snapshot are searched exactly beside
 *             the graph (the delta set); past opt.compact_rows
 *             wv_mirror_needs_compaction turns true and wv_mirror_compact
 *             re-snapshots the graph from the (flushed) commit log -- the CPU
 *             index's own graph -- or, without a log directory, builds it on
 *             the device (wv_index_build_graph).
 * Any failed write marks the mirror stale: every read then returns
 * WV_ESTALE (the decorator answers from the CPU index).  With
 * opt.auto_resync the mirror heals itself: a background thread flushes the
 * CPU index's log through opt.flush and rebuilds as an async startup does,
 * backing off (1 s doubling to 60 s) while it keeps failing.  Reads and
 * writes may run concurrently from many threads; growth, compaction and
 * install are exclusive. */
typedef struct wv_mirror wv_mirror;
enum { WV_ESTALE = 6,      /* mirror not serving: answer from the CPU index */
       WV_ENOTFOUND = 7 }; /* vector source: no object for this doc id */
enum { WV_MIRROR_IDLE = 0, WV_MIRROR_STARTING = 1, WV_MIRROR_LIVE = 2, WV_MIRROR_STALE = 3 };
/* the CPU index's Flush (commit log to disk) before a resync reads the log */
typedef int (*wv_flush_fn)(void *ctx);
typedef struct {
    int dim;                   /* 0: learnt from the first vector */
    uint64_t initial_capacity; /* 0: 25000 (maintainance.go:22 initialSize) */
    int max_batch;             /* micro-batcher: queries per launch (0: 1024) */
    int max_wait_us;           /* micro-batcher linger at an idle device (0: none) */
    uint64_t compact_rows;     /* delta rows that ask for a compaction (0: 8192) */
    int ef_construction;       /* device-build compaction (0: 128) */
    uint64_t build_seed;       /* device-build level draw */
    const char *commitlog_dir; /* NULL: no commit log, compaction builds on the device */
    int auto_resync;           /* 1: a stale mirror rebuilds itself in the background */
    wv_flush_fn flush;         /* nullable: called before a resync reads the log */
    void *flush_ctx;
    int resync_backoff_ms;     /* first delay before a resync (0: 1000) */
} wv_mirror_options;
/* VectorForIDThunk for one doc id: WV_OK with *len = the vector's length
 * (copied to out when *len <= cap), WV_ENOTFOUND for a deleted object, any
 * other status is an error.  The async startup and resyncs call it from the
 * mirror's own thread: ctx must stay valid until wv_mirror_destroy. */
typedef int (*wv_vector_source)(void *ctx, uint64_t id, float *out, int cap, int *len);
typedef struct {
    int live;                  /* serving (state == WV_MIRROR_LIVE) */
    int dim;
    uint64_t capacity, n_rows, delta_rows, graph_nodes;
    uint64_t growths, compactions, startup_rows, startup_missing;
    uint64_t batcher_requests, batcher_batches;
    int state;                 /* WV_MIRROR_* */
    int pq;                    /* serving PQ-compressed (KMeans codes on the device) */
    uint64_t startups, resyncs, failed_startups, replayed_writes;
} wv_mirror_stats;
int wv_mirror_create(int metric, const wv_config *cfg, const wv_mirror_options *opt, wv_mirror **out);
int wv_mirror_post_startup(wv_mirror *m, wv_vector_source src, void *ctx);
int wv_mirror_post_startup_async(wv_mirror *m, wv_vector_source src, void *ctx);
/* WV_OK once live; WV_ESTALE if not live after timeout_ms (< 0: wait for the
 * running startup / resync to end) */
int wv_mirror_wait_live(wv_mirror *m, int timeout_ms);
/* the caller knows the mirror missed a write: stale now (resync if enabled) */
int wv_mirror_mark_stale(wv_mirror *m);
int wv_mirror_add(wv_mirror *m, uint64_t id, const float *vector, int len);
int wv_mirror_delete(wv_mirror *m, const uint64_t *ids, uint64_t n);
/* filtered != 0: allow_ids[n_allow] ascending doc ids (may be empty: nothing
 * allowed); filtered == 0: no allow list */
int wv_mirror_search(wv_mirror *m, const float *vector, int len, int k, int filtered, const uint64_t *allow_ids,
                     uint64_t n_allow, uint64_t *out_ids, float *out_dists, int32_t *out_n);
int wv_mirror_search_by_distance(wv_mirror *m, const float *vector, int len, float target_distance,
                                 int64_t max_limit, int filtered, const uint64_t *allow_ids, uint64_t n_allow,
                                 uint64_t *out_ids, float *out_dists, int64_t out_cap, int64_t *out_n);
int wv_mirror_update_config(wv_mirror *m, const wv_config *cfg);
int wv_mirror_needs_compaction(wv_mirror *m);
int wv_mirror_compact(wv_mirror *m);
int wv_mirror_get_stats(wv_mirror *m, wv_mirror_stats *st);
int wv_mirror_destroy(wv_mirror *m);

const char *wv_last_error(void);
const char *wv_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WVGPU_H */
