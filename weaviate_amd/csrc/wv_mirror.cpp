// wv_mirror.cpp -- the GPU mirror of one shard's hnsw index: startup from the
// shard's commit log and object store, writes, reads through the
// micro-batcher, capacity growth, delta compaction, staleness.  Host-only C++
// over the C ABI of include/wvgpu.h (no kernels).
//
// Reference lifecycle it mirrors (adapters/repos/db/vector/hnsw):
//   hnsw.New -> restoreFromDisk   startup.go:56-152  commit log -> nodes,
//                                 entrypoint, tombstones
//   PostStartup -> prefillCache   startup.go:169-205 vectors read through
//                                 VectorForIDThunk (shard_read.go:145-161)
//   Add                           insert.go:43-65    dims from the first vector
//                                                    (ValidateBeforeInsert),
//                                 growIndexToAccomodateNode
//                                 maintainance.go:22-24, 69-100
//   Delete                        delete.go:29-84    tombstones
//   SearchByVector / ...Distance  search.go:64-158
// The decorator in go/vector/gpu/gpu.go is a thin cgo binding of these calls.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/wvgpu.h"

extern "C" void wv_internal_set_error(const char* msg);

namespace {

constexpr uint64_t kInitialSize = 25000;        // maintainance.go:22
constexpr uint64_t kMinGrowthDelta = 25000;     // maintainance.go:23
constexpr double kGrowthRate = 1.25;            // maintainance.go:24
constexpr int kMaxDim = 65536;

int err(int code, const std::string& m) {
    wv_internal_set_error(m.c_str());
    return code;
}

// growIndexToAccomodateNode's size rule (maintainance.go:69-100)
uint64_t grown_size(uint64_t prev, uint64_t id) {
    uint64_t n = (kGrowthRate - 1) * (double)prev < (double)kMinGrowthDelta ? prev + kMinGrowthDelta
                                                                            : (uint64_t)((double)prev * kGrowthRate);
    if (n <= id) n = id + kMinGrowthDelta;
    return n;
}

inline bool bit(const std::vector<uint64_t>& b, uint64_t i) { return (i >> 6) < b.size() && (b[i >> 6] >> (i & 63) & 1); }
inline void set_bit(std::vector<uint64_t>& b, uint64_t i) {
    if ((i >> 6) >= b.size()) b.resize((i >> 6) + 1, 0);
    b[i >> 6] |= 1ull << (i & 63);
}

// The fixed-degree CSR of a replayed commit log, in wv_index_upload_graph's
// layout (the `upper` level stride re-laid to the entrypoint's max_level, as
// weaviate_amd/index.py upload_graph does).
struct Csr {
    uint64_t n = 0, n_upper = 0, entrypoint = 0;
    int deg0 = 0, degU = 1, max_level = 0, compressed = 0;
    std::vector<int8_t> levels;
    std::vector<uint32_t> layer0, upper_row, upper;
    std::vector<uint64_t> tomb;
};

int load_csr(const std::string& dir, int M, Csr& c) {
    wv_graph* g = nullptr;
    int rc = wv_graph_load_commitlog_dir(dir.c_str(), &g);
    if (rc) return rc;
    wv_graph_info info;
    rc = wv_graph_get_info(g, &info);
    if (rc) { wv_graph_destroy(g); return rc; }
    c.n = info.n_slots;
    c.compressed = info.compressed;
    c.entrypoint = info.entrypoint;
    c.max_level = info.max_level;
    c.n_upper = info.n_upper;
    if (c.n == 0 || c.compressed) { wv_graph_destroy(g); return WV_OK; }
    c.deg0 = std::max(2 * M, info.max_deg0);
    c.degU = std::max(std::max(M, info.max_degU), 1);
    const int ml_exp = std::max(1, info.max_node_level);
    c.levels.resize(c.n);
    c.layer0.resize(c.n * (size_t)c.deg0);
    c.upper_row.resize(c.n);
    std::vector<uint32_t> up(std::max<uint64_t>(1, c.n_upper) * (size_t)ml_exp * c.degU);
    c.tomb.resize((c.n + 63) / 64);
    rc = wv_graph_export_csr(g, c.deg0, c.degU, c.levels.data(), c.layer0.data(), c.upper_row.data(), up.data(),
                             c.tomb.data());
    wv_graph_destroy(g);
    if (rc) return rc;
    if (c.max_level > 0) {
        if (ml_exp == c.max_level) {
            c.upper.swap(up);
        } else {
            c.upper.assign(c.n_upper * (size_t)c.max_level * c.degU, 0xFFFFFFFFu);
            const int keep = std::min(ml_exp, c.max_level);
            for (uint64_t r = 0; r < c.n_upper; ++r)
                for (int l = 0; l < keep; ++l)
                    std::memcpy(&c.upper[(r * c.max_level + l) * c.degU], &up[(r * ml_exp + l) * c.degU],
                                sizeof(uint32_t) * c.degU);
        }
    }
    return WV_OK;
}

// Reader-writer lock that cannot starve its writer: 8 searchers holding it
// shared back to back would otherwise keep a compaction's snapshot upload
// (glibc's rwlock prefers readers) waiting for the whole run.
struct FairRW {
    std::shared_mutex rw;
    std::mutex gate;   // held by an exclusive locker from its arrival to its unlock
    void lock_shared() {
        { std::lock_guard<std::mutex> g(gate); }
        rw.lock_shared();
    }
    void unlock_shared() { rw.unlock_shared(); }
    void lock() {
        gate.lock();
        rw.lock();
    }
    void unlock() {
        rw.unlock();
        gate.unlock();
    }
};

}  // namespace

struct wv_mirror {
    int metric = 0;
    wv_config cfg{};
    wv_mirror_options opt{};
    std::string log_dir;
    // reads and writes shared; index creation, growth, snapshot uploads and
    // startup exclusive (the ABI forbids uploads racing searches)
    FairRW mu;
    std::mutex compact_mu;            // one compaction at a time
    std::mutex bm_mu;                 // the host bitmaps below
    wv_index* ix = nullptr;
    wv_batcher* b = nullptr;
    std::atomic<int> dim{0};
    std::atomic<uint64_t> capacity{0};
    std::atomic<bool> live{false};
    std::vector<uint64_t> have;       // ids holding a vector in the mirror
    std::vector<uint64_t> in_snap;    // ids that are nodes of the uploaded graph
    std::vector<uint64_t> tomb;       // ids deleted through the mirror
    std::atomic<uint64_t> delta{0};   // rows holding a vector that the graph does not hold
    uint64_t snap_nodes = 0;
    std::atomic<uint64_t> growths{0}, compactions{0}, startup_rows{0}, startup_missing{0};

    void drop_index() {
        if (b) wv_batcher_destroy(b);
        if (ix) wv_index_destroy(ix);
        b = nullptr;
        ix = nullptr;
        capacity = 0;
    }

    // exclusive lock held
    int create_index(int d, uint64_t cap) {
        if (d <= 0 || d > kMaxDim) return err(WV_EINVAL, "wv_mirror: bad vector length");
        int rc = wv_index_create(d, metric, &cfg, cap, &ix);
        if (rc) { ix = nullptr; return rc; }
        rc = wv_batcher_create(ix, d, opt.max_batch, opt.max_wait_us, &b);
        if (rc) { wv_index_destroy(ix); ix = nullptr; b = nullptr; return rc; }
        dim = d;
        capacity = cap;
        return WV_OK;
    }

    // exclusive lock held
    int grow_to(uint64_t id) {
        if (id < capacity) return WV_OK;
        const uint64_t n = grown_size(capacity, id);
        int rc = wv_index_reserve(ix, n);
        if (rc) return rc;
        capacity = n;
        growths++;
        return WV_OK;
    }

    uint64_t count_delta() {   // bm_mu held
        uint64_t d = 0;
        for (size_t w = 0; w < have.size(); ++w)
            d += (uint64_t)__builtin_popcountll(have[w] & ~(w < in_snap.size() ? in_snap[w] : 0ull));
        return d;
    }

    // exclusive lock held: c's graph becomes the index's; nodes whose row the
    // mirror does not hold are nil (search.go's not-found path skips them)
    int upload_snapshot(Csr& c, uint64_t* missing) {
        uint64_t miss = 0;
        {
            std::lock_guard<std::mutex> l(bm_mu);
            for (uint64_t i = 0; i < c.n; ++i)
                if (c.levels[i] >= 0 && !bit(have, i)) { c.levels[i] = -1; ++miss; }
        }
        if (missing) *missing = miss;
        if (c.levels[c.entrypoint] < 0)
            return err(WV_EDELETED, "wv_mirror: the commit log's entrypoint has no object");
        int rc = wv_index_upload_graph(ix, c.n, c.levels.data(), c.layer0.data(), c.deg0, c.upper_row.data(),
                                       c.max_level > 0 ? c.upper.data() : nullptr, c.n_upper, c.degU, c.max_level,
                                       c.entrypoint);
        if (rc) return rc;
        std::lock_guard<std::mutex> l(bm_mu);
        std::vector<uint64_t> t(std::max(tomb.size(), c.tomb.size()), 0);
        for (size_t w = 0; w < t.size(); ++w)
            t[w] = (w < tomb.size() ? tomb[w] : 0) | (w < c.tomb.size() ? c.tomb[w] : 0);
        if (c.n & 63 && !c.tomb.empty()) {   // bits past n in the log's last word are not tombstones
            const size_t w = c.tomb.size() - 1;
            t[w] = (w < tomb.size() ? tomb[w] : 0) | (c.tomb[w] & ((1ull << (c.n & 63)) - 1));
        }
        const uint64_t nb = std::min<uint64_t>(t.size() * 64, capacity);
        rc = wv_index_set_tombstones(ix, t.data(), nb);
        if (rc) return rc;
        in_snap.assign((c.n + 63) / 64, 0);
        for (uint64_t i = 0; i < c.n; ++i)
            if (c.levels[i] >= 0) in_snap[i >> 6] |= 1ull << (i & 63);
        snap_nodes = c.n;
        delta = count_delta();
        return WV_OK;
    }
};

extern "C" {

int wv_mirror_create(int metric, const wv_config* cfg, const wv_mirror_options* opt, wv_mirror** out) {
    if (!out || metric < 0 || metric > 2) return err(WV_EINVAL, "wv_mirror_create: bad argument");
    auto* m = new wv_mirror();
    m->metric = metric;
    if (cfg) m->cfg = *cfg; else wv_config_default(&m->cfg);
    if (opt) m->opt = *opt;
    if (m->opt.initial_capacity == 0) m->opt.initial_capacity = kInitialSize;
    if (m->opt.max_batch <= 0) m->opt.max_batch = 1024;
    if (m->opt.max_wait_us <= 0) m->opt.max_wait_us = 200;
    if (m->opt.compact_rows == 0) m->opt.compact_rows = 8192;
    if (m->opt.ef_construction <= 0) m->opt.ef_construction = 128;
    if (m->opt.commitlog_dir) m->log_dir = m->opt.commitlog_dir;
    m->opt.commitlog_dir = nullptr;   // (the caller's string is not retained)
    if (m->opt.dim < 0 || m->opt.dim > kMaxDim) { delete m; return err(WV_EINVAL, "wv_mirror_create: bad dim"); }
    m->dim = m->opt.dim;
    *out = m;
    return WV_OK;
}

// restoreFromDisk + PostStartup's prefill: the commit log's graph, every
// node's row from the vector source, the log's tombstones; then serving.
int wv_mirror_post_startup(wv_mirror* m, wv_vector_source src, void* ctx) {
    if (!m || !src) return err(WV_EINVAL, "wv_mirror_post_startup: bad argument");
    std::lock_guard<std::mutex> cl(m->compact_mu);
    std::unique_lock<FairRW> l(m->mu);
    m->live = false;
    m->drop_index();
    {
        std::lock_guard<std::mutex> bl(m->bm_mu);
        m->have.clear();
        m->in_snap.clear();
        m->tomb.clear();
        m->delta = 0;
        m->snap_nodes = 0;
    }
    Csr c;
    if (!m->log_dir.empty()) {
        int rc = load_csr(m->log_dir, m->cfg.max_connections, c);
        if (rc) return rc;
        if (c.compressed)   // the factory keeps PQ classes on the CPU index
            return err(WV_ESTATE, "wv_mirror: the commit log holds a PQ-compressed index");
    }
    int d = m->dim;
    if (d > 0) {
        int rc = m->create_index(d, std::max<uint64_t>(m->opt.initial_capacity, c.n));
        if (rc) return rc;
    }
    // rows in chunks (wv_index_add takes arbitrary ids: nil nodes and missing
    // objects leave holes)
    constexpr uint64_t CH = 8192;
    std::vector<float> buf(kMaxDim), rows;
    std::vector<uint64_t> ids;
    uint64_t got = 0, missing = 0;
    auto flush = [&]() -> int {
        if (ids.empty()) return WV_OK;
        int rc = wv_index_add(m->ix, ids.data(), rows.data(), ids.size());
        if (rc) return rc;
        std::lock_guard<std::mutex> bl(m->bm_mu);
        for (uint64_t id : ids) set_bit(m->have, id);
        ids.clear();
        rows.clear();
        return WV_OK;
    };
    for (uint64_t id = 0; id < c.n; ++id) {
        if (c.levels[id] < 0) continue;
        int len = 0;
        int rc = src(ctx, id, buf.data(), kMaxDim, &len);
        if (rc == WV_ENOTFOUND) { ++missing; continue; }
        if (rc) return err(rc, "wv_mirror_post_startup: vector source failed for id " + std::to_string(id));
        if (len <= 0 || len > kMaxDim) return err(WV_EINVAL, "wv_mirror_post_startup: bad vector length");
        if (!m->ix) {
            rc = m->create_index(len, std::max<uint64_t>(m->opt.initial_capacity, c.n));
            if (rc) return rc;
        }
        if (len != m->dim) return err(WV_EINVAL, "wv_mirror_post_startup: vector length differs from the index's");
        ids.push_back(id);
        rows.insert(rows.end(), buf.begin(), buf.begin() + len);
        ++got;
        if (ids.size() == CH && (rc = flush())) return rc;
    }
    if (int rc = flush()) return rc;
    m->startup_rows = got;
    m->startup_missing = missing;
    if (c.n > 0 && m->ix) {
        int rc = m->upload_snapshot(c, nullptr);
        if (rc) return rc;
    }
    m->live = true;
    return WV_OK;
}

int wv_mirror_add(wv_mirror* m, uint64_t id, const float* vector, int len) {
    if (!m || !vector || len <= 0) return err(WV_EINVAL, "wv_mirror_add: bad argument");
    if (id >= (1ull << 31) - 1) { m->live = false; return err(WV_EINVAL, "wv_mirror_add: id beyond the mirror's id space"); }
    for (;;) {
        {
            std::shared_lock<FairRW> l(m->mu);
            if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
            if (m->ix && id < m->capacity) {
                if (len != m->dim) {   // ValidateBeforeInsert would have refused it (insert.go:27-41)
                    m->live = false;
                    return err(WV_EINVAL, "wv_mirror_add: vector length differs from the index's");
                }
                int rc = wv_index_add(m->ix, &id, vector, 1);
                if (rc) { m->live = false; return rc; }
                std::lock_guard<std::mutex> bl(m->bm_mu);
                if (!bit(m->have, id)) {
                    set_bit(m->have, id);
                    if (!bit(m->in_snap, id)) m->delta++;
                }
                return WV_OK;
            }
        }
        // first vector (dims) or an id past the capacity: exclusive
        std::unique_lock<FairRW> l(m->mu);
        if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
        int rc = WV_OK;
        if (!m->ix) rc = m->create_index(len, std::max<uint64_t>(m->opt.initial_capacity, id + 1));
        else if (id >= m->capacity) rc = m->grow_to(id);
        if (rc) { m->live = false; return rc; }
    }
}

int wv_mirror_delete(wv_mirror* m, const uint64_t* ids, uint64_t n) {
    if (!m || (n && !ids)) return err(WV_EINVAL, "wv_mirror_delete: bad argument");
    std::shared_lock<FairRW> l(m->mu);
    if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
    std::vector<uint64_t> in;
    in.reserve(n);
    {
        std::lock_guard<std::mutex> bl(m->bm_mu);
        for (uint64_t i = 0; i < n; ++i) {
            set_bit(m->tomb, ids[i]);   // kept for later snapshots and growth
            if (ids[i] < m->capacity) in.push_back(ids[i]);
        }
    }
    if (in.empty() || !m->ix) return WV_OK;
    int rc = wv_index_add_tombstones(m->ix, in.data(), in.size());
    if (rc) m->live = false;
    return rc;
}

namespace {
// the AllowList's ids as the bitmap of the ABI (ids past the capacity hold no
// row: dropped)
void allow_bitmap(const uint64_t* ids, uint64_t n, uint64_t cap, std::vector<uint64_t>& bits, uint64_t& nbits) {
    uint64_t hi = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (ids[i] < cap) hi = std::max(hi, ids[i] + 1);
    nbits = std::max<uint64_t>(hi, 1);
    bits.assign((nbits + 63) / 64, 0);
    for (uint64_t i = 0; i < n; ++i)
        if (ids[i] < cap) bits[ids[i] >> 6] |= 1ull << (ids[i] & 63);
}
}  // namespace

int wv_mirror_search(wv_mirror* m, const float* vector, int len, int k, int filtered, const uint64_t* allow_ids,
                     uint64_t n_allow, uint64_t* out_ids, float* out_dists, int32_t* out_n) {
    if (!m || !vector || k <= 0 || !out_ids || !out_dists || !out_n || (n_allow && !allow_ids))
        return err(WV_EINVAL, "wv_mirror_search: bad argument");
    if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");   // (not waiting out a startup)
    std::shared_lock<FairRW> l(m->mu);
    if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
    if (!m->ix) { *out_n = 0; return WV_OK; }   // empty index (search.go:463-465)
    if (len != m->dim) return err(WV_ESTALE, "wv_mirror_search: vector length differs from the index's");
    // ids past the capacity hold no row: the list is cut there (ascending)
    const uint64_t cap = m->capacity;
    while (n_allow && allow_ids[n_allow - 1] >= cap) --n_allow;
    return wv_batcher_search_ids(m->b, vector, k, filtered, allow_ids, n_allow, out_ids, out_dists, out_n);
}

int wv_mirror_search_by_distance(wv_mirror* m, const float* vector, int len, float target_distance,
                                 int64_t max_limit, int filtered, const uint64_t* allow_ids, uint64_t n_allow,
                                 uint64_t* out_ids, float* out_dists, int64_t out_cap, int64_t* out_n) {
    if (!m || !vector || !out_n || (n_allow && !allow_ids)) return err(WV_EINVAL, "wv_mirror_search_by_distance: bad argument");
    if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
    std::shared_lock<FairRW> l(m->mu);
    if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
    if (!m->ix) { *out_n = 0; return WV_OK; }
    if (len != m->dim) return err(WV_ESTALE, "wv_mirror_search_by_distance: vector length differs from the index's");
    std::vector<uint64_t> bits;
    uint64_t nbits = 0;
    if (filtered) allow_bitmap(allow_ids, n_allow, m->capacity, bits, nbits);
    return wv_search_by_vector_distance(m->ix, vector, target_distance, max_limit, filtered ? bits.data() : nullptr,
                                        nbits, out_ids, out_dists, out_cap, out_n);
}

int wv_mirror_update_config(wv_mirror* m, const wv_config* cfg) {
    if (!m || !cfg) return err(WV_EINVAL, "wv_mirror_update_config: bad argument");
    std::shared_lock<FairRW> l(m->mu);
    const int dev = m->cfg.device;
    m->cfg = *cfg;
    m->cfg.device = dev;
    if (!m->ix) return WV_OK;
    int rc = wv_index_update_config(m->ix, cfg);
    if (rc) m->live = false;
    return rc;
}

int wv_mirror_needs_compaction(wv_mirror* m) {
    return m && m->live && m->ix && m->delta.load() >= m->opt.compact_rows ? 1 : 0;
}

// Re-snapshot: the graph of the flushed commit log (the CPU index's own
// graph; rows added since stay in the delta), or a device build.
int wv_mirror_compact(wv_mirror* m) {
    if (!m) return err(WV_EINVAL, "wv_mirror_compact: bad argument");
    std::lock_guard<std::mutex> cl(m->compact_mu);
    if (!m->live) return err(WV_ESTALE, "wv_mirror: stale");
    if (!m->log_dir.empty()) {
        Csr c;   // read without blocking searches
        int rc = load_csr(m->log_dir, m->cfg.max_connections, c);
        if (rc) return rc;
        if (c.compressed) { m->live = false; return err(WV_ESTATE, "wv_mirror: the commit log became PQ-compressed"); }
        if (c.n == 0) return WV_OK;
        std::unique_lock<FairRW> l(m->mu);
        if (!m->live || !m->ix) return err(WV_ESTALE, "wv_mirror: stale");
        if ((rc = m->grow_to(c.n - 1))) { m->live = false; return rc; }
        rc = m->upload_snapshot(c, nullptr);
        if (rc == WV_EDELETED) return rc;   // the old snapshot keeps serving
        if (rc) { m->live = false; return rc; }
        m->compactions++;
        return WV_OK;
    }
    std::unique_lock<FairRW> l(m->mu);
    if (!m->live || !m->ix) return err(WV_ESTALE, "wv_mirror: stale");
    int rc = wv_index_build_graph(m->ix, m->opt.ef_construction, m->opt.build_seed, 32);
    if (rc) return rc;   // e.g. holes below n_rows: the delta keeps serving exactly
    uint64_t n = 0;
    wv_index_graph_info(m->ix, &n, nullptr, nullptr, nullptr, nullptr, nullptr);
    std::lock_guard<std::mutex> bl(m->bm_mu);
    m->in_snap.assign((n + 63) / 64, 0);
    for (uint64_t i = 0; i < n; ++i)
        if (bit(m->have, i)) m->in_snap[i >> 6] |= 1ull << (i & 63);
    m->snap_nodes = n;
    m->delta = m->count_delta();
    m->compactions++;
    return WV_OK;
}

int wv_mirror_get_stats(wv_mirror* m, wv_mirror_stats* st) {
    if (!m || !st) return err(WV_EINVAL, "wv_mirror_get_stats: bad argument");
    std::memset(st, 0, sizeof(*st));
    std::shared_lock<FairRW> l(m->mu);
    st->live = m->live ? 1 : 0;
    st->dim = m->dim;
    st->capacity = m->capacity;
    st->delta_rows = m->delta;
    st->graph_nodes = m->snap_nodes;
    st->growths = m->growths;
    st->compactions = m->compactions;
    st->startup_rows = m->startup_rows;
    st->startup_missing = m->startup_missing;
    if (m->ix) wv_index_capacity(m->ix, nullptr, &st->n_rows);
    if (m->b) wv_batcher_stats(m->b, &st->batcher_requests, &st->batcher_batches);
    return WV_OK;
}

int wv_mirror_destroy(wv_mirror* m) {
    if (!m) return WV_OK;
    {
        std::lock_guard<std::mutex> cl(m->compact_mu);
        std::unique_lock<FairRW> l(m->mu);
        m->live = false;
        m->drop_index();
    }
    delete m;
    return WV_OK;
}

}  // extern "C"
