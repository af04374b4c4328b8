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
//   compressed classes            compress.go:39-99  the AddPQ record's KMeans
//                                 centres; codes encoded on the device
// The decorator in go/vector/gpu/gpu.go is a thin cgo binding of these calls.
//
// States: IDLE -> STARTING (a startup builds a new index off-lock: the log,
// the rows, the graph) -> LIVE (installed under the exclusive lock, with the
// writes that arrived meanwhile replayed) -> STALE (a write failed) ->
// STARTING again when auto_resync is on (a background thread, backing off).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wvgpu.h"

extern "C" void wv_internal_set_error(const char* msg);

// condition-variable deadlines on steady_clock (pthread_cond_clockwait); the
// ThreadSanitizer build (tests/native/Makefile mirror_replay_tsan) uses
// system_clock, whose pthread_cond_timedwait GCC 11's libtsan intercepts --
// it has no pthread_cond_clockwait interceptor, so every steady wait would
// look like a lock never released
#ifdef WV_TSAN_BUILD
using wait_clock = std::chrono::system_clock;
#else
using wait_clock = std::chrono::steady_clock;
#endif

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
    wv_graph_pq pq{};
    std::vector<float> pq_table;
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
    if (c.compressed) {
        wv_graph_get_pq(g, &c.pq, nullptr, 0);
        c.pq_table.resize(c.pq.table_floats);
        wv_graph_get_pq(g, &c.pq, c.pq_table.data(), c.pq_table.size());
    }
    if (c.n == 0) { wv_graph_destroy(g); return WV_OK; }
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

// The log's entrypoint whose object is gone: the reference's search would
// fail on it until the tombstone cleanup reassigns it (search.go:467-476,
// delete.go:281-411).  The mirror instead enters at the live node of the
// highest level (lowest id among equal ones), the upper layers re-laid to
// that level; no live node at all: no graph (every row is served exactly).
// Returns false when the graph is empty.
bool repair_entrypoint(Csr& c) {
    if (c.n == 0) return false;
    if (c.levels[c.entrypoint] >= 0) return true;
    int best = -1;
    uint64_t ep = 0;
    for (uint64_t i = 0; i < c.n; ++i)
        if (c.levels[i] > best) { best = c.levels[i]; ep = i; }
    if (best < 0) return false;
    c.entrypoint = ep;
    const int nl = std::min(best, c.max_level);
    if (nl < c.max_level && c.max_level > 0) {
        std::vector<uint32_t> up(std::max<uint64_t>(1, c.n_upper) * (size_t)std::max(nl, 1) * c.degU, 0xFFFFFFFFu);
        for (uint64_t r = 0; r < c.n_upper && nl > 0; ++r)
            for (int l = 0; l < nl; ++l)
                std::memcpy(&up[(r * nl + l) * c.degU], &c.upper[(r * c.max_level + l) * c.degU], sizeof(uint32_t) * c.degU);
        c.upper.swap(up);
    }
    c.max_level = nl;
    return true;
}

}  // namespace

struct wv_mirror {
    int metric = 0;
    std::mutex cfg_mu;                // cfg (update_config vs startups and compactions)
    wv_config cfg{};
    wv_mirror_options opt{};
    std::string log_dir;
    // reads and writes shared; index install, growth and snapshot uploads
    // exclusive (the ABI forbids uploads racing searches)
    FairRW mu;
    std::mutex compact_mu;            // one compaction or startup build at a time
    std::mutex bm_mu;                 // the host bitmaps below
    wv_index* ix = nullptr;
    wv_batcher* b = nullptr;
    std::atomic<int> dim{0};
    std::atomic<uint64_t> capacity{0};
    std::atomic<int> state{WV_MIRROR_IDLE};
    std::atomic<bool> pq{false};
    // the log's entrypoint has no object (its row is gone from the store):
    // the device graph runs from a live replacement, but every search that
    // would take the HNSW path answers WV_EDELETED as knnSearchByVector does
    // (search.go:467-476) until a compaction reads a log whose entrypoint
    // the CPU index's cleanup has moved
    std::atomic<bool> ep_gone{false};
    std::vector<uint64_t> have;       // ids holding a vector in the mirror
    std::vector<uint64_t> in_snap;    // ids that are nodes of the uploaded graph
    std::vector<uint64_t> tomb;       // ids deleted through the mirror (never cleared: doc ids are not reused)
    std::atomic<uint64_t> delta{0};   // live rows holding a vector that the graph does not hold
    uint64_t snap_nodes = 0;
    std::atomic<uint64_t> growths{0}, compactions{0}, startup_rows{0}, startup_missing{0};
    std::atomic<uint64_t> startups{0}, resyncs{0}, failed_startups{0}, replayed{0};
    // writes that arrive while a startup builds (replayed at install)
    std::mutex pend_mu;
    std::vector<uint64_t> pend_ids;
    std::vector<int> pend_len;
    std::vector<float> pend_rows;
    // the vector source of the last startup, for resyncs
    wv_vector_source src = nullptr;
    void* src_ctx = nullptr;
    // background startups and resyncs
    std::mutex wk_mu;
    std::condition_variable wk_cv;
    std::thread worker;
    bool want_start = false, resync_next = false, busy = false;
    // a startup posted while another build ran (wv_mirror_post_startup_async
    // does not wait for it: its Go caller may hold the lock the running
    // resync's flush callback takes): the worker adopts this source and
    // starts it after the current install
    bool fresh_pending = false;
    wv_vector_source next_src = nullptr;
    void* next_ctx = nullptr;
    std::atomic<bool> stop{false};
    int backoff_ms = 0;
    // failure injection for the replay harness: hold the worker this long
    // between a startup's install (state LIVE) and busy = false, the window
    // in which a failed write used to lose its resync
    int test_post_install_ms = 0;

    bool live() const { return state.load() == WV_MIRROR_LIVE; }
    // SearchByVector's dispatch (search.go:74-78): only a flat search runs
    // without the entrypoint
    int check_entrypoint(int filtered, uint64_t n_allow) {
        if (!ep_gone) return WV_OK;
        const wv_config c = config();
        if (filtered && !c.forbid_flat && (int64_t)n_allow < c.flat_search_cutoff) return WV_OK;
        return err(WV_EDELETED, "entrypoint was deleted in the object store, it has been flagged for cleanup and "
                                "should be fixed in the next cleanup cycle");
    }
    wv_config config() {
        std::lock_guard<std::mutex> l(cfg_mu);
        return cfg;
    }

    void drop_index() {
        if (b) wv_batcher_destroy(b);
        if (ix) wv_index_destroy(ix);
        b = nullptr;
        ix = nullptr;
        capacity = 0;
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

    uint64_t count_delta() {   // bm_mu held: rows beside the graph, tombstoned ones excluded
        uint64_t d = 0;
        for (size_t w = 0; w < have.size(); ++w)
            d += (uint64_t)__builtin_popcountll(have[w] & ~(w < in_snap.size() ? in_snap[w] : 0ull) &
                                                ~(w < tomb.size() ? tomb[w] : 0ull));
        return d;
    }

    // the union of the mirror's and a log's tombstones, as the index's bitmap (bm_mu held)
    std::vector<uint64_t> tomb_union(const Csr& c, uint64_t cap) {
        std::vector<uint64_t> t(std::max(tomb.size(), c.tomb.size()), 0);
        for (size_t w = 0; w < t.size(); ++w) t[w] = w < tomb.size() ? tomb[w] : 0;
        for (size_t w = 0; w < c.tomb.size(); ++w) {
            uint64_t lw = c.tomb[w];
            if (w == c.tomb.size() - 1 && (c.n & 63)) lw &= (1ull << (c.n & 63)) - 1;   // bits past n: no node
            t[w] |= lw;
        }
        t.resize(std::min<uint64_t>(t.size(), (cap + 63) / 64));
        return t;
    }

    // a compressed log: the quantizer from its AddPQ record, codes encoded
    // on the device (rows added later are encoded on write)
    int enable_pq(wv_index* x, const Csr& c, int d) {
        if (c.pq.encoder != WV_PQ_KMEANS)
            return err(WV_ESTATE, "wv_mirror: a tile-encoded PQ index stays on the CPU index");
        if (c.pq.dims != d || c.pq.segments <= 0 || c.pq_table.size() != (size_t)c.pq.centroids * d)
            return err(WV_ESTATE, "wv_mirror: the AddPQ record does not match the index");
        int rc = wv_index_set_pq(x, c.pq.segments, c.pq.centroids, c.pq.use_bits_encoding, WV_PQ_KMEANS,
                                 c.pq_table.data());
        if (!rc) rc = wv_index_pq_encode(x);
        if (!rc) rc = wv_index_set_compressed(x, 1);
        return rc;
    }

    // graph of c into x (exclusive access to x): nil for nodes without a row,
    // the entrypoint repaired; sets in_snap / snap_nodes of the caller's copy
    int upload_graph(wv_index* x, Csr& c, const std::vector<uint64_t>& have_rows, std::vector<uint64_t>& snap,
                     uint64_t& nodes, bool& gone) {
        for (uint64_t i = 0; i < c.n; ++i)
            if (c.levels[i] >= 0 && !bit(have_rows, i)) c.levels[i] = -1;
        snap.assign((c.n + 63) / 64, 0);
        nodes = 0;
        gone = c.n > 0 && c.levels[c.entrypoint] < 0;
        if (!repair_entrypoint(c)) return WV_OK;   // no live node: every row stays in the delta
        int rc = wv_index_upload_graph(x, c.n, c.levels.data(), c.layer0.data(), c.deg0, c.upper_row.data(),
                                       c.max_level > 0 ? c.upper.data() : nullptr, c.n_upper, c.degU, c.max_level,
                                       c.entrypoint);
        if (rc) return rc;
        for (uint64_t i = 0; i < c.n; ++i)
            if (c.levels[i] >= 0) snap[i >> 6] |= 1ull << (i & 63);
        nodes = c.n;
        return WV_OK;
    }

    // ---- startup: build off-lock, install under the exclusive lock ----
    struct Built {
        wv_index* ix = nullptr;
        wv_batcher* b = nullptr;
        int dim = 0;
        uint64_t capacity = 0, nodes = 0, rows = 0, missing = 0;
        bool pq = false, ep_gone = false;
        std::vector<uint64_t> have, in_snap;
        Csr c;
        void release() {
            if (b) wv_batcher_destroy(b);
            if (ix) wv_index_destroy(ix);
            b = nullptr;
            ix = nullptr;
        }
    };

    int create_into(Built& nb, int d, uint64_t cap) {
        if (d <= 0 || d > kMaxDim) return err(WV_EINVAL, "wv_mirror: bad vector length");
        const wv_config cf = config();
        int rc = wv_index_create(d, metric, &cf, cap, &nb.ix);
        if (rc) { nb.ix = nullptr; return rc; }
        rc = wv_batcher_create(nb.ix, d, opt.max_batch, opt.max_wait_us, &nb.b);
        if (rc) { nb.b = nullptr; return rc; }
        nb.dim = d;
        nb.capacity = cap;
        return WV_OK;
    }

    int build(Built& nb) {   // compact_mu held, no mirror lock
        Csr& c = nb.c;
        if (!log_dir.empty()) {
            int rc = load_csr(log_dir, config().max_connections, c);
            if (rc) return rc;
        }
        int d = dim;
        const uint64_t cap0 = std::max<uint64_t>(opt.initial_capacity, c.n);
        if (d > 0) {
            int rc = create_into(nb, d, cap0);
            if (rc) return rc;
        }
        // rows in chunks (wv_index_add takes arbitrary ids: nil nodes and
        // missing objects leave holes)
        constexpr uint64_t CH = 8192;
        std::vector<float> buf(kMaxDim), rows;
        std::vector<uint64_t> ids;
        auto flush_rows = [&]() -> int {
            if (ids.empty()) return WV_OK;
            int rc = wv_index_add(nb.ix, ids.data(), rows.data(), ids.size());
            if (rc) return rc;
            for (uint64_t id : ids) set_bit(nb.have, id);
            ids.clear();
            rows.clear();
            return WV_OK;
        };
        for (uint64_t id = 0; id < c.n; ++id) {
            if (c.levels[id] < 0) continue;
            if ((id & 1023) == 0 && stop) return err(WV_ESTATE, "wv_mirror: destroyed during startup");
            int len = 0;
            int rc = src(src_ctx, id, buf.data(), kMaxDim, &len);
            if (rc == WV_ENOTFOUND) { ++nb.missing; continue; }
            if (rc) return err(rc, "wv_mirror startup: vector source failed for id " + std::to_string(id));
            if (len <= 0 || len > kMaxDim) return err(WV_EINVAL, "wv_mirror startup: bad vector length");
            if (!nb.ix && (rc = create_into(nb, len, cap0))) return rc;
            if (len != nb.dim) return err(WV_EINVAL, "wv_mirror startup: vector length differs from the index's");
            ids.push_back(id);
            rows.insert(rows.end(), buf.begin(), buf.begin() + len);
            ++nb.rows;
            if (ids.size() == CH && (rc = flush_rows())) return rc;
        }
        if (int rc = flush_rows()) return rc;
        if (!nb.ix) return WV_OK;   // nothing to learn the dimension from yet
        if (c.compressed) {
            if (int rc = enable_pq(nb.ix, c, nb.dim)) return rc;
            nb.pq = true;
        }
        if (c.n > 0) {
            if (int rc = upload_graph(nb.ix, c, nb.have, nb.in_snap, nb.nodes, nb.ep_gone)) return rc;
        }
        return WV_OK;
    }

    // exclusive lock + pend_mu held: the built index replaces the old one;
    // the writes that arrived meanwhile are replayed on it
    int install(Built& nb) {
        drop_index();
        ix = nb.ix;
        b = nb.b;
        nb.ix = nullptr;
        nb.b = nullptr;
        if (nb.dim) dim = nb.dim;
        capacity = nb.capacity;
        pq = nb.pq;
        ep_gone = nb.ep_gone;
        {
            std::lock_guard<std::mutex> bl(bm_mu);
            have.swap(nb.have);
            in_snap.swap(nb.in_snap);
            snap_nodes = nb.nodes;
        }
        startup_rows = nb.rows;
        startup_missing = nb.missing;
        for (size_t i = 0, off = 0; i < pend_ids.size(); off += pend_len[i], ++i) {
            const uint64_t id = pend_ids[i];
            const int len = pend_len[i];
            int rc = WV_OK;
            if (!ix) {
                Built fresh;
                rc = create_into(fresh, len, std::max<uint64_t>(opt.initial_capacity, id + 1));
                if (rc) { fresh.release(); return rc; }
                ix = fresh.ix; b = fresh.b; dim = len; capacity = fresh.capacity;
            }
            if (len != dim) return err(WV_EINVAL, "wv_mirror: a write during startup has another vector length");
            if (id >= capacity && (rc = grow_to(id))) return rc;
            if ((rc = wv_index_add(ix, &id, &pend_rows[off], 1))) return rc;
            std::lock_guard<std::mutex> bl(bm_mu);
            set_bit(have, id);
            replayed++;
        }
        pend_ids.clear();
        pend_len.clear();
        pend_rows.clear();
        if (ix) {
            const wv_config cf = config();   // (a config update during the build)
            int rc = wv_index_update_config(ix, &cf);
            if (rc) return rc;
            std::lock_guard<std::mutex> bl(bm_mu);
            const std::vector<uint64_t> t = tomb_union(nb.c, capacity);
            if (!t.empty() && (rc = wv_index_set_tombstones(ix, t.data(), std::min<uint64_t>(t.size() * 64, capacity))))
                return rc;
            delta = count_delta();
        }
        return WV_OK;
    }

    void begin_start() {   // writes from now on are kept for the install
        std::lock_guard<std::mutex> pl(pend_mu);
        state = WV_MIRROR_STARTING;
        pend_ids.clear();
        pend_len.clear();
        pend_rows.clear();
    }

    // one startup (state already STARTING)
    int run_startup() {
        std::lock_guard<std::mutex> cl(compact_mu);
        Built nb;
        int rc = build(nb);
        if (!rc) {
            std::unique_lock<FairRW> l(mu);
            std::lock_guard<std::mutex> pl(pend_mu);
            if (stop) rc = err(WV_ESTATE, "wv_mirror: destroyed during startup");
            else if ((rc = install(nb)) == WV_OK) state = WV_MIRROR_LIVE;
            if (rc) {
                drop_index();
                state = WV_MIRROR_STALE;
            }
        } else {
            std::lock_guard<std::mutex> pl(pend_mu);
            state = WV_MIRROR_STALE;
        }
        nb.release();
        startups++;
        if (rc) failed_startups++;
        return rc;
    }

    // ---- the background thread: async startups and resyncs ----
    void ensure_worker() {   // wk_mu held
        if (!worker.joinable()) worker = std::thread([this] { worker_loop(); });
    }
    void worker_loop() {
        std::unique_lock<std::mutex> l(wk_mu);
        for (;;) {
            wk_cv.wait(l, [&] { return stop.load() || want_start; });
            if (stop) return;
            bool resync = resync_next;
            want_start = false;
            resync_next = false;
            if (fresh_pending) {   // (a posted startup supersedes a queued resync)
                fresh_pending = false;
                resync = false;
                src = next_src;
                src_ctx = next_ctx;
                begin_start();   // (wk_mu -> pend_mu: no path takes them the other way)
            }
            if (resync) {
                const int delay = backoff_ms;
                if (delay > 0 && wk_cv.wait_until(l, wait_clock::now() + std::chrono::milliseconds(delay), [&] { return stop.load(); }))
                    return;
                if (state.load() != WV_MIRROR_STALE) continue;   // (a manual startup got there first)
            }
            busy = true;
            l.unlock();
            int rc = WV_OK;
            if (resync) {
                begin_start();
                if (opt.flush && opt.flush(opt.flush_ctx) != 0) {
                    rc = err(WV_ESTATE, "wv_mirror: the CPU index's flush failed");
                    std::lock_guard<std::mutex> pl(pend_mu);
                    state = WV_MIRROR_STALE;
                }
            }
            if (!rc) rc = run_startup();
            if (!rc && resync) resyncs++;
            if (test_post_install_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(test_post_install_ms));
            l.lock();
            busy = false;
            if (rc) {
                backoff_ms = std::min(60000, std::max(opt.resync_backoff_ms, 2 * backoff_ms));
                if (opt.auto_resync && src && !stop) { want_start = true; resync_next = true; }
            } else {
                backoff_ms = 0;
                // a write that failed between the install (state LIVE) and
                // busy = false marked the mirror stale while request_resync
                // saw busy and returned: schedule that resync here, or no
                // later failure would (mark_stale only acts on LIVE)
                if (state.load() == WV_MIRROR_STALE && opt.auto_resync && src && !stop && !want_start) {
                    want_start = true;
                    resync_next = true;
                    backoff_ms = opt.resync_backoff_ms;
                }
            }
            wk_cv.notify_all();
        }
    }
    void request_resync() {   // after a failed write
        if (!opt.auto_resync || !src || stop) return;
        std::lock_guard<std::mutex> l(wk_mu);
        if (want_start || busy) return;
        want_start = true;
        resync_next = true;
        backoff_ms = std::max(backoff_ms, opt.resync_backoff_ms);
        ensure_worker();
        wk_cv.notify_all();
    }
    void mark_stale() {
        int s = WV_MIRROR_LIVE;
        if (state.compare_exchange_strong(s, WV_MIRROR_STALE)) request_resync();
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
    if (m->opt.max_wait_us < 0) m->opt.max_wait_us = 0;
    if (m->opt.compact_rows == 0) m->opt.compact_rows = 8192;
    if (m->opt.ef_construction <= 0) m->opt.ef_construction = 128;
    if (m->opt.resync_backoff_ms <= 0) m->opt.resync_backoff_ms = 1000;
    if (m->opt.commitlog_dir) m->log_dir = m->opt.commitlog_dir;
    m->opt.commitlog_dir = nullptr;   // (the caller's string is not retained)
    if (m->opt.dim < 0 || m->opt.dim > kMaxDim) { delete m; return err(WV_EINVAL, "wv_mirror_create: bad dim"); }
    m->dim = m->opt.dim;
    if (const char* e = std::getenv("WV_MIRROR_TEST_POST_INSTALL_MS")) m->test_post_install_ms = std::atoi(e);
    *out = m;
    return WV_OK;
}

// restoreFromDisk + PostStartup's prefill on the caller's thread
int wv_mirror_post_startup(wv_mirror* m, wv_vector_source src, void* ctx) {
    if (!m || !src) return err(WV_EINVAL, "wv_mirror_post_startup: bad argument");
    {
        std::unique_lock<std::mutex> l(m->wk_mu);   // (no background startup at the same time)
        m->wk_cv.wait(l, [&] { return !m->busy; });
        m->want_start = false;
        m->src = src;
        m->src_ctx = ctx;
    }
    m->begin_start();
    return m->run_startup();
}

// the same on the mirror's thread (startup.go:174-203 prefills in a
// goroutine): returns at once; reads answer WV_ESTALE until it is installed
int wv_mirror_post_startup_async(wv_mirror* m, wv_vector_source src, void* ctx) {
    if (!m || !src) return err(WV_EINVAL, "wv_mirror_post_startup_async: bad argument");
    std::unique_lock<std::mutex> l(m->wk_mu);
    if (m->busy) {
        // a startup or resync in flight installs first (begin_start would
        // clear the writes queued for that install, and run_startup assumes
        // STARTING): the worker starts this one after it.  No wait here --
        // the running build may call the flush callback, which takes the
        // caller's lock (PostStartup holds g.mu)
        m->next_src = src;
        m->next_ctx = ctx;
        m->fresh_pending = true;
        m->want_start = true;
        m->resync_next = false;
        m->wk_cv.notify_all();
        return WV_OK;
    }
    m->src = src;
    m->src_ctx = ctx;
    m->begin_start();
    m->want_start = true;
    m->resync_next = false;
    m->ensure_worker();
    m->wk_cv.notify_all();
    return WV_OK;
}

int wv_mirror_wait_live(wv_mirror* m, int timeout_ms) {
    if (!m) return err(WV_EINVAL, "wv_mirror_wait_live: bad argument");
    std::unique_lock<std::mutex> l(m->wk_mu);
    auto done = [&] { return (m->live() && !m->fresh_pending) || (!m->busy && !m->want_start); };
    if (timeout_ms < 0) m->wk_cv.wait(l, done);
    else m->wk_cv.wait_until(l, wait_clock::now() + std::chrono::milliseconds(timeout_ms), done);
    return m->live() ? WV_OK : err(WV_ESTALE, "wv_mirror: not live");
}

int wv_mirror_mark_stale(wv_mirror* m) {
    if (!m) return err(WV_EINVAL, "wv_mirror_mark_stale: bad argument");
    m->mark_stale();
    return WV_OK;
}

int wv_mirror_add(wv_mirror* m, uint64_t id, const float* vector, int len) {
    if (!m || !vector || len <= 0) return err(WV_EINVAL, "wv_mirror_add: bad argument");
    if (id >= (1ull << 31) - 1) { m->mark_stale(); return err(WV_EINVAL, "wv_mirror_add: id beyond the mirror's id space"); }
    {
        std::lock_guard<std::mutex> pl(m->pend_mu);
        if (m->state == WV_MIRROR_STARTING) {   // kept for the install
            m->pend_ids.push_back(id);
            m->pend_len.push_back(len);
            m->pend_rows.insert(m->pend_rows.end(), vector, vector + len);
            return WV_OK;
        }
    }
    for (;;) {
        {
            std::shared_lock<FairRW> l(m->mu);
            if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");
            if (m->ix && id < m->capacity) {
                if (len != m->dim) {   // ValidateBeforeInsert would have refused it (insert.go:27-41)
                    m->mark_stale();
                    return err(WV_EINVAL, "wv_mirror_add: vector length differs from the index's");
                }
                int rc = wv_index_add(m->ix, &id, vector, 1);
                if (rc) { m->mark_stale(); return rc; }
                std::lock_guard<std::mutex> bl(m->bm_mu);
                if (!bit(m->have, id)) {
                    set_bit(m->have, id);
                    if (!bit(m->in_snap, id) && !bit(m->tomb, id)) m->delta++;
                }
                return WV_OK;
            }
        }
        // first vector (dims) or an id past the capacity: exclusive
        std::unique_lock<FairRW> l(m->mu);
        if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");
        int rc = WV_OK;
        if (!m->ix) {
            wv_mirror::Built nb;
            rc = m->create_into(nb, len, std::max<uint64_t>(m->opt.initial_capacity, id + 1));
            if (rc) nb.release();
            else { m->ix = nb.ix; m->b = nb.b; m->dim = len; m->capacity = nb.capacity; }
        } else if (id >= m->capacity) {
            rc = m->grow_to(id);
        }
        if (rc) {
            l.unlock();
            m->mark_stale();
            return rc;
        }
    }
}

int wv_mirror_delete(wv_mirror* m, const uint64_t* ids, uint64_t n) {
    if (!m || (n && !ids)) return err(WV_EINVAL, "wv_mirror_delete: bad argument");
    // tombstones are recorded in every state: a startup or resync applies them
    std::shared_lock<FairRW> l(m->mu);
    std::vector<uint64_t> in;
    in.reserve(n);
    {
        std::lock_guard<std::mutex> bl(m->bm_mu);
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t id = ids[i];
            if (bit(m->tomb, id)) continue;
            set_bit(m->tomb, id);
            if (bit(m->have, id) && !bit(m->in_snap, id)) m->delta--;   // (a delta row no longer counts)
            if (id < m->capacity) in.push_back(id);
        }
    }
    if (!m->live()) return WV_OK;
    if (in.empty() || !m->ix) return WV_OK;
    int rc = wv_index_add_tombstones(m->ix, in.data(), in.size());
    if (rc) {
        l.unlock();
        m->mark_stale();
    }
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
    if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");   // (not waiting out a startup)
    std::shared_lock<FairRW> l(m->mu);
    if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");
    if (!m->ix) { *out_n = 0; return WV_OK; }   // empty index (search.go:463-465)
    if (len != m->dim) return err(WV_ESTALE, "wv_mirror_search: vector length differs from the index's");
    if (int rc = m->check_entrypoint(filtered, n_allow)) return rc;
    // ids past the capacity hold no row: the list is cut there (ascending)
    const uint64_t cap = m->capacity;
    while (n_allow && allow_ids[n_allow - 1] >= cap) --n_allow;
    return wv_batcher_search_ids(m->b, vector, k, filtered, allow_ids, n_allow, out_ids, out_dists, out_n);
}

int wv_mirror_search_by_distance(wv_mirror* m, const float* vector, int len, float target_distance,
                                 int64_t max_limit, int filtered, const uint64_t* allow_ids, uint64_t n_allow,
                                 uint64_t* out_ids, float* out_dists, int64_t out_cap, int64_t* out_n) {
    if (!m || !vector || !out_n || (n_allow && !allow_ids)) return err(WV_EINVAL, "wv_mirror_search_by_distance: bad argument");
    if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");
    std::shared_lock<FairRW> l(m->mu);
    if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");
    if (!m->ix) { *out_n = 0; return WV_OK; }
    if (len != m->dim) return err(WV_ESTALE, "wv_mirror_search_by_distance: vector length differs from the index's");
    if (int rc = m->check_entrypoint(filtered, n_allow)) return rc;   // (each deepening round is a SearchByVector)
    // through the micro-batcher: concurrent distance searches coalesce into
    // one batched SearchByVectorDistance (ids past the capacity hold no row)
    const uint64_t cap = m->capacity;
    while (n_allow && allow_ids[n_allow - 1] >= cap) --n_allow;
    return wv_batcher_search_distance_ids(m->b, vector, target_distance, max_limit, filtered, allow_ids, n_allow,
                                          out_ids, out_dists, out_cap, out_n);
}

int wv_mirror_update_config(wv_mirror* m, const wv_config* cfg) {
    if (!m || !cfg) return err(WV_EINVAL, "wv_mirror_update_config: bad argument");
    std::shared_lock<FairRW> l(m->mu);
    wv_config c;
    {
        std::lock_guard<std::mutex> cl(m->cfg_mu);
        const int dev = m->cfg.device;
        m->cfg = *cfg;
        m->cfg.device = dev;
        c = m->cfg;
    }
    if (!m->ix || !m->live()) return WV_OK;   // (a startup applies it at install)
    int rc = wv_index_update_config(m->ix, &c);
    if (rc) {
        l.unlock();
        m->mark_stale();
    }
    return rc;
}

int wv_mirror_needs_compaction(wv_mirror* m) {
    if (!m || !m->live() || m->delta.load() < m->opt.compact_rows) return 0;
    std::shared_lock<FairRW> l(m->mu);   // (ix is replaced under the exclusive lock)
    return m->live() && m->ix ? 1 : 0;
}

// Re-snapshot: the graph of the flushed commit log (the CPU index's own
// graph; rows added since stay in the delta), or a device build.
int wv_mirror_compact(wv_mirror* m) {
    if (!m) return err(WV_EINVAL, "wv_mirror_compact: bad argument");
    std::lock_guard<std::mutex> cl(m->compact_mu);
    if (!m->live()) return err(WV_ESTALE, "wv_mirror: stale");
    if (!m->log_dir.empty()) {
        Csr c;   // read without blocking searches
        int rc = load_csr(m->log_dir, m->config().max_connections, c);
        if (rc) return rc;
        if (c.n == 0 && !c.compressed) return WV_OK;
        std::unique_lock<FairRW> l(m->mu);
        if (!m->live() || !m->ix) return err(WV_ESTALE, "wv_mirror: stale");
        auto fail_stale = [&](int code) {
            l.unlock();
            m->mark_stale();
            return code;
        };
        if (c.n && (rc = m->grow_to(c.n - 1))) return fail_stale(rc);
        if (c.compressed && !m->pq) {   // compressed since startup (compress.go:39-99)
            if ((rc = m->enable_pq(m->ix, c, m->dim))) return fail_stale(rc);
            m->pq = true;
        }
        if (c.n == 0) return WV_OK;
        std::vector<uint64_t> have_now, snap;
        {
            std::lock_guard<std::mutex> bl(m->bm_mu);
            have_now = m->have;
        }
        uint64_t nodes = 0;
        bool gone = false;
        if ((rc = m->upload_graph(m->ix, c, have_now, snap, nodes, gone))) return fail_stale(rc);
        m->ep_gone = gone;
        std::lock_guard<std::mutex> bl(m->bm_mu);
        const std::vector<uint64_t> t = m->tomb_union(c, m->capacity);
        if (!t.empty() && (rc = wv_index_set_tombstones(m->ix, t.data(), std::min<uint64_t>(t.size() * 64, m->capacity))))
            return fail_stale(rc);
        m->in_snap.swap(snap);
        m->snap_nodes = nodes;
        m->delta = m->count_delta();
        m->compactions++;
        return WV_OK;
    }
    std::unique_lock<FairRW> l(m->mu);
    if (!m->live() || !m->ix) return err(WV_ESTALE, "wv_mirror: stale");
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
    st->state = m->state;
    st->live = m->live() ? 1 : 0;
    st->dim = m->dim;
    st->capacity = m->capacity;
    st->delta_rows = m->delta;
    st->graph_nodes = m->snap_nodes;
    st->growths = m->growths;
    st->compactions = m->compactions;
    st->startup_rows = m->startup_rows;
    st->startup_missing = m->startup_missing;
    st->pq = m->pq ? 1 : 0;
    st->startups = m->startups;
    st->resyncs = m->resyncs;
    st->failed_startups = m->failed_startups;
    st->replayed_writes = m->replayed;
    if (m->ix) wv_index_capacity(m->ix, nullptr, &st->n_rows);
    if (m->b) wv_batcher_stats(m->b, &st->batcher_requests, &st->batcher_batches);
    return WV_OK;
}

int wv_mirror_destroy(wv_mirror* m) {
    if (!m) return WV_OK;
    {
        std::lock_guard<std::mutex> l(m->wk_mu);
        m->stop = true;
        m->wk_cv.notify_all();
    }
    if (m->worker.joinable()) m->worker.join();
    {
        std::lock_guard<std::mutex> cl(m->compact_mu);
        std::unique_lock<FairRW> l(m->mu);
        m->state = WV_MIRROR_STALE;
        m->drop_index();
    }
    delete m;
    return WV_OK;
}

}  // extern "C"
