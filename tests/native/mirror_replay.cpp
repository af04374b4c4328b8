// mirror_replay.cpp -- the cgo decorator's lifecycle (go/vector/gpu/gpu.go
// over wv_mirror_*) replayed natively against the CPU restatement as "the
// shard's hnsw index": test infrastructure (links oracle/libwvoracle.so as the
// checker and as the CPU index whose commit log the mirror reads).
//
//   startup    the restatement inserts N0 rows one by one, writing its commit
//              log (commitlog/logger.go records, as insert.go writes them),
//              tombstones 600 ids and loses 100 of their objects; the log goes
//              to <dir>/main.hnsw.commitlog.d/<ts>.  wv_mirror_post_startup
//              replays that directory and pulls rows through a
//              VectorForIDThunk stand-in (no wv_index_build_graph shortcut).
//              Check 1: searches (HNSW, flat and filtered-HNSW by the cutoff)
//              equal the restatement's SearchByVector, ids and distances.
//   serving    a writer adds N_ADD rows (the restatement's Add then
//              wv_mirror_add, as the decorator does: the mirror grows past its
//              25 000-row initial size) and deletes ids; a maintenance thread
//              flushes the log and calls wv_mirror_compact whenever
//              wv_mirror_needs_compaction; 8 searchers query through
//              wv_mirror_search (allow lists as ascending ids) and assert that
//              no id deleted before a search started is returned and that a
//              row added before it started is found first while it sits in
//              the delta set.  Check 2: the delta stays bounded.
//   quiescent  final flush + compaction; check 3: searches equal the
//              restatement's again, and the delta is empty.
// Modes (argv[3]):
//   sync   (default) the above, PostStartup on the caller's thread;
//   async  wv_mirror_post_startup_async: writers and searchers start at once
//          while the mirror builds on its own thread (the vector source is
//          slowed so that writes do arrive meanwhile); searchers answered
//          WV_ESTALE until it is live (the CPU index serves); every write
//          made during the build must be replayed (stats) and then found;
//   heal   auto_resync with the log flush as the flush callback: a third of
//          the way through, one add reaches the CPU index but not the mirror
//          and the mirror is marked stale (a failed write); it must resync by
//          itself (stats.resyncs), find that row afterwards, and end equal to
//          the restatement;
//   pq     the CPU index is compressed before startup (KMeans quantizer,
//          compress.go:39-99; the AddPQ record appended to its log): the
//          mirror must load the quantizer from the log, serve compressed
//          (stats.pq), and equal the restatement's PQ searches; async start.
// Exit 0 with one JSON line, or 1 with the first violation.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <sys/stat.h>

#include "../../include/wvgpu.h"
#include "../../oracle/wv_oracle.h"

namespace {

constexpr int DIM = 32;
#ifdef WV_REPLAY_TSAN   // (ThreadSanitizer build over the CPU stand-in: the same scenario, smaller)
constexpr uint64_t N0 = 2000;
constexpr uint64_t N_ADD = 2000;
constexpr uint64_t INIT_CAP = 2500;
constexpr uint64_t COMPACT_ROWS = 512;
#else
constexpr uint64_t N0 = 20000;
constexpr uint64_t N_ADD = 20000;
constexpr uint64_t INIT_CAP = 25000;   // (the mirror's default, maintainance.go:22)
constexpr uint64_t COMPACT_ROWS = 4096;
#endif
constexpr uint64_t CAP = N0 + N_ADD;
constexpr int M = 16, EFC = 64, EF = 64, K = 10;
constexpr int64_t CUTOFF = 5000;
constexpr int SEARCHERS = 8;
constexpr int NQ_CHECK = 400;

std::atomic<bool> failed{false};
std::mutex err_mu;
std::string first_err;
void violation(const std::string& m) {
    std::lock_guard<std::mutex> l(err_mu);
    if (!failed.exchange(true)) first_err = m;
}

float urand(uint64_t id, int j) {
    uint64_t x = id * 0x9E3779B97F4A7C15ull + (uint64_t)j * 0xBF58476D1CE4E5B9ull + 0x94D049BB133111EBull;
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31;
    return (float)(x >> 40) * (1.0f / 16777216.0f);
}
void row(uint64_t id, float* out) { for (int j = 0; j < DIM; ++j) out[j] = urand(id, j); }

// the shard's object store (VectorForIDThunk stand-in)
std::vector<float> store(CAP * DIM);
std::vector<uint8_t> in_store(CAP, 0);

std::atomic<int> source_delay_us{0};
int vector_for_id(void*, uint64_t id, float* out, int cap, int* len) {
    if (const int d = source_delay_us.load()) std::this_thread::sleep_for(std::chrono::microseconds(d));
    if (id >= CAP || !in_store[id]) return WV_ENOTFOUND;
    *len = DIM;
    if (cap >= DIM) std::memcpy(out, &store[id * DIM], DIM * sizeof(float));
    return WV_OK;
}

// the CPU index and its commit log file
std::mutex cpu_mu;
wvo_index* cpu = nullptr;
std::string log_file;
uint64_t log_written = 0;

void flush_log() {   // hnsw.Flush(): the buffered log reaches the file (cpu_mu held)
    const uint64_t n = wvo_log_size(cpu);
    std::vector<uint8_t> buf(n);
    wvo_log_copy(cpu, buf.data(), n);
    FILE* f = std::fopen(log_file.c_str(), "ab");
    if (!f) { violation("cannot write " + log_file); return; }
    std::fwrite(buf.data() + log_written, 1, n - log_written, f);
    std::fclose(f);
    log_written = n;
}

std::vector<uint64_t> allow_ids(std::mt19937_64& g, uint64_t n_ids, uint64_t range) {
    std::vector<uint64_t> a;
    a.reserve(n_ids);
    for (uint64_t i = 0; i < n_ids; ++i) a.push_back(g() % range);
    std::sort(a.begin(), a.end());
    a.erase(std::unique(a.begin(), a.end()), a.end());
    return a;
}
int exact_fallbacks = 0;   // filtered HNSW queries answered by the exact scan

std::vector<uint64_t> to_bits(const std::vector<uint64_t>& ids, uint64_t range) {
    std::vector<uint64_t> b((range + 63) / 64, 0);
    for (uint64_t id : ids) b[id >> 6] |= 1ull << (id & 63);
    return b;
}

// KMeans quantizer for the pq mode: PQ_M segments of DIM / PQ_M dims, PQ_KS
// centres each taken from spread-out rows (a fitted table stands in for
// KMeans.Fit, which is not restated); the AddPQ record in logger.go:77-96's
// layout (KMeans data: kmeans.go:61-69)
constexpr int PQ_M = 8, PQ_KS = 256;
std::vector<float> pq_table() {
    const int ds = DIM / PQ_M;
    std::vector<float> t((size_t)PQ_M * PQ_KS * ds);
    for (int i = 0; i < PQ_M; ++i)
        for (int c = 0; c < PQ_KS; ++c)
            for (int j = 0; j < ds; ++j) t[((size_t)i * PQ_KS + c) * ds + j] = store[(uint64_t)(c * 73 + i) % N0 * DIM + i * ds + j];
    return t;
}
std::vector<uint8_t> add_pq_record(const std::vector<float>& t) {
    std::vector<uint8_t> r = {11};   // AddPQ
    auto u16 = [&](uint16_t v) { r.push_back(v & 0xFF); r.push_back(v >> 8); };
    u16(DIM);
    r.push_back(1);   // UseKMeansEncoder
    u16(PQ_KS);
    u16(PQ_M);
    r.push_back(0);   // distribution (tile encoder only)
    r.push_back(0);   // useBitsEncoding
    for (float f : t) {
        uint32_t u;
        std::memcpy(&u, &f, 4);
        for (int b = 0; b < 4; ++b) r.push_back((u >> (8 * b)) & 0xFF);
    }
    return r;
}

// heal mode: the decorator's flush callback (wvgpuFlush: hnsw.Flush under
// the write lock); every row added before it is then in the log's graph
std::atomic<uint64_t>* g_n_added = nullptr;
std::mutex* g_in_graph_mu = nullptr;
std::vector<uint8_t>* g_compacted = nullptr;
std::atomic<int> flushes{0};
// postheal mode: the lock the decorator's PostStartup holds around
// wv_mirror_post_startup_async (g.mu) -- wvgpuFlush takes it too
std::mutex* g_caller_mu = nullptr;
int flush_cb(void*) {
    std::unique_lock<std::mutex> cl;
    if (g_caller_mu) cl = std::unique_lock<std::mutex>(*g_caller_mu);
    std::lock_guard<std::mutex> l(cpu_mu);
    flush_log();
    const uint64_t na = g_n_added ? g_n_added->load() : 0;
    if (g_compacted) {
        std::lock_guard<std::mutex> gl(*g_in_graph_mu);
        for (uint64_t a = 0; a < na; ++a) (*g_compacted)[N0 + a] = 1;
    }
    flushes++;
    return 0;
}

// mirror vs restatement on NQ_CHECK queries (a third unfiltered, a third with
// a small allow list -> flatSearch, a third with a large one -> filtered HNSW)
int compare(wv_mirror* m, uint64_t range, int seed, const char* phase) {
#ifdef WV_REPLAY_TSAN
    (void)m; (void)range; (void)seed; (void)phase;
    return 0;   // the CPU stand-in (tsan/cpu_index.cpp) searches exactly: no HNSW parity to check
#endif
    std::mt19937_64 g(seed);
    std::vector<float> q(DIM);
    uint64_t oi[K], mi[K];
    float od[K], md[K];
    int diffs = 0;
    for (int i = 0; i < NQ_CHECK; ++i) {
        row(g() % range, q.data());
        for (int j = 0; j < DIM; ++j) q[j] += 0.02f * (urand(g(), j) - 0.5f);
        std::vector<uint64_t> al;
        if (i % 3 == 1) al = allow_ids(g, 1500, range);
        if (i % 3 == 2) al = allow_ids(g, 14000, range);
        const std::vector<uint64_t> bits = to_bits(al, range);
        int on = 0;
        int32_t mn = 0;
        {
            std::lock_guard<std::mutex> l(cpu_mu);
            wvo_search_by_vector(cpu, q.data(), K, i % 3 ? bits.data() : nullptr, i % 3 ? range : 0, oi, od, &on,
                                 nullptr);
        }
        const int rc = wv_mirror_search(m, q.data(), DIM, K, i % 3 != 0, al.data(), al.size(), mi, md, &mn);
        if (rc) { violation(std::string(phase) + ": mirror search: " + wv_last_error()); return -1; }
        bool same = mn == on;
        for (int j = 0; same && j < on; ++j) same = mi[j] == oi[j] && std::memcmp(&md[j], &od[j], 4) == 0;
        if (!same && i % 3 == 2) {
            // a filtered HNSW query whose side candidates outgrow the wave's
            // LDS is answered by the exact filtered scan (a
            // superset in quality): then it must equal flatSearch's answer
            int fn = 0;
            {
                std::lock_guard<std::mutex> l(cpu_mu);
                wvo_flat_search(cpu, q.data(), K, bits.data(), range, oi, od, &fn);
            }
            same = mn == fn;
            for (int j = 0; same && j < fn; ++j) same = mi[j] == oi[j] && std::memcmp(&md[j], &od[j], 4) == 0;
            if (same) ++exact_fallbacks;
        }
        if (!same) {
            if (++diffs == 1)
                std::fprintf(stderr, "%s: query %d differs (mirror n=%d id0=%llu, restatement n=%d id0=%llu)\n", phase, i,
                             mn, (unsigned long long)(mn ? mi[0] : 0), on, (unsigned long long)(on ? oi[0] : 0));
        }
    }
    return diffs;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: mirror_replay <dir> [device] [sync|async|heal|pq]\n"); return 2; }
    const std::string root = argv[1];
    const int device = argc > 2 ? std::atoi(argv[2]) : 0;
    const std::string mode = argc > 3 ? argv[3] : "sync";
    const bool async_start = mode == "async" || mode == "pq", pqm = mode == "pq";
    bool heal = mode == "heal";
    const bool epgone = mode == "epgone";
    // pqlive: the class is compressed while serving (UpdateUserConfig with
    // PQ.Enabled, config_update.go:97-120 -> Compress, compress.go:39-99),
    // with no write after it: the decorator's callback flushes the log and
    // compacts, and the mirror serves PQ codes from then on
    const bool pqlive = mode == "pqlive";
    // postheal: heal's self-healing mirror, and a PostStartup posted (under
    // the decorator's lock, which the resync's flush callback also takes)
    // while that resync waits in its flush: post_startup_async must return
    // without waiting for the worker, which then runs the posted startup
    const bool postheal = mode == "postheal";
    if (postheal) heal = true;
    if (mode != "sync" && !async_start && !heal && !epgone && !pqlive) { std::fprintf(stderr, "unknown mode %s\n", mode.c_str()); return 2; }
    const std::string log_dir = root + "/main.hnsw.commitlog.d";
    mkdir(root.c_str(), 0755);
    mkdir(log_dir.c_str(), 0755);
    log_file = log_dir + "/1700000000";
    std::remove(log_file.c_str());

    // ---- startup state: the CPU index as restoreFromDisk would find it ----
    cpu = wvo_create(DIM, WVO_L2, M, EFC, CAP, 7);
    wvo_set_search_config(cpu, EF, 100, 500, 8, CUTOFF, 0);
    wvo_log_enable(cpu, 1);
    std::vector<float> v(DIM);
    for (uint64_t id = 0; id < N0; ++id) {
        row(id, &store[id * DIM]);
        in_store[id] = 1;
        wvo_add(cpu, id, &store[id * DIM]);
    }
    std::mt19937_64 g0(5);
    std::vector<uint64_t> deleted;   // append-only: ids deleted before each point in time
    for (int i = 0; i < 600; ++i) {
        const uint64_t id = 1 + g0() % (N0 - 1);
        wvo_add_tombstone(cpu, id);
        deleted.push_back(id);
    }
    uint64_t gone = 0;
    for (int i = 0; i < 100; ++i) {   // objects deleted from the store as well
        const uint64_t id = deleted[i];
        uint64_t ns = 0, ep = 0, nu = 0;
        int ml = 0;
        wvo_graph_info(cpu, &ns, &ep, &ml, &nu);
        if (id == ep || !in_store[id]) continue;
        in_store[id] = 0;
        wvo_clear_vector(cpu, id);
        ++gone;
    }
    if (epgone) {   // the entrypoint's object deleted from the store, its node not cleaned up yet
        uint64_t ns = 0, ep = 0, nu = 0;
        int ml = 0;
        wvo_graph_info(cpu, &ns, &ep, &ml, &nu);
        wvo_add_tombstone(cpu, ep);
        in_store[ep] = 0;
        wvo_clear_vector(cpu, ep);
        ++gone;
    }
    flush_log();
    if (pqm) {   // Compress (compress.go:39-89): codes of every stored row, then the AddPQ record
        const std::vector<float> t = pq_table();
        std::vector<uint8_t> codes((size_t)N0 * PQ_M), has(N0, 0);
        for (uint64_t id = 0; id < N0; ++id) has[id] = in_store[id];
        wvo_pq_encode_kmeans(store.data(), N0, DIM, PQ_M, PQ_KS, t.data(), 0, codes.data());
        if (wvo_compress(cpu, PQ_M, PQ_KS, 0, t.data(), codes.data(), has.data(), N0)) {
            std::fprintf(stderr, "restatement compress failed\n");
            return 1;
        }
        const std::vector<uint8_t> rec = add_pq_record(t);
        FILE* f = std::fopen(log_file.c_str(), "ab");
        std::fwrite(rec.data(), 1, rec.size(), f);
        std::fclose(f);
    }

    wv_config cfg;
    wv_config_default(&cfg);
    cfg.device = device;
    cfg.max_connections = M;
    cfg.ef = EF;
    cfg.flat_search_cutoff = CUTOFF;
    wv_mirror_options opt{};
    opt.compact_rows = COMPACT_ROWS;
    if (INIT_CAP != 25000) opt.initial_capacity = INIT_CAP;
    opt.max_batch = 256;
    opt.commitlog_dir = log_dir.c_str();
    if (heal) {
        // (the library holds its worker 200 ms after each install: the second
        // failure below lands inside that window)
        setenv("WV_MIRROR_TEST_POST_INSTALL_MS", "200", 1);
        opt.auto_resync = 1;
        opt.flush = flush_cb;
        opt.resync_backoff_ms = 50;
    }
    std::mutex caller_mu;
    if (postheal) g_caller_mu = &caller_mu;
    wv_mirror* m = nullptr;
    if (wv_mirror_create(WV_L2_SQUARED, &cfg, &opt, &m)) { std::fprintf(stderr, "create: %s\n", wv_last_error()); return 1; }
    {
        // before PostStartup the mirror does not serve: the CPU index answers
        uint64_t i0[K]; float d0[K]; int32_t n0 = 0;
        if (wv_mirror_search(m, &store[0], DIM, K, 0, nullptr, 0, i0, d0, &n0) != WV_ESTALE)
            violation("a mirror serves before PostStartup");
    }
    const auto t_start = std::chrono::steady_clock::now();
    wv_mirror_stats st0{};
    int diffs_startup = -1;
    if (!async_start) {
        if (wv_mirror_post_startup(m, vector_for_id, nullptr)) {
            std::fprintf(stderr, "post_startup: %s\n", wv_last_error());
            return 1;
        }
        wv_mirror_get_stats(m, &st0);
        if (!st0.live || st0.dim != DIM || st0.startup_missing != gone || st0.startup_rows != N0 - gone ||
            st0.graph_nodes != N0 || st0.delta_rows != 0 || st0.capacity != INIT_CAP)
            violation("startup stats: live " + std::to_string(st0.live) + " dim " + std::to_string(st0.dim) + " rows " +
                      std::to_string(st0.startup_rows) + " missing " + std::to_string(st0.startup_missing) + " nodes " +
                      std::to_string(st0.graph_nodes) + " delta " + std::to_string(st0.delta_rows) + " capacity " +
                      std::to_string(st0.capacity));
        diffs_startup = failed ? -1 : epgone ? 0 : compare(m, N0, 11, "startup");
    } else {
        // PostStartup returns at once; the build runs on the mirror's thread
        // while the writer and the searchers below already run
        source_delay_us = 40;   // ~0.8 s of vector source: writes land during the build
        if (wv_mirror_post_startup_async(m, vector_for_id, nullptr)) {
            std::fprintf(stderr, "post_startup_async: %s\n", wv_last_error());
            return 1;
        }
        wv_mirror_stats s;
        wv_mirror_get_stats(m, &s);
        if (s.state != WV_MIRROR_STARTING) violation("async startup: the mirror is not starting after the call");
        diffs_startup = 0;   // (no quiescent point: the final comparison covers it)
    }
    const double startup_call_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    if (epgone) {
        // the log's entrypoint lost its object: knnSearchByVector errors
        // (search.go:467-476) -- the mirror too -- while a flat search (a
        // small allow list, search.go:74-78) still answers as flatSearch
        uint64_t ns = 0, ep = 0, nu = 0;
        int ml = 0;
        wvo_graph_info(cpu, &ns, &ep, &ml, &nu);
        if (in_store[ep]) violation("epgone: the entrypoint still has its object");
        uint64_t ids[K], oi[K];
        float ds[K], od[K];
        int32_t n = 0;
        int on = 0;
        int rc = wv_mirror_search(m, &store[5 * DIM], DIM, K, 0, nullptr, 0, ids, ds, &n);
        if (rc != WV_EDELETED) violation("epgone: an unfiltered search returned " + std::to_string(rc));
        std::mt19937_64 g(3);
        const std::vector<uint64_t> al = allow_ids(g, 1500, N0), al_big = allow_ids(g, 14000, N0);
        if ((int64_t)al_big.size() >= CUTOFF) {   // (the TSAN build's corpus is below the cutoff)
            rc = wv_mirror_search(m, &store[5 * DIM], DIM, K, 1, al_big.data(), al_big.size(), ids, ds, &n);
            if (rc != WV_EDELETED) violation("epgone: a filtered HNSW search returned " + std::to_string(rc));
        }
        rc = wv_mirror_search(m, &store[5 * DIM], DIM, K, 1, al.data(), al.size(), ids, ds, &n);
        const std::vector<uint64_t> bits = to_bits(al, N0);
        wvo_flat_search(cpu, &store[5 * DIM], K, bits.data(), N0, oi, od, &on);
        bool same = rc == 0 && n == on;
        for (int j = 0; same && j < on; ++j) same = ids[j] == oi[j] && std::memcmp(&ds[j], &od[j], 4) == 0;
#ifdef WV_REPLAY_TSAN
        same = rc == 0;   // (the CPU stand-in's exact search is not flatSearch's: only the status is checked)
#endif
        if (!same) violation("epgone: a flat search differs from flatSearch (rc " + std::to_string(rc) + ")");
        int64_t nd = 0;
        rc = wv_mirror_search_by_distance(m, &store[5 * DIM], DIM, 1.f, -1, 0, nullptr, 0, ids, ds, K, &nd);
        if (rc != WV_EDELETED) violation("epgone: an unfiltered search by distance returned " + std::to_string(rc));
        wv_mirror_destroy(m);
        wvo_destroy(cpu);
        if (failed) {
            std::fprintf(stderr, "VIOLATION: %s\n", first_err.c_str());
            return 1;
        }
        std::printf("{\"ok\": true, \"mode\": \"epgone\", \"flat_ids\": %d}\n", n);
        return 0;
    }

    // ---- serving: adds, deletes, compactions and searches at once ----
    std::atomic<int> n_deleted{(int)deleted.size()};
    deleted.resize(deleted.size() + N_ADD);   // (no reallocation while readers scan it)
    std::atomic<uint64_t> n_added{0};
    std::atomic<bool> writer_done{false}, stop_maint{false};
    std::atomic<uint64_t> max_delta{0}, n_compact{0}, n_search{0}, n_added_checks{0}, n_filtered{0}, n_dist_search{0};
    std::mutex in_graph_mu;
    std::vector<uint8_t> compacted(CAP, 0);   // added rows that a compaction moved into the graph
    g_n_added = &n_added;
    g_in_graph_mu = &in_graph_mu;
    g_compacted = &compacted;
    std::atomic<uint64_t> stale_answers{0};   // searches the CPU index answered (mirror not live)
    std::atomic<uint64_t> missed_id{UINT64_MAX}, missed_id2{UINT64_MAX};
    std::atomic<bool> live_seen{!async_start};

    auto writer = std::thread([&] {
        std::mt19937_64 g(21);
        for (uint64_t a = 0; a < N_ADD && !failed; ++a) {
            const uint64_t id = N0 + a;
            row(id, &store[id * DIM]);
            in_store[id] = 1;
            {
                std::lock_guard<std::mutex> l(cpu_mu);
                wvo_add(cpu, id, &store[id * DIM]);
            }
            if (postheal && a == N_ADD / 3) {
                missed_id = missed_id2 = id;
                wv_mirror_stats s0;
                wv_mirror_get_stats(m, &s0);
                std::unique_lock<std::mutex> cl(caller_mu);   // PostStartup's g.mu.Lock()
                wv_mirror_mark_stale(m);
                // the resync has begun (STARTING) and blocks in the flush
                // callback on caller_mu
                const auto t_poll = std::chrono::steady_clock::now();
                for (;;) {
                    wv_mirror_stats s;
                    wv_mirror_get_stats(m, &s);
                    if (s.state == WV_MIRROR_STARTING) break;
                    if (std::chrono::steady_clock::now() - t_poll > std::chrono::seconds(60)) {
                        violation("postheal: the resync did not start");
                        break;
                    }
                    std::this_thread::sleep_for(std::chrono::microseconds(50));
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(20));   // (into the callback)
                auto call = std::async(std::launch::async, [&] { return wv_mirror_post_startup_async(m, vector_for_id, nullptr); });
                if (call.wait_for(std::chrono::seconds(20)) != std::future_status::ready) {
                    std::fprintf(stderr, "VIOLATION: postheal: post_startup_async waits for the resync whose flush "
                                         "needs the caller's lock (deadlock)\n");
                    std::_Exit(1);
                }
                if (call.get()) violation(std::string("postheal post_startup_async: ") + wv_last_error());
                cl.unlock();
                if (wv_mirror_wait_live(m, 120000)) violation("postheal: the posted startup did not go live");
                wv_mirror_stats s1;
                wv_mirror_get_stats(m, &s1);
                if (s1.startups < s0.startups + 2)
                    violation("postheal: the posted startup did not run after the resync (startups " +
                              std::to_string(s0.startups) + " -> " + std::to_string(s1.startups) + ")");
            } else if (heal && a == N_ADD / 3) {
                // a write the mirror never saw (the decorator's propagation
                // failed): stale now, the mirror must heal itself
                missed_id = id;
                wv_mirror_mark_stale(m);
                // and a second failure the moment that resync goes live
                // (polled: it lands while the worker is still busy finishing
                // the resync -- the library holds it 200 ms there in this
                // mode): the mirror must heal again
                const auto t_poll = std::chrono::steady_clock::now();
                wv_mirror_stats s;
                for (;;) {
                    wv_mirror_get_stats(m, &s);
                    if (s.state == WV_MIRROR_LIVE) break;
                    if (std::chrono::steady_clock::now() - t_poll > std::chrono::seconds(120)) {
                        violation("heal: the first resync did not go live");
                        break;
                    }
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                }
                missed_id2 = id;
                wv_mirror_mark_stale(m);
            } else {
                const int rc = wv_mirror_add(m, id, &store[id * DIM], DIM);
                if (rc && !(heal && rc == WV_ESTALE)) violation(std::string("add: ") + wv_last_error());
            }
            n_added.store(a + 1, std::memory_order_release);
            // async / pq: half of the writes land during the build, the rest
            // once the mirror serves (so compactions run while serving)
            if (async_start && a == N_ADD / 2 && wv_mirror_wait_live(m, 120000))
                violation("async startup: the mirror did not become live");
            if (a % 3 == 0) {
                const uint64_t del = a % 9 == 0 && a > 16 ? N0 + a - 16 : g() % N0;
                {
                    std::lock_guard<std::mutex> l(cpu_mu);
                    wvo_add_tombstone(cpu, del);
                }
                if (wv_mirror_delete(m, &del, 1)) violation(std::string("delete: ") + wv_last_error());
                const int d = n_deleted.load();
                deleted[d] = del;
                n_deleted.store(d + 1, std::memory_order_release);
            }
            wv_mirror_stats s;
            wv_mirror_get_stats(m, &s);
            uint64_t md = max_delta.load();
            while (s.delta_rows > md && !max_delta.compare_exchange_weak(md, s.delta_rows)) {}
        }
        writer_done = true;
    });
    auto maint = std::thread([&] {   // the decorator's compaction goroutine
        while (!stop_maint && !failed) {
            if (wv_mirror_needs_compaction(m)) {
                const uint64_t na = n_added.load(std::memory_order_acquire);
                {
                    std::lock_guard<std::mutex> l(cpu_mu);
                    flush_log();
                }
                const int crc = wv_mirror_compact(m);
                if (crc && !(crc == WV_ESTALE && (heal || async_start)))
                    violation(std::string("compact: ") + wv_last_error());
                {
                    std::lock_guard<std::mutex> l(in_graph_mu);
                    for (uint64_t a = 0; a < na; ++a) compacted[N0 + a] = 1;
                }
                n_compact++;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(500));
        }
    });
    auto searcher = [&](int t) {
        std::mt19937_64 g(100 + t);
        std::vector<float> q(DIM);
        uint64_t ids[K];
        float ds[K];
        uint64_t it = 0;
        while (!writer_done && !failed) {
            ++it;
            const int nd = n_deleted.load(std::memory_order_acquire);
            const uint64_t na = n_added.load(std::memory_order_acquire);
            std::vector<uint8_t> del_now(CAP, 0);
            for (int i = 0; i < nd; ++i) del_now[deleted[i]] = 1;
            uint64_t target = UINT64_MAX;
            bool target_in_graph = false;
            if (na > 0 && it % 2 == 0) {
                target = N0 + g() % na;
                row(target, q.data());
                std::lock_guard<std::mutex> l(in_graph_mu);
                target_in_graph = compacted[target];
            } else {
                row(g() % N0, q.data());
                for (int j = 0; j < DIM; ++j) q[j] += 0.01f * urand(g(), j);
            }
            const bool filtered = it % 5 == 0;
            std::vector<uint64_t> al;
            if (filtered) {
                al = allow_ids(g, 1500, N0 + na);
                if (target != UINT64_MAX) {
                    al.push_back(target);
                    std::sort(al.begin(), al.end());
                    al.erase(std::unique(al.begin(), al.end()), al.end());
                }
                n_filtered++;
            }
            int32_t n = 0;
            const int rc = wv_mirror_search(m, q.data(), DIM, K, filtered, al.data(), al.size(), ids, ds, &n);
            if (rc == WV_ESTALE && (async_start || heal)) {   // starting / resyncing: the CPU index answers
                stale_answers++;
                continue;
            }
            if (rc) { violation(std::string("search: ") + wv_last_error()); return; }
            live_seen = true;
            n_search++;
            for (int i = 0; i < n; ++i) {
                if (ids[i] >= CAP) violation("id out of range");
                else if (del_now[ids[i]]) violation("search returned deleted id " + std::to_string(ids[i]));
                if (filtered && !std::binary_search(al.begin(), al.end(), ids[i]))
                    violation("filtered search returned a disallowed id");
            }
            // (pq: a compressed index ranks by the PQ distance, under which a
            // row's own vector need not come first -- no such check there)
            if (!pqm && target != UINT64_MAX && !del_now[target] && (filtered || !target_in_graph)) {
                n_added_checks++;
                bool deleted_since = false;
                const int nd2 = n_deleted.load(std::memory_order_acquire);
                for (int i = nd; i < nd2; ++i) deleted_since |= deleted[i] == target;
                if (!(n > 0 && ids[0] == target && ds[0] == 0.f) && !deleted_since)
                    violation("added id " + std::to_string(target) + " not found first");
            }
            // SearchByVectorDistance through the batcher, concurrently with
            // the k-NN callers: within the target, no deleted or disallowed id
            if (it % 7 == 3 && n > 0) {
                const float td = ds[n - 1];
                uint64_t dids[4 * K];
                float dds[4 * K];
                int64_t dn = 0;
                const int drc = wv_mirror_search_by_distance(m, q.data(), DIM, td, -1, filtered, al.data(), al.size(),
                                                             dids, dds, 4 * K, &dn);
                if (drc == WV_ESTALE && (async_start || heal)) {
                    stale_answers++;
                    continue;
                }
                if (drc) { violation(std::string("search by distance: ") + wv_last_error()); return; }
                n_dist_search++;
                for (int64_t i = 0; i < std::min<int64_t>(dn, 4 * K); ++i) {
                    if (dids[i] >= CAP) violation("distance search: id out of range");
                    else if (del_now[dids[i]]) violation("distance search returned deleted id " + std::to_string(dids[i]));
                    if (filtered && !std::binary_search(al.begin(), al.end(), dids[i]))
                        violation("filtered distance search returned a disallowed id");
                    if (!(dds[i] <= td || std::fabs((double)dds[i] - (double)td) <= 1e-6))
                        violation("distance search returned an entry beyond the target");
                }
            }
        }
    };
    std::vector<std::thread> ts;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < SEARCHERS; ++t) ts.emplace_back(searcher, t);
    writer.join();
    for (auto& t : ts) t.join();
    stop_maint = true;
    maint.join();
    const double serve_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    // ---- quiescent: live again, final flush + compaction, then the restatement ----
    if (!failed && wv_mirror_wait_live(m, 120000)) violation("the mirror did not become live");
    if (async_start) {
        wv_mirror_stats s;
        wv_mirror_get_stats(m, &s);
        st0 = s;
        if (s.replayed_writes == 0) violation("async startup: no write arrived during the build (test too fast)");
        if (pqm && !s.pq) violation("pq: the mirror does not serve compressed");
    }
    if (heal && !failed) {
        // the missed rows: found first by an exact (filtered) search
        for (const uint64_t id : {missed_id.load(), missed_id2.load()}) {
            uint64_t ids[K];
            float ds[K];
            int32_t n = 0;
            const int rc = wv_mirror_search(m, &store[id * DIM], DIM, K, 1, &id, 1, ids, ds, &n);
            if (rc || n != 1 || ids[0] != id || ds[0] != 0.f)
                violation("heal: missed row " + std::to_string(id) + " is not served after the resyncs");
        }
    }
    if (pqlive && !failed) {
        // Compress on the CPU index: codes of every stored row, then the
        // AddPQ record; the mirror still serves uncompressed (it has not
        // seen the record) -- the decorator answers from the CPU index until
        // the callback's flush + compaction below turned the mirror to PQ
        {
            std::lock_guard<std::mutex> l(cpu_mu);
            const std::vector<float> t = pq_table();
            std::vector<uint8_t> codes((size_t)CAP * PQ_M), has(CAP, 0);
            for (uint64_t id = 0; id < CAP; ++id) has[id] = in_store[id];
            wvo_pq_encode_kmeans(store.data(), CAP, DIM, PQ_M, PQ_KS, t.data(), 0, codes.data());
            if (wvo_compress(cpu, PQ_M, PQ_KS, 0, t.data(), codes.data(), has.data(), CAP)) violation("restatement compress failed");
            flush_log();
            const std::vector<uint8_t> rec = add_pq_record(t);
            FILE* f = std::fopen(log_file.c_str(), "ab");
            std::fwrite(rec.data(), 1, rec.size(), f);
            std::fclose(f);
        }
        wv_mirror_stats s0;
        wv_mirror_get_stats(m, &s0);
        if (s0.pq) violation("pqlive: the mirror is compressed before it saw the log");
        if (wv_mirror_compact(m)) violation(std::string("pqlive compact: ") + wv_last_error());
        wv_mirror_stats s1;
        wv_mirror_get_stats(m, &s1);
        if (!s1.pq) violation("pqlive: the mirror does not serve compressed after the compaction");
    }
    {
        std::lock_guard<std::mutex> l(cpu_mu);
        flush_log();
    }
    if (!failed && wv_mirror_compact(m)) violation(std::string("final compact: ") + wv_last_error());
    wv_mirror_stats st;
    wv_mirror_get_stats(m, &st);
    if (heal && !postheal && !failed && (st.resyncs < 2 || flushes < 2))
        violation("heal: the mirror did not resync by itself after both failures (resyncs " + std::to_string(st.resyncs) + ")");
    const int diffs_final = failed ? -1 : compare(m, CAP, 12, "final");
    if (!failed && st.delta_rows != 0) violation("delta not empty after the final compaction");
    // (async / pq: the writes replayed at install join the delta at once)
    if (!failed && max_delta > (async_start ? N_ADD : 0) + 2 * COMPACT_ROWS)
        violation("delta grew to " + std::to_string(max_delta.load()));
    if (!failed && st.growths < 1) violation("the mirror never grew past its initial capacity");
    // (async / heal: the mirror serves only part of the writer's run)
    if (!failed && n_compact < (async_start || heal ? 1u : 2u)) violation("too few compactions while serving");
    if (!failed && (diffs_startup != 0 || diffs_final != 0))
        violation("searches differ from the restatement: startup " + std::to_string(diffs_startup) + ", final " +
                  std::to_string(diffs_final) + " of " + std::to_string(NQ_CHECK));
    wv_mirror_destroy(m);
    wvo_destroy(cpu);
    if (failed) {
        std::fprintf(stderr, "VIOLATION: %s\n", first_err.c_str());
        return 1;
    }
    std::printf("{\"ok\": true, \"mode\": \"%s\", \"resyncs\": %llu, \"replayed_writes\": %llu, \"pq\": %d, "
                "\"stale_answers\": %llu, \"startup_call_s\": %.3f, \"startup_rows\": %llu, \"startup_missing\": %llu, "
                "\"diffs_startup\": %d, \"diffs_final\": %d, \"exact_fallbacks\": %d, \"checked\": %d, \"adds\": %llu, \"deletes\": %d, "
                "\"compactions\": %llu, \"max_delta\": %llu, \"capacity\": %llu, \"growths\": %llu, "
                "\"searches\": %llu, \"distance_searches\": %llu, \"added_checks\": %llu, \"filtered\": %llu, \"batcher_requests\": %llu, "
                "\"batcher_batches\": %llu, \"serve_s\": %.2f}\n",
                mode.c_str(), (unsigned long long)st.resyncs, (unsigned long long)st.replayed_writes, st.pq,
                (unsigned long long)stale_answers.load(), startup_call_s,
                (unsigned long long)st0.startup_rows, (unsigned long long)st0.startup_missing,
                diffs_startup, diffs_final, exact_fallbacks, NQ_CHECK, (unsigned long long)n_added.load(), n_deleted.load(),
                (unsigned long long)st.compactions, (unsigned long long)max_delta.load(),
                (unsigned long long)st.capacity, (unsigned long long)st.growths, (unsigned long long)n_search.load(),
                (unsigned long long)n_dist_search.load(),
                (unsigned long long)n_added_checks.load(), (unsigned long long)n_filtered.load(),
                (unsigned long long)st.batcher_requests, (unsigned long long)st.batcher_batches, serve_s);
    return 0;
}
