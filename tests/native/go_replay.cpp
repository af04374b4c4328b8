// go_replay.cpp -- replays the C call sequence of go/vector/gpu/gpu.go (the
// cgo decorator behind Weaviate's VectorIndex, vector_index.go:23-40) against
// libwvgpu.so on the GPU, from many threads at once:
//
//   8 searcher threads  SearchByVector -> wv_batcher_search (unfiltered: HNSW
//                       via the AUTO dispatch; some with an allow list:
//                       flatSearch) and a few SearchByVectorDistance calls
//   1 writer thread     Add    -> wv_index_add            (insert.go:43-65)
//                       Delete -> wv_index_add_tombstones (delete.go:29-84)
//   1 resync            SyncFromCPU (exclusive): a fresh GPU-built snapshot
//                       that now holds the added rows (wv_index_build_graph)
//
// Every search records, before it starts, how many deletes and adds had
// returned (release/acquire counters over append-only logs).  It then asserts
//   - no id deleted before the search started is ever returned, and
//   - a search for the exact vector of an id added before it started returns
//     that id first (distance 0), i.e. added rows are findable at once,
// exactly what a Go caller relies on after Delete / Add return.
// Exit 0 and one JSON line on success; exit 1 with the first violation.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wvgpu.h"

namespace {

constexpr int DIM = 32;
constexpr uint64_t N0 = 20000;      // rows in the startup snapshot
constexpr uint64_t N_ADD = 2000;    // rows added while serving
constexpr uint64_t CAP = N0 + N_ADD;
constexpr int N_DELETE = 3000;
constexpr int SEARCHERS = 8;
constexpr int K = 10;

std::atomic<bool> failed{false};
std::mutex err_mu;
std::string first_err;

void violation(const std::string& m) {
    std::lock_guard<std::mutex> l(err_mu);
    if (!failed.exchange(true)) first_err = m;
}

float urand(uint64_t id, int j) {   // counter-based U[0,1): rows reproducible per id
    uint64_t x = id * 0x9E3779B97F4A7C15ull + (uint64_t)j * 0xBF58476D1CE4E5B9ull + 0x94D049BB133111EBull;
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31;
    return (float)(x >> 40) * (1.0f / 16777216.0f);
}

void row(uint64_t id, float* out) {
    for (int j = 0; j < DIM; ++j) out[j] = urand(id, j);
}

// append-only logs published by counters (writer: store entry, then
// count.store(release); reader: count.load(acquire), then entries < count)
std::vector<uint64_t> deleted_log(N_DELETE);
std::atomic<int> n_deleted{0};
std::atomic<uint64_t> n_added{0};   // ids N0 .. N0 + n_added - 1 are added
// added rows still in the delta set (scanned exactly by every search) must be
// found strictly; rows a resync moved into the HNSW graph are found with the
// graph's recall (as in the reference after its insert), counted instead
std::atomic<uint64_t> added_at_resync{0};

bool deleted_since(int nd_before, uint64_t id) {   // deleted while a search ran?
    const int nd = n_deleted.load(std::memory_order_acquire);
    for (int i = nd_before; i < nd; ++i)
        if (deleted_log[i] == id) return true;
    return false;
}

// the decorator's RWMutex: searches shared, SyncFromCPU exclusive.  Go's
// sync.RWMutex is writer-preferring (a blocked Lock holds off new readers);
// std::shared_mutex (glibc) is not, and 8 back-to-back searchers would starve
// the resync forever -- so a gate gives the same semantics.
struct GoRWMutex {
    std::shared_mutex rw;
    std::mutex gate;
    void lock_shared() {
        { std::lock_guard<std::mutex> g(gate); }
        rw.lock_shared();
    }
    void unlock_shared() { rw.unlock_shared(); }
    void lock() { gate.lock(); rw.lock(); }
    void unlock() { rw.unlock(); gate.unlock(); }
};
GoRWMutex sync_mu;

}  // namespace

int main(int argc, char** argv) {
    const int device = argc > 1 ? std::atoi(argv[1]) : 0;
    wv_config cfg;
    wv_config_default(&cfg);
    cfg.device = device;
    cfg.max_connections = 16;
    cfg.flat_search_cutoff = 2000;   // allow lists below this go flat (search.go:71-75)
    wv_index* ix = nullptr;
    if (wv_index_create(DIM, WV_L2_SQUARED, &cfg, CAP, &ix)) {
        std::fprintf(stderr, "create: %s\n", wv_last_error());
        return 1;
    }
    // PostStartup: SyncFromCPU of the startup state
    std::vector<float> base(N0 * DIM);
    for (uint64_t i = 0; i < N0; ++i) row(i, base.data() + i * DIM);
    if (wv_index_upload_vectors(ix, base.data(), N0, 0) || wv_index_build_graph(ix, 64, 7, 64)) {
        std::fprintf(stderr, "startup: %s\n", wv_last_error());
        return 1;
    }
    wv_batcher* b = nullptr;
    if (wv_batcher_create(ix, DIM, 256, 200, &b)) {
        std::fprintf(stderr, "batcher: %s\n", wv_last_error());
        return 1;
    }
    // deletes: a fixed random permutation of startup ids plus some added ids
    {
        std::mt19937_64 g(11);
        std::vector<uint64_t> perm(N0);
        for (uint64_t i = 0; i < N0; ++i) perm[i] = i;
        std::shuffle(perm.begin(), perm.end(), g);
        for (int i = 0; i < N_DELETE; ++i) deleted_log[i] = perm[i];
        // every 10th delete targets an already added row (filled in by the writer)
    }

    std::atomic<bool> writer_done{false};
    std::atomic<uint64_t> n_search{0}, n_added_checks{0}, n_filtered{0}, n_dist{0}, n_resync{0};
    std::atomic<uint64_t> n_graph_checks{0}, n_graph_misses{0};

    auto writer = std::thread([&] {
        std::vector<float> v(DIM);
        int d = 0;
        for (uint64_t a = 0; a < N_ADD && !failed; ++a) {
            const uint64_t id = N0 + a;
            row(id, v.data());
            {
                std::shared_lock<GoRWMutex> l(sync_mu);
                if (wv_index_add(ix, &id, v.data(), 1)) violation(std::string("add: ") + wv_last_error());
            }
            n_added.store(a + 1, std::memory_order_release);
            // an import's pace (a few thousand objects per second), so the
            // searchers overlap every phase of the writer
            std::this_thread::sleep_for(std::chrono::microseconds(400));
            // interleave deletes: ~3 per 2 adds
            for (int r = 0; r < 3 && a % 2 == 0 && d < N_DELETE; ++r, ++d) {
                uint64_t del = deleted_log[d];
                if (d % 10 == 9 && a > 8) del = N0 + (a - 8);   // delete a row added earlier
                deleted_log[d] = del;
                {
                    std::shared_lock<GoRWMutex> l(sync_mu);
                    if (wv_index_add_tombstones(ix, &del, 1))
                        violation(std::string("tombstone: ") + wv_last_error());
                }
                n_deleted.store(d + 1, std::memory_order_release);
            }
            if (a == N_ADD / 2) {
                // SyncFromCPU: exclusive, a fresh snapshot holding the added rows
                std::unique_lock<GoRWMutex> l(sync_mu);
                if (wv_index_build_graph(ix, 64, 7, 64)) violation(std::string("resync: ") + wv_last_error());
                added_at_resync.store(a + 1, std::memory_order_release);
                n_resync++;
            }
        }
        writer_done = true;
    });

    auto searcher = [&](int t) {
        std::mt19937_64 g(100 + t);
        std::vector<float> q(DIM);
        std::vector<uint64_t> ids(K);
        std::vector<float> ds(K);
        std::vector<uint64_t> allow((CAP + 63) / 64);
        uint64_t it = 0;
        while (!writer_done && !failed) {
            ++it;
            const int nd = n_deleted.load(std::memory_order_acquire);
            const uint64_t na = n_added.load(std::memory_order_acquire);
            const uint64_t in_graph = added_at_resync.load(std::memory_order_acquire);
            std::vector<uint8_t> del_now(CAP, 0);
            for (int i = 0; i < nd; ++i) del_now[deleted_log[i]] = 1;
            // target: an added row (exact vector) or a perturbed startup row
            uint64_t target = UINT64_MAX;
            if (na > 0 && it % 2 == 0) {
                target = N0 + g() % na;
                row(target, q.data());
            } else {
                row(g() % N0, q.data());
                for (int j = 0; j < DIM; ++j) q[j] += 0.01f * urand(g(), j);
            }
            const bool filtered = it % 5 == 0;
            const bool by_dist = it % 17 == 0;
            int32_t n = 0;
            std::shared_lock<GoRWMutex> l(sync_mu);
            if (by_dist) {
                std::vector<uint64_t> di(4096);
                std::vector<float> dd(4096);
                int64_t nn = 0;
                if (wv_search_by_vector_distance(ix, q.data(), 0.5f, 200, nullptr, 0, di.data(), dd.data(), 4096,
                                                 &nn)) {
                    violation(std::string("distance search: ") + wv_last_error());
                    return;
                }
                for (int64_t i = 0; i < std::min<int64_t>(nn, 4096); ++i)
                    if (di[i] < CAP && del_now[di[i]]) violation("distance search returned deleted id " + std::to_string(di[i]));
                if (target != UINT64_MAX && !del_now[target] && target - N0 >= in_graph &&
                    (nn == 0 || di[0] != target) && !deleted_since(nd, target))
                    violation("distance search missed added id " + std::to_string(target));
                n_dist++;
                continue;
            }
            if (filtered) {
                // an allow list of ~1500 ids (below the cutoff: flatSearch), always holding target
                std::fill(allow.begin(), allow.end(), 0);
                for (int i = 0; i < 1500; ++i) {
                    const uint64_t id = g() % (N0 + na);
                    allow[id >> 6] |= 1ull << (id & 63);
                }
                if (target != UINT64_MAX) allow[target >> 6] |= 1ull << (target & 63);
                n_filtered++;
            }
            if (wv_batcher_search(b, q.data(), K, filtered ? allow.data() : nullptr, filtered ? CAP : 0, ids.data(),
                                  ds.data(), &n)) {
                violation(std::string("search: ") + wv_last_error());
                return;
            }
            n_search++;
            for (int i = 0; i < n; ++i) {
                if (ids[i] >= CAP) violation("id out of range " + std::to_string(ids[i]));
                else if (del_now[ids[i]]) violation("search returned deleted id " + std::to_string(ids[i]));
                if (filtered && ids[i] < CAP && !(allow[ids[i] >> 6] >> (ids[i] & 63) & 1))
                    violation("filtered search returned a disallowed id");
            }
            if (target != UINT64_MAX && !del_now[target]) {
                const bool hit = n > 0 && ids[0] == target && ds[0] == 0.f;
                if (filtered || target - N0 >= in_graph) {   // exact: flatSearch or the delta set
                    n_added_checks++;
                    if (!hit && !deleted_since(nd, target))
                        violation("added id " + std::to_string(target) + " not found first (got " +
                                  (n ? std::to_string(ids[0]) : std::string("nothing")) + ")");
                } else {
                    n_graph_checks++;
                    if (!hit && !deleted_since(nd, target)) n_graph_misses++;
                }
            }
        }
    };
    std::vector<std::thread> ts;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < SEARCHERS; ++t) ts.emplace_back(searcher, t);
    writer.join();
    for (auto& t : ts) t.join();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t req = 0, batches = 0;
    wv_batcher_stats(b, &req, &batches);
    wv_batcher_destroy(b);
    wv_index_destroy(ix);
    if (!failed && n_graph_misses * 50 > n_graph_checks)
        violation("hnsw self-recall of resynced rows below 0.98: " + std::to_string(n_graph_misses) + " misses of " +
                  std::to_string(n_graph_checks));
    if (failed) {
        std::fprintf(stderr, "VIOLATION: %s\n", first_err.c_str());
        return 1;
    }
    std::printf("{\"ok\": true, \"searches\": %llu, \"added_checks\": %llu, \"filtered\": %llu, "
                "\"graph_checks\": %llu, \"graph_misses\": %llu, \"distance_searches\": %llu, \"adds\": %llu, \"deletes\": %d, \"resyncs\": %llu, "
                "\"batcher_requests\": %llu, \"batcher_batches\": %llu, \"seconds\": %.2f}\n",
                (unsigned long long)n_search.load(), (unsigned long long)n_added_checks.load(),
                (unsigned long long)n_filtered.load(), (unsigned long long)n_graph_checks.load(),
                (unsigned long long)n_graph_misses.load(), (unsigned long long)n_dist.load(),
                (unsigned long long)n_added.load(), n_deleted.load(), (unsigned long long)n_resync.load(),
                (unsigned long long)req, (unsigned long long)batches, secs);
    return 0;
}
