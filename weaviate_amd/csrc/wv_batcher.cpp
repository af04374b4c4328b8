// wv_batcher.cpp -- native micro-batcher for concurrent single-query searches.
//
// The reference calls VectorIndex.SearchByVector once per request, from many
// goroutines at once: concurrent HTTP/gRPC requests plus the per-shard errgroup
// of Index.objectVectorSearch (adapters/repos/db/index.go:988-1028) reach
// Shard.objectVectorSearch -> SearchByVector (shard_read.go:246-252).  One
// query is far too little work for a GPU launch, so callers hand their query to
// a dispatcher thread that coalesces up to max_batch waiting requests into one
// wv_search_batch call and fans the rows back out.  Each caller blocks until its own row is written;
// no caller pointer is kept after its call returns (cgo pointer rules).
//
// Requests are grouped by (k, filtered): searchTimeEF depends on k
// (search.go:30-62), and a filtered group carries one allow bitmap per query
// (allow_stride_words), so the AUTO dispatch of search.go:64-79 (flat vs HNSW
// by allowList.Len()) is still decided per query inside the batch.  An allow
// list crosses as a bitmap or as ascending ids (the AllowList's Slice(),
// helpers/allow_list.go:19-118), written straight into the batch's row; a
// group whose requests all carry the same list sends it once (shared).
//
// Dispatch is latency-first ("natural batching"): one batch runs on the device
// at a time, and a free worker takes EVERY request queued meanwhile the moment
// the device is free -- a lone request on an idle device launches at once, and
// under load the batch size follows the arrival rate times one batch's device
// time.  Right after a batch of n finished, its callers resubmit as they wake:
// the next batch waits for n queued requests, or refill_us(n) past the
// batch's end, whichever comes first -- otherwise the first caller to return would be
// launched alone and the rest would queue behind it, two half batches taking
// turns (each caller then waits two device times).  max_wait_us is an
// optional linger for an idle device (the oldest request waits at most that
// long for company; 0 = none).  Two workers: while one fans a finished batch's
// rows back out, the other is already launching the next.  Each caller sleeps
// on its own condition variable and is woken alone when its row is written;
// the wakeups run as 8 chains (the worker wakes the heads, every woken caller
// the next of its chain), so a batch of n pays n/8 sequential wakeups, not n.
// The workers' staging buffers live as long as the batcher (no per-batch heap
// allocation once they have grown to max_batch).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
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

struct Request {
    const float* q;
    int k;
    const uint64_t* allow;        // bitmap, or
    uint64_t allow_nbits;
    const uint64_t* allow_ids;    // ascending ids (filtered with either)
    uint64_t n_ids = 0;
    bool filtered = false;
    uint64_t* out_ids;
    float* out_d;
    int32_t* out_n;
    // SearchByVectorDistance (search.go:90-158): a target, maxLimit and an
    // output of out_cap entries with a 64-bit count (dist: set)
    bool dist = false;
    float target = 0.f;
    int64_t max_limit = -1, out_cap = 0;
    int64_t* out_n64 = nullptr;
    int rc = WV_OK;
    std::string err;
    wait_clock::time_point arrived;
    // the caller's own wakeup: set and notified under m by its waker (the
    // worker, or the previous caller of its chain), which touches nothing of
    // the request after releasing m
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    Request* chain_next = nullptr;   // the caller this one wakes once it is woken
    uint64_t batch = 0;              // the batch that answered it (set before the wakeup)
    bool resub = false;              // its thread's previous call was answered by the last batch
};

// the batch that answered this thread's last call, per batcher: a caller
// resubmitting right after its answer is one the refill wait may expect
thread_local const void* tl_batcher = nullptr;
thread_local uint64_t tl_batch = 0;

void wake(Request* r) {
    std::lock_guard<std::mutex> g(r->m);
    r->done = true;
    r->cv.notify_one();
}

constexpr int WAKE_CHAINS = 8;
// how long the next batch waits for the last one's callers: a base plus a
// share per caller (the wakeup chains' hops), capped -- and only while they
// are coming back: the first resubmission within REFILL_GAP_US of the batch's
// end, each next within REFILL_GAP_US of the one before (an open-loop request
// at an idle device is launched at once)
int refill_us(int n) { return std::min(300, 50 + n); }
constexpr int REFILL_GAP_US = 40;   // (WV_BATCHER_REFILL_GAP_US; < 0: wait to the cap, round 5)

// one worker's staging, reused batch after batch
struct Staging {
    uint64_t seq = 0;   // the batch being run
    std::vector<Request*> take, g;
    std::vector<char> used;
    std::vector<float> q, ds, tg;
    std::vector<uint64_t> bits, ids;
    std::vector<int32_t> cnt;
    std::vector<int64_t> cnt64;
    int64_t cap = 0;    // (distance groups) entries per query in ids / ds
};

}  // namespace

struct wv_batcher {
    wv_index* ix = nullptr;
    wv_group* grp = nullptr;   // a multi-GPU group instead of one index
    int dim = 0;
    int max_batch = 256;
    int max_wait_us = 0;
    int refill_gap_us = REFILL_GAP_US;
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Request*> queue;
    bool stop = false;
    bool device_busy = false;      // a worker holds the device (one batch at a time)
    wait_clock::time_point idle_since{};   // when the last batch finished
    int expect = 0;                        // its size: the callers about to resubmit
    uint64_t seq_started = 0, seq_done = 0;   // batches taken / the last one finished
    int resub_seen = 0;                    // its callers back in the queue since
    wait_clock::time_point last_resub{};   // the latest of them
    // a worker waiting for company (refill or linger) wants this many queued:
    // submitters wake it only then (0: any submit at an idle device wakes)
    int wake_at = 0;
    std::vector<std::thread> th;   // the workers
    Staging st[2];
    uint64_t n_requests = 0, n_batches = 0, n_launch_rows = 0;

    static uint64_t nbits_of(const Request* r) {
        if (r->allow) return r->allow_nbits;
        return r->n_ids ? r->allow_ids[r->n_ids - 1] + 1 : 0;
    }
    static bool same_list(const Request* a, const Request* b) {
        if (a->allow || b->allow)
            return a->allow && b->allow && a->allow_nbits == b->allow_nbits &&
                   (a->allow == b->allow || std::memcmp(a->allow, b->allow, (a->allow_nbits + 63) / 64 * 8) == 0);
        return a->n_ids == b->n_ids &&
               (a->allow_ids == b->allow_ids || std::memcmp(a->allow_ids, b->allow_ids, a->n_ids * 8) == 0);
    }
    static void write_row(const Request* r, uint64_t* row) {
        if (r->allow) {
            const uint64_t w = (r->allow_nbits + 63) / 64;
            std::memcpy(row, r->allow, w * 8);
            if (r->allow_nbits & 63)   // bits past a request's own nbits are not allowed
                row[w - 1] &= (1ull << (r->allow_nbits & 63)) - 1;
        } else {
            for (uint64_t i = 0; i < r->n_ids; ++i) row[r->allow_ids[i] >> 6] |= 1ull << (r->allow_ids[i] & 63);
        }
    }

    // one (k, filtered) group on the device; returns the call's status
    int run_group(Staging& s) {
        const int n = (int)s.g.size();
        const int k = s.g[0]->k;
        const bool filtered = s.g[0]->filtered;
        s.q.resize((size_t)n * dim);
        for (int i = 0; i < n; ++i) std::memcpy(s.q.data() + (size_t)i * dim, s.g[i]->q, sizeof(float) * dim);
        uint64_t nbits = 0, stride = 0;
        if (filtered) {
            bool shared = true;
            for (int i = 1; i < n && shared; ++i) shared = same_list(s.g[0], s.g[i]);
            for (Request* r : s.g) nbits = std::max(nbits, nbits_of(r));
            nbits = std::max<uint64_t>(nbits, 1);   // (an empty list allows nothing)
            const uint64_t words = (nbits + 63) / 64;
            stride = shared ? 0 : words;
            s.bits.assign((size_t)(shared ? 1 : n) * words, 0);
            for (int i = 0; i < (shared ? 1 : n); ++i) write_row(s.g[i], s.bits.data() + (size_t)i * words);
        }
        const uint64_t* bits = filtered ? s.bits.data() : nullptr;
        if (s.g[0]->dist) {
            // one batched SearchByVectorDistance (same maxLimit in a group)
            s.cap = 0;
            s.tg.resize(n);
            for (int i = 0; i < n; ++i) {
                s.cap = std::max(s.cap, s.g[i]->out_cap);
                s.tg[i] = s.g[i]->target;
            }
            s.ids.resize((size_t)n * std::max<int64_t>(s.cap, 1));
            s.ds.resize((size_t)n * std::max<int64_t>(s.cap, 1));
            s.cnt64.resize(n);
            if (grp)
                return wv_group_search_by_vector_distance_batch(grp, s.q.data(), n, s.tg.data(), s.g[0]->max_limit,
                                                                bits, nbits, stride, s.ids.data(), s.ds.data(), s.cap,
                                                                s.cnt64.data());
            return wv_search_by_vector_distance_batch(ix, s.q.data(), n, s.tg.data(), s.g[0]->max_limit, bits, nbits,
                                                      stride, s.ids.data(), s.ds.data(), s.cap, s.cnt64.data());
        }
        s.ids.resize((size_t)n * k);
        s.ds.resize((size_t)n * k);
        s.cnt.resize(n);
        return grp ? wv_group_search_batch(grp, s.q.data(), n, k, 0, bits, nbits, stride, WV_MODE_AUTO, s.ids.data(),
                                           s.ds.data(), s.cnt.data())
                   : wv_search_batch(ix, s.q.data(), n, k, 0, bits, nbits, stride, WV_MODE_AUTO, s.ids.data(),
                                     s.ds.data(), s.cnt.data());
    }

    // every caller's row, then the heads of the wakeup chains
    static void fan_out(Staging& s, int rc, const std::string& msg) {
        const int k = s.g[0]->k;
        const size_t n = s.g.size();
        for (size_t i = 0; i < n; ++i) {
            Request* r = s.g[i];
            r->rc = rc;
            r->batch = s.seq;
            if (rc) {
                r->err = msg;
            } else if (r->dist) {
                const int64_t m = std::min(s.cnt64[i], r->out_cap);
                if (m > 0) {
                    std::memcpy(r->out_ids, s.ids.data() + i * s.cap, sizeof(uint64_t) * m);
                    std::memcpy(r->out_d, s.ds.data() + i * s.cap, sizeof(float) * m);
                }
                *r->out_n64 = s.cnt64[i];
            } else {
                const int m = s.cnt[i];
                std::memcpy(r->out_ids, s.ids.data() + i * k, sizeof(uint64_t) * m);
                std::memcpy(r->out_d, s.ds.data() + i * k, sizeof(float) * m);
                *r->out_n = m;
            }
            r->chain_next = i + WAKE_CHAINS < n ? s.g[i + WAKE_CHAINS] : nullptr;
        }
        for (size_t i = 0; i < n && i < (size_t)WAKE_CHAINS; ++i) wake(s.g[i]);
    }

    void loop(Staging& s) {
        std::unique_lock<std::mutex> l(mu);
        for (;;) {
            cv_work.wait(l, [&] { return (!queue.empty() && !device_busy) || (stop && queue.empty()); });
            if (queue.empty()) return;   // (stop)
            const int want = std::min(expect, max_batch);
            if (!stop && (int)queue.size() < want) {
                // the finished batch's callers are still resubmitting: wait
                // for them while they keep coming, up to the cap
                const auto cap = idle_since + std::chrono::microseconds(refill_us(want));
                const auto gap = std::chrono::microseconds(refill_gap_us);
                for (;;) {
                    const auto now = wait_clock::now();
                    const auto until = refill_gap_us < 0 ? cap : std::min(cap, (resub_seen ? last_resub : idle_since) + gap);
                    if (now >= until) break;
                    wake_at = want;
                    const bool full = cv_work.wait_until(
                        l, until, [&] { return stop || device_busy || (int)queue.size() >= want; });
                    wake_at = 0;
                    if (full) break;
                }
                if (device_busy || queue.empty()) continue;   // (the other worker took them)
            }
            if (max_wait_us > 0 && (int)queue.size() < max_batch && !stop) {
                // linger at an idle device: until max_batch or the oldest request's deadline
                const auto deadline = queue.front()->arrived + std::chrono::microseconds(max_wait_us);
                wake_at = max_batch;
                cv_work.wait_until(l, deadline, [&] { return stop || (int)queue.size() >= max_batch; });
                wake_at = 0;
                if (device_busy || queue.empty()) continue;   // (the other worker took them)
            }
            device_busy = true;
            s.seq = ++seq_started;
            s.take.clear();
            while (!queue.empty() && (int)s.take.size() < max_batch) {
                s.take.push_back(queue.front());
                queue.pop_front();
            }
            l.unlock();
            // group by (k, filtered) -- distance searches by (maxLimit,
            // filtered) -- keeping arrival order inside a group
            s.used.assign(s.take.size(), 0);
            size_t left = s.take.size();
            for (size_t i = 0; i < s.take.size(); ++i) {
                if (s.used[i]) continue;
                s.g.clear();
                for (size_t j = i; j < s.take.size(); ++j) {
                    const Request* a = s.take[i];
                    const Request* c = s.take[j];
                    if (s.used[j] || c->k != a->k || c->filtered != a->filtered || c->dist != a->dist ||
                        (a->dist && c->max_limit != a->max_limit))
                        continue;
                    s.used[j] = 1;
                    s.g.push_back(s.take[j]);
                }
                left -= s.g.size();
                const int rc = run_group(s);
                const std::string msg = rc ? wv_last_error() : std::string();
                if (left == 0) {
                    // the device is free: the other worker launches the next
                    // batch while this one wakes its callers
                    l.lock();
                    device_busy = false;
                    idle_since = wait_clock::now();
                    expect = (int)s.take.size();
                    seq_done = s.seq;
                    resub_seen = 0;
                    n_batches++;
                    n_launch_rows += s.take.size();
                    l.unlock();
                    cv_work.notify_all();
                }
                fan_out(s, rc, msg);
            }
            l.lock();
        }
    }
};

extern "C" {

static int create_batcher(wv_index* ix, wv_group* grp, int dim, int max_batch, int max_wait_us, wv_batcher** out) {
    if ((!ix && !grp) || !out || dim <= 0 || max_batch <= 0 || max_wait_us < 0) {
        wv_internal_set_error("wv_batcher_create: bad argument");
        return WV_EINVAL;
    }
    auto* b = new wv_batcher();
    b->ix = ix;
    b->grp = grp;
    b->dim = dim;
    b->max_batch = max_batch;
    b->max_wait_us = max_wait_us;
    if (const char* e = std::getenv("WV_BATCHER_REFILL_GAP_US")) b->refill_gap_us = std::atoi(e);
    for (int w = 0; w < 2; ++w) b->th.emplace_back([b, w] { b->loop(b->st[w]); });
    *out = b;
    return WV_OK;
}

int wv_batcher_create(wv_index* ix, int dim, int max_batch, int max_wait_us, wv_batcher** out) {
    return create_batcher(ix, nullptr, dim, max_batch, max_wait_us, out);
}

int wv_batcher_create_group(wv_group* g, int dim, int max_batch, int max_wait_us, wv_batcher** out) {
    return create_batcher(nullptr, g, dim, max_batch, max_wait_us, out);
}

static int submit(wv_batcher* b, Request& r) {
    r.arrived = wait_clock::now();
    bool notify = false;
    {
        std::lock_guard<std::mutex> l(b->mu);
        if (b->stop) {
            wv_internal_set_error("wv_batcher_search: batcher is shut down");
            return WV_ESTATE;
        }
        b->queue.push_back(&r);
        b->n_requests++;
        if (tl_batcher == b && tl_batch == b->seq_done && b->seq_done) {
            r.resub = true;
            b->resub_seen++;
            b->last_resub = r.arrived;
        }
        // a busy device: the worker that frees it takes the queue; a worker
        // waiting for company: only once the count it waits for is there
        notify = !b->device_busy && (b->wake_at == 0 || (int)b->queue.size() >= b->wake_at);
    }
    if (notify) b->cv_work.notify_all();   // (two workers: whichever is free)
    {
        std::unique_lock<std::mutex> l(r.m);
        r.cv.wait(l, [&] { return r.done; });
    }
    if (r.chain_next) wake(r.chain_next);
    tl_batcher = b;
    tl_batch = r.batch;
    if (r.rc) wv_internal_set_error(r.err.c_str());
    return r.rc;
}
int wv_batcher_search(wv_batcher* b, const float* vector, int k, const uint64_t* allow_bits, uint64_t allow_nbits,
                      uint64_t* out_ids, float* out_dists, int32_t* out_n) {
    if (!b || !vector || k <= 0 || !out_ids || !out_dists || !out_n) {
        wv_internal_set_error("wv_batcher_search: bad argument");
        return WV_EINVAL;
    }
    Request r;
    r.q = vector;
    r.k = k;
    r.allow = allow_bits;
    r.allow_nbits = allow_bits ? allow_nbits : 0;
    r.allow_ids = nullptr;
    r.filtered = allow_bits != nullptr;
    r.out_ids = out_ids;
    r.out_d = out_dists;
    r.out_n = out_n;
    return submit(b, r);
}

int wv_batcher_search_ids(wv_batcher* b, const float* vector, int k, int filtered, const uint64_t* allow_ids,
                          uint64_t n_allow, uint64_t* out_ids, float* out_dists, int32_t* out_n) {
    if (!b || !vector || k <= 0 || !out_ids || !out_dists || !out_n || (n_allow && !allow_ids)) {
        wv_internal_set_error("wv_batcher_search_ids: bad argument");
        return WV_EINVAL;
    }
    for (uint64_t i = 1; i < n_allow; ++i)
        if (allow_ids[i] <= allow_ids[i - 1]) {
            wv_internal_set_error("wv_batcher_search_ids: allow ids must be strictly ascending");
            return WV_EINVAL;
        }
    Request r;
    r.q = vector;
    r.k = k;
    r.allow = nullptr;
    r.allow_nbits = 0;
    r.allow_ids = allow_ids;
    r.n_ids = filtered ? n_allow : 0;
    r.filtered = filtered != 0;
    r.out_ids = out_ids;
    r.out_d = out_dists;
    r.out_n = out_n;
    return submit(b, r);
}

int wv_batcher_search_distance_ids(wv_batcher* b, const float* vector, float target_distance, int64_t max_limit,
                                   int filtered, const uint64_t* allow_ids, uint64_t n_allow, uint64_t* out_ids,
                                   float* out_dists, int64_t out_cap, int64_t* out_n) {
    if (!b || !vector || !out_n || out_cap < 0 || (out_cap && (!out_ids || !out_dists)) || (n_allow && !allow_ids)) {
        wv_internal_set_error("wv_batcher_search_distance_ids: bad argument");
        return WV_EINVAL;
    }
    for (uint64_t i = 1; i < n_allow; ++i)
        if (allow_ids[i] <= allow_ids[i - 1]) {
            wv_internal_set_error("wv_batcher_search_distance_ids: allow ids must be strictly ascending");
            return WV_EINVAL;
        }
    Request r;
    r.q = vector;
    r.k = 0;
    r.allow = nullptr;
    r.allow_nbits = 0;
    r.allow_ids = allow_ids;
    r.n_ids = filtered ? n_allow : 0;
    r.filtered = filtered != 0;
    r.out_ids = out_ids;
    r.out_d = out_dists;
    r.out_n = nullptr;
    r.dist = true;
    r.target = target_distance;
    r.max_limit = max_limit;
    r.out_cap = out_cap;
    r.out_n64 = out_n;
    return submit(b, r);
}

int wv_batcher_stats(wv_batcher* b, uint64_t* requests, uint64_t* batches) {
    if (!b) return WV_EINVAL;
    std::lock_guard<std::mutex> l(b->mu);
    if (requests) *requests = b->n_requests;
    if (batches) *batches = b->n_batches;
    return WV_OK;
}

int wv_batcher_destroy(wv_batcher* b) {
    if (!b) return WV_OK;
    {
        std::lock_guard<std::mutex> l(b->mu);
        b->stop = true;
    }
    b->cv_work.notify_all();
    for (auto& t : b->th) t.join();   // the workers drain the queue before they exit
    delete b;
    return WV_OK;
}

}  // extern "C"
