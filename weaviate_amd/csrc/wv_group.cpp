// wv_group.cpp -- one process, several MI355X: the in-library multi-GPU group.
//
// The reference serves one class from several shards and merges their
// answers (adapters/repos/db/index.go:967-1044: objectVectorSearch fans out
// one search per shard, then sorts the union by distance and cuts to the
// limit).  The Go server is a single process, so the GPUs of a node are
// driven from one process here: a group owns one wv_index per device and
// exposes the batched search signature of wv_search_batch.
//
//   WV_GROUP_SHARD    the corpus is split by id range (global id = base_i +
//                     local id, base_i a multiple of 64 so allow bitmaps slice
//                     by words).  Every member searches the whole batch over
//                     its shard on its own stream; the per-shard top-k lists
//                     are gathered to the root device over RCCL (one
//                     communicator from ncclCommInitAll, one grouped
//                     ncclGather per output array) and merged there by
//                     wv_merge_shards_device -- the sort-and-cut of
//                     index.go:1030-1043 on the device.
//   WV_GROUP_REPLICA  every member holds the whole corpus; a batch is split
//                     into n contiguous query ranges, one per member, with no
//                     collective (the layout for a corpus that fits one GPU:
//                     an HNSW search costs the same per query on any shard,
//                     so query-splitting scales where corpus-splitting
//                     does not).
//
// Members sharing a device (a one-GPU box rehearsing the layout) cannot join
// one communicator, so their lists reach the root by device copies instead;
// WV_GROUP_NO_RCCL=1 forces the copy path (peer copies over xGMI) everywhere.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wvgpu.h"

extern "C" void wv_internal_set_error(const char* msg);

namespace {

int gfail(int code, const std::string& m) {
    wv_internal_set_error(m.c_str());
    return code;
}

#define G_HIP(x)                                                                                 \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) return gfail(WV_EDEVICE, std::string("hip: ") + hipGetErrorString(e_)); \
    } while (0)
#define G_NCCL(x)                                                                                \
    do {                                                                                         \
        ncclResult_t r_ = (x);                                                                   \
        if (r_ != ncclSuccess) return gfail(WV_EDEVICE, std::string("rccl: ") + ncclGetErrorString(r_)); \
    } while (0)

struct DBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(bytes, 64));
        if (e == hipSuccess) n = std::max<size_t>(bytes, 64);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// pinned host staging: an async copy from it is truly asynchronous, and it
// outlives the call, so nothing has to wait for a copy before the call returns
struct HBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault);
        if (e == hipSuccess) n = std::max<size_t>(bytes, 64);
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

struct Member {
    wv_index* ix = nullptr;
    int dev = 0;
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    uint64_t base = 0, cap = 0, rows = 0;   // global ids [base, base + cap); rows written below base + rows
    DBuf q, allow, ids, d, n;
    HBuf h_allow;                           // this member's slice of the allow list
    int rc = WV_OK;
    std::string err;
};

}  // namespace

struct wv_group {
    int layout = WV_GROUP_SHARD;
    int dim = 0, ld = 0;
    uint64_t capacity = 0;
    std::vector<Member> m;
    std::vector<ncclComm_t> comms;   // empty: copy path
    DBuf r_ids, r_d, r_n, o_ids, o_d, o_n;   // on the root (member 0's device)
    HBuf h_q;                                // the batch, staged once for every member's upload
    std::mutex mu;
    // one persistent host thread per member (more than one member): a call
    // hands every worker the same task instead of spawning a thread per
    // member per search
    struct Pool {
        std::mutex mu, call;
        std::condition_variable cv, done;
        uint64_t gen = 0;
        int pending = 0;
        bool stop = false;
        const std::function<int(int)>* task = nullptr;
        std::vector<std::thread> th;
    } pool;
};

namespace {

// member i's pool worker: its device set once, then every task handed out
void pool_worker(wv_group* g, int i) {
    Member& mb = g->m[i];
    const bool dev_ok = hipSetDevice(mb.dev) == hipSuccess;
    auto& P = g->pool;
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(P.mu);
    for (;;) {
        P.cv.wait(l, [&] { return P.stop || P.gen != seen; });
        if (P.stop) return;
        seen = P.gen;
        const std::function<int(int)>* task = P.task;
        l.unlock();
        if (!dev_ok) {
            mb.rc = WV_EDEVICE;
            mb.err = "hipSetDevice";
        } else {
            mb.rc = (*task)(i);
            if (mb.rc) mb.err = wv_last_error();
        }
        l.lock();
        if (--P.pending == 0) P.done.notify_all();
    }
}

void pool_start(wv_group* g) {
    if (g->m.size() < 2) return;
    for (size_t i = 0; i < g->m.size(); ++i) g->pool.th.emplace_back(pool_worker, g, (int)i);
}

void pool_stop(wv_group* g) {
    {
        std::lock_guard<std::mutex> l(g->pool.mu);
        g->pool.stop = true;
    }
    g->pool.cv.notify_all();
    for (auto& t : g->pool.th) t.join();
    g->pool.th.clear();
}

// run f(i) for every member, each on its own device: one member inline on
// the caller's thread (its device restored after), several on the pool's
// workers in parallel; first error wins
template <class F>
int each_member(wv_group* g, F&& f) {
    if (g->pool.th.empty()) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        for (size_t i = 0; i < g->m.size(); ++i) {
            Member& mb = g->m[i];
            if (hipSetDevice(mb.dev) != hipSuccess) {
                mb.rc = WV_EDEVICE;
                mb.err = "hipSetDevice";
                continue;
            }
            mb.rc = f((int)i);
            if (mb.rc) mb.err = wv_last_error();
        }
        (void)hipSetDevice(prev);
    } else {
        const std::function<int(int)> task = [&](int i) { return f(i); };
        auto& P = g->pool;
        std::lock_guard<std::mutex> c(P.call);
        {
            std::lock_guard<std::mutex> l(P.mu);
            P.task = &task;
            P.pending = (int)g->m.size();
            ++P.gen;
        }
        P.cv.notify_all();
        std::unique_lock<std::mutex> l(P.mu);
        P.done.wait(l, [&] { return P.pending == 0; });
        P.task = nullptr;
    }
    for (auto& mb : g->m)
        if (mb.rc) return gfail(mb.rc, mb.err);
    return WV_OK;
}

// the members owning global ids [lo, hi): (member, local lo, local hi)
struct Span {
    int i;
    uint64_t lo, hi;
};
std::vector<Span> spans(const wv_group* g, uint64_t lo, uint64_t hi) {
    std::vector<Span> out;
    for (size_t i = 0; i < g->m.size(); ++i) {
        const Member& mb = g->m[i];
        if (g->layout == WV_GROUP_REPLICA) {
            out.push_back({(int)i, lo, hi});
            continue;
        }
        const uint64_t a = std::max(lo, mb.base), b = std::min(hi, mb.base + mb.cap);
        if (a < b) out.push_back({(int)i, a - mb.base, b - mb.base});
    }
    return out;
}

// wait for every member's stream (error paths: the pinned staging must be
// idle before a later call rewrites it)
void drain_members(wv_group* g) {
    for (auto& mb : g->m) {
        if (hipSetDevice(mb.dev) == hipSuccess && mb.s) (void)hipStreamSynchronize(mb.s);
    }
}

int search_shards(wv_group* g, const float* queries, int nq, int k, int ef, const uint64_t* allow_bits,
                  uint64_t allow_nbits, uint64_t allow_stride, int mode, uint64_t* out_ids, float* out_d,
                  int32_t* out_n) {
    const int n = (int)g->m.size();
    const size_t nk = (size_t)nq * k;
    // 0. the batch into pinned staging once (a previous call's copies from
    // it have landed: every call ends after its root stream, which waited
    // for every member's results, hence for their copies of the staging)
    G_HIP(g->h_q.ensure((size_t)nq * g->dim * 4));
    std::memcpy(g->h_q.p, queries, (size_t)nq * g->dim * 4);
    // 1. every member: its queries, its slice of the allow list, its search
    // (queued, not waited for: the staging is pinned and owned by the group)
    int rc = each_member(g, [&](int i) -> int {
        Member& mb = g->m[i];
        G_HIP(mb.q.ensure((size_t)nq * g->ld * 4));
        G_HIP(mb.ids.ensure(nk * 8));
        G_HIP(mb.d.ensure(nk * 4));
        G_HIP(mb.n.ensure((size_t)nq * 4));
        G_HIP(hipMemcpy2DAsync(mb.q.p, (size_t)g->ld * 4, g->h_q.p, (size_t)g->dim * 4, (size_t)g->dim * 4, nq,
                               hipMemcpyHostToDevice, mb.s));
        const uint64_t* d_allow = nullptr;
        uint64_t nbits = 0, stride = 0;
        if (allow_bits) {
            // global bits [base, base + cap) -> local bits [0, cap); base % 64 == 0
            nbits = allow_nbits > mb.base ? std::min(allow_nbits - mb.base, mb.cap) : 0;
            const uint64_t w = (nbits + 63) / 64, w0 = mb.base / 64;
            const uint64_t gw = allow_stride ? allow_stride : (allow_nbits + 63) / 64;
            const int rows_a = allow_stride ? nq : 1;
            const uint64_t ws = std::max<uint64_t>(w, 1);
            stride = allow_stride ? ws : 0;
            G_HIP(mb.h_allow.ensure((size_t)rows_a * ws * 8));
            auto* slice = static_cast<uint64_t*>(mb.h_allow.p);
            for (int r = 0; r < rows_a; ++r)
                for (uint64_t j = 0; j < ws; ++j)
                    slice[(size_t)r * ws + j] = j < w && w0 + j < gw ? allow_bits[(size_t)r * gw + w0 + j] : 0;
            G_HIP(mb.allow.ensure((size_t)rows_a * ws * 8));
            G_HIP(hipMemcpyAsync(mb.allow.p, slice, (size_t)rows_a * ws * 8, hipMemcpyHostToDevice, mb.s));
            d_allow = static_cast<const uint64_t*>(mb.allow.p);
        }
        return wv_search_batch_device(mb.ix, static_cast<const float*>(mb.q.p), nq, k, ef, d_allow, nbits, stride,
                                      mode, static_cast<uint64_t*>(mb.ids.p), static_cast<float*>(mb.d.p),
                                      static_cast<int32_t*>(mb.n.p), mb.s);
    });
    if (rc) {
        drain_members(g);   // no copy from the staging may still be in flight
        return rc;
    }
    // 2.-3. gather on the root, merge, results to the host; on an error every
    // member's stream is drained before returning
    rc = [&]() -> int {
        // 2. gather the per-shard lists on the root
        Member& root = g->m[0];
        G_HIP(hipSetDevice(root.dev));
        G_HIP(g->r_ids.ensure((size_t)n * nk * 8));
        G_HIP(g->r_d.ensure((size_t)n * nk * 4));
        G_HIP(g->r_n.ensure((size_t)n * nq * 4));
        G_HIP(g->o_ids.ensure(nk * 8));
        G_HIP(g->o_d.ensure(nk * 4));
        G_HIP(g->o_n.ensure((size_t)nq * 4));
        auto* rid = static_cast<uint64_t*>(g->r_ids.p);
        auto* rd = static_cast<float*>(g->r_d.p);
        auto* rn = static_cast<int32_t*>(g->r_n.p);
        if (!g->comms.empty()) {
            G_NCCL(ncclGroupStart());
            for (int i = 0; i < n; ++i) {
                Member& mb = g->m[i];
                const bool is_root = i == 0;
                G_NCCL(ncclGather(mb.ids.p, is_root ? rid : nullptr, nk, ncclUint64, 0, g->comms[i], mb.s));
                G_NCCL(ncclGather(mb.d.p, is_root ? rd : nullptr, nk, ncclFloat32, 0, g->comms[i], mb.s));
                G_NCCL(ncclGather(mb.n.p, is_root ? rn : nullptr, (size_t)nq, ncclInt32, 0, g->comms[i], mb.s));
            }
            G_NCCL(ncclGroupEnd());
            // (no drain of the senders: their next writes to ids / d / n are
            // queued on the same streams, after these sends; and the root's
            // gather completing -- waited for below -- means every sender's
            // data left, so the staging the next call rewrites is free)
            G_HIP(hipSetDevice(root.dev));
        } else {
            for (int i = 0; i < n; ++i) {
                Member& mb = g->m[i];
                G_HIP(hipSetDevice(mb.dev));
                G_HIP(hipMemcpyPeerAsync(rid + (size_t)i * nk, root.dev, mb.ids.p, mb.dev, nk * 8, mb.s));
                G_HIP(hipMemcpyPeerAsync(rd + (size_t)i * nk, root.dev, mb.d.p, mb.dev, nk * 4, mb.s));
                G_HIP(hipMemcpyPeerAsync(rn + (size_t)i * nq, root.dev, mb.n.p, mb.dev, (size_t)nq * 4, mb.s));
                G_HIP(hipEventRecord(mb.done, mb.s));
            }
            G_HIP(hipSetDevice(root.dev));
            for (int i = 1; i < n; ++i) G_HIP(hipStreamWaitEvent(root.s, g->m[i].done, 0));
        }
        // 3. merge on the root (index.go:1030-1043), results to the host
        int rc = wv_merge_shards_device(rd, rid, rn, n, nq, k, static_cast<float*>(g->o_d.p),
                                    static_cast<uint64_t*>(g->o_ids.p), static_cast<int32_t*>(g->o_n.p), root.s);
        if (rc) return rc;
        G_HIP(hipMemcpyAsync(out_ids, g->o_ids.p, nk * 8, hipMemcpyDeviceToHost, root.s));
        G_HIP(hipMemcpyAsync(out_d, g->o_d.p, nk * 4, hipMemcpyDeviceToHost, root.s));
        G_HIP(hipMemcpyAsync(out_n, g->o_n.p, (size_t)nq * 4, hipMemcpyDeviceToHost, root.s));
        // the one wait of a call (its results go to the host): the root's
        // stream waited for every member's copies (events) or gather, so the
        // members' streams need no drain -- the next call's work queues
        // behind this call's on each of them
        G_HIP(hipStreamSynchronize(root.s));
        return WV_OK;
    }();
    if (rc) drain_members(g);
    return rc;
}

int search_replicas(wv_group* g, const float* queries, int nq, int k, int ef, const uint64_t* allow_bits,
                    uint64_t allow_nbits, uint64_t allow_stride, int mode, uint64_t* out_ids, float* out_d,
                    int32_t* out_n) {
    const int n = (int)g->m.size();
    const int per = (nq + n - 1) / n;
    return each_member(g, [&](int i) -> int {
        const int q0 = std::min(nq, i * per), q1 = std::min(nq, q0 + per);
        if (q1 <= q0) return WV_OK;
        const uint64_t* al = allow_bits ? allow_bits + (allow_stride ? (size_t)q0 * allow_stride : 0) : nullptr;
        return wv_search_batch(g->m[i].ix, queries + (size_t)q0 * g->dim, q1 - q0, k, ef, al, allow_nbits,
                               allow_stride, mode, out_ids + (size_t)q0 * k, out_d + (size_t)q0 * k, out_n + q0);
    });
}

void destroy_members(wv_group* g) {
    for (auto c : g->comms) (void)ncclCommDestroy(c);
    g->comms.clear();
    for (auto& mb : g->m) {
        (void)hipSetDevice(mb.dev);
        for (DBuf* b : {&mb.q, &mb.allow, &mb.ids, &mb.d, &mb.n}) b->release();
        mb.h_allow.release();
        if (mb.done) (void)hipEventDestroy(mb.done);
        if (mb.s) (void)hipStreamDestroy(mb.s);
        if (mb.ix) wv_index_destroy(mb.ix);
    }
    if (!g->m.empty()) {
        (void)hipSetDevice(g->m[0].dev);
        for (DBuf* b : {&g->r_ids, &g->r_d, &g->r_n, &g->o_ids, &g->o_d, &g->o_n}) b->release();
    }
    g->h_q.release();
    g->m.clear();
}

}  // namespace

extern "C" {

int wv_group_create(const int* devices, int n_devices, int dim, int metric, const wv_config* cfg, uint64_t capacity,
                    int layout, wv_group** out) {
    if (!devices || n_devices < 1 || dim < 1 || !cfg || !out || capacity == 0 ||
        (layout != WV_GROUP_SHARD && layout != WV_GROUP_REPLICA))
        return gfail(WV_EINVAL, "wv_group_create: bad argument");
    // the device merge (wv_merge_shards_device) takes at most 16 shard lists
    if (layout == WV_GROUP_SHARD && n_devices > 16)
        return gfail(WV_EINVAL, "wv_group_create: at most 16 shard members");
    int n_vis = 0;
    G_HIP(hipGetDeviceCount(&n_vis));
    for (int i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= n_vis) return gfail(WV_EINVAL, "wv_group_create: no such device");
    auto* g = new wv_group();
    g->layout = layout;
    g->dim = dim;
    g->capacity = capacity;
    // shard capacity: a multiple of 64 ids, so allow bitmaps slice by words
    const uint64_t shard = layout == WV_GROUP_SHARD ? ((capacity + n_devices - 1) / n_devices + 63) / 64 * 64 : capacity;
    g->m.resize(n_devices);
    for (int i = 0; i < n_devices; ++i) {
        Member& mb = g->m[i];
        mb.dev = devices[i];
        mb.base = layout == WV_GROUP_SHARD ? (uint64_t)i * shard : 0;
        mb.cap = layout == WV_GROUP_SHARD ? std::min(shard, capacity > mb.base ? capacity - mb.base : 0) : capacity;
        if (mb.cap == 0) mb.cap = 64;   // an empty tail shard still answers (with nothing)
        wv_config c = *cfg;
        c.device = mb.dev;
        c.id_base = cfg->id_base + mb.base;
        int rc = wv_index_create(dim, metric, &c, mb.cap, &mb.ix);
        if (rc == WV_OK && hipSetDevice(mb.dev) == hipSuccess &&
            hipStreamCreateWithFlags(&mb.s, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&mb.done, hipEventDisableTiming) == hipSuccess) {
            continue;
        }
        const std::string e = rc ? wv_last_error() : "wv_group_create: stream/event";
        destroy_members(g);
        delete g;
        return gfail(rc ? rc : WV_EDEVICE, e);
    }
    g->ld = wv_index_query_ld(g->m[0].ix);
    std::vector<int> devs(devices, devices + n_devices);
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (layout == WV_GROUP_SHARD && n_devices > 1 && distinct && !std::getenv("WV_GROUP_NO_RCCL")) {
        g->comms.resize(n_devices);
        ncclResult_t r = ncclCommInitAll(g->comms.data(), n_devices, devs.data());
        if (r != ncclSuccess) {
            g->comms.clear();
            destroy_members(g);
            delete g;
            return gfail(WV_EDEVICE, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        }
    }
    pool_start(g);
    *out = g;
    return WV_OK;
}

int wv_group_destroy(wv_group* g) {
    if (!g) return WV_OK;
    pool_stop(g);
    destroy_members(g);
    delete g;
    return WV_OK;
}

int wv_group_info(const wv_group* g, int* n_members, int* uses_rccl) {
    if (!g) return gfail(WV_EINVAL, "wv_group_info: bad argument");
    if (n_members) *n_members = (int)g->m.size();
    if (uses_rccl) *uses_rccl = g->comms.empty() ? 0 : 1;
    return WV_OK;
}

int wv_group_member(wv_group* g, int i, wv_index** ix, uint64_t* id_base, uint64_t* capacity) {
    if (!g || i < 0 || i >= (int)g->m.size()) return gfail(WV_EINVAL, "wv_group_member: bad argument");
    if (ix) *ix = g->m[i].ix;
    if (id_base) *id_base = g->m[i].base;
    if (capacity) *capacity = g->m[i].cap;
    return WV_OK;
}

int wv_group_upload_vectors(wv_group* g, const float* rows, uint64_t n, uint64_t first_id) {
    if (!g || (n && !rows) || first_id + n > g->capacity) return gfail(WV_EINVAL, "wv_group_upload_vectors: bad argument");
    std::lock_guard<std::mutex> l(g->mu);
    const auto sp = spans(g, first_id, first_id + n);
    for (const Span& s : sp) {
        Member& mb = g->m[s.i];
        const uint64_t g_lo = (g->layout == WV_GROUP_SHARD ? mb.base : 0) + s.lo;
        int rc = wv_index_upload_vectors(mb.ix, rows + (g_lo - first_id) * (size_t)g->dim, s.hi - s.lo, s.lo);
        if (rc) return rc;
        mb.rows = std::max(mb.rows, s.hi);
    }
    return WV_OK;
}

int wv_group_build_graph(wv_group* g, int ef_construction, uint64_t seed, int batch_div) {
    if (!g) return gfail(WV_EINVAL, "wv_group_build_graph: bad argument");
    std::lock_guard<std::mutex> l(g->mu);
    // every shard builds its own graph, as every Weaviate shard holds its own hnsw
    return each_member(g, [&](int i) -> int {
        if (g->m[i].rows == 0) return WV_OK;
        return wv_index_build_graph(g->m[i].ix, ef_construction, seed, batch_div);
    });
}

static int route_ids(wv_group* g, const uint64_t* ids, uint64_t n, const float* rows, int what) {
    if (!g || (n && !ids) || (what == 0 && n && !rows)) return gfail(WV_EINVAL, "wv_group: bad argument");
    std::lock_guard<std::mutex> l(g->mu);
    for (uint64_t j = 0; j < n; ++j)
        if (ids[j] >= g->capacity) return gfail(WV_EINVAL, "wv_group: id beyond capacity");
    for (size_t i = 0; i < g->m.size(); ++i) {
        Member& mb = g->m[i];
        std::vector<uint64_t> loc;
        std::vector<float> r;
        for (uint64_t j = 0; j < n; ++j) {
            const bool mine = g->layout == WV_GROUP_REPLICA || (ids[j] >= mb.base && ids[j] < mb.base + mb.cap);
            if (!mine) continue;
            loc.push_back(ids[j] - (g->layout == WV_GROUP_SHARD ? mb.base : 0));
            if (what == 0) r.insert(r.end(), rows + j * (size_t)g->dim, rows + (j + 1) * (size_t)g->dim);
        }
        if (loc.empty()) continue;
        int rc = what == 0   ? wv_index_add(mb.ix, loc.data(), r.data(), loc.size())
                 : what == 1 ? wv_index_add_tombstones(mb.ix, loc.data(), loc.size())
                             : wv_index_remove_tombstones(mb.ix, loc.data(), loc.size());
        if (rc) return rc;
        if (what == 0)
            for (uint64_t id : loc) mb.rows = std::max(mb.rows, id + 1);
    }
    return WV_OK;
}

int wv_group_add(wv_group* g, const uint64_t* ids, const float* rows, uint64_t n) { return route_ids(g, ids, n, rows, 0); }
int wv_group_add_tombstones(wv_group* g, const uint64_t* ids, uint64_t n) { return route_ids(g, ids, n, nullptr, 1); }
int wv_group_remove_tombstones(wv_group* g, const uint64_t* ids, uint64_t n) {
    return route_ids(g, ids, n, nullptr, 2);
}

int wv_group_update_config(wv_group* g, const wv_config* cfg) {
    if (!g || !cfg) return gfail(WV_EINVAL, "wv_group_update_config: bad argument");
    std::lock_guard<std::mutex> l(g->mu);
    for (auto& mb : g->m) {
        wv_config c = *cfg;
        c.device = mb.dev;
        c.id_base = cfg->id_base + mb.base;
        int rc = wv_index_update_config(mb.ix, &c);
        if (rc) return rc;
    }
    return WV_OK;
}

// SearchByVectorDistance over the group (index.go:967-1044 with a distance:
// every shard answers within the target, the union sorted by distance): a
// replica group asks one member; a shard group asks each member its batch
// over its id range (the allow lists sliced as in search_shards) and merges
// each query's lists by (distance, id).
int wv_group_search_by_vector_distance_batch(wv_group* g, const float* queries, int nq, const float* targets,
                                             int64_t max_limit, const uint64_t* allow_bits, uint64_t allow_nbits,
                                             uint64_t allow_stride, uint64_t* out_ids, float* out_dists,
                                             int64_t out_cap, int64_t* out_n) {
    if (!g || nq < 0 || out_cap < 0 || (nq && (!queries || !targets || !out_n)) ||
        (out_cap && nq && (!out_ids || !out_dists)))
        return gfail(WV_EINVAL, "wv_group_search_by_vector_distance_batch: bad argument");
    if (nq == 0) return WV_OK;
    std::lock_guard<std::mutex> l(g->mu);
    if (g->layout == WV_GROUP_REPLICA || g->m.size() == 1)
        return wv_search_by_vector_distance_batch(g->m[0].ix, queries, nq, targets, max_limit, allow_bits, allow_nbits,
                                                  allow_stride, out_ids, out_dists, out_cap, out_n);
    // each member's lists in full (a shard's entries past the merged cut are
    // dropped only after the merge)
    const int n = (int)g->m.size();
    std::vector<std::vector<uint64_t>> mids(n);
    std::vector<std::vector<float>> mds(n);
    std::vector<std::vector<int64_t>> mcnt(n, std::vector<int64_t>(nq));
    std::vector<int64_t> mcap(n);
    for (int i = 0; i < n; ++i) {
        Member& mb = g->m[i];
        std::vector<uint64_t> slice;
        uint64_t nbits = 0, stride = 0;
        if (allow_bits) {
            nbits = allow_nbits > mb.base ? std::min(allow_nbits - mb.base, mb.cap) : 0;
            const uint64_t w = (nbits + 63) / 64, w0 = mb.base / 64;
            const uint64_t gw = allow_stride ? allow_stride : (allow_nbits + 63) / 64;
            const int rows_a = allow_stride ? nq : 1;
            const uint64_t ws = std::max<uint64_t>(w, 1);
            stride = allow_stride ? ws : 0;
            slice.assign((size_t)rows_a * ws, 0);
            for (int r = 0; r < rows_a; ++r)
                for (uint64_t j = 0; j < ws; ++j)
                    slice[(size_t)r * ws + j] = j < w && w0 + j < gw ? allow_bits[(size_t)r * gw + w0 + j] : 0;
        }
        int64_t cap = std::max<int64_t>(out_cap, 1);
        for (int pass = 0; pass < 2; ++pass) {   // (once more with room for every result)
            mids[i].assign((size_t)nq * cap, 0);
            mds[i].assign((size_t)nq * cap, 0.f);
            const int rc = wv_search_by_vector_distance_batch(mb.ix, queries, nq, targets, max_limit,
                                                              allow_bits ? slice.data() : nullptr, nbits, stride,
                                                              mids[i].data(), mds[i].data(), cap, mcnt[i].data());
            if (rc) return rc;
            const int64_t mx = *std::max_element(mcnt[i].begin(), mcnt[i].end());
            if (mx <= cap) break;
            cap = mx;
        }
        mcap[i] = cap;
    }
    for (int q = 0; q < nq; ++q) {
        std::vector<std::pair<float, uint64_t>> u;
        for (int i = 0; i < n; ++i)
            for (int64_t j = 0; j < mcnt[i][q]; ++j)
                u.emplace_back(mds[i][(size_t)q * mcap[i] + j], mids[i][(size_t)q * mcap[i] + j]);
        std::sort(u.begin(), u.end());
        out_n[q] = (int64_t)u.size();
        for (int64_t j = 0; j < std::min<int64_t>(out_cap, (int64_t)u.size()); ++j) {
            out_ids[(size_t)q * out_cap + j] = u[j].second;
            out_dists[(size_t)q * out_cap + j] = u[j].first;
        }
    }
    return WV_OK;
}

int wv_group_search_batch(wv_group* g, const float* queries, int nq, int k, int ef, const uint64_t* allow_bits,
                          uint64_t allow_nbits, uint64_t allow_stride_words, int mode, uint64_t* out_ids,
                          float* out_dists, int32_t* out_n) {
    if (!g || nq < 0 || k < 1 || (nq && (!queries || !out_ids || !out_dists || !out_n)))
        return gfail(WV_EINVAL, "wv_group_search_batch: bad argument");
    if (nq == 0) return WV_OK;
    std::lock_guard<std::mutex> l(g->mu);
    if (g->layout == WV_GROUP_REPLICA || g->m.size() == 1)
        return search_replicas(g, queries, nq, k, ef, allow_bits, allow_nbits, allow_stride_words, mode, out_ids,
                               out_dists, out_n);
    return search_shards(g, queries, nq, k, ef, allow_bits, allow_nbits, allow_stride_words, mode, out_ids, out_dists,
                         out_n);
}

}  // extern "C"
