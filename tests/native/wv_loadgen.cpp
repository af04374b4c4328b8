// wv_loadgen.cpp -- measurement infrastructure (libwvload.so, loaded by
// bench.py): T concurrent single-query callers, the way Weaviate calls
// SearchByVector -- once per request, from many goroutines
// (adapters/repos/db/index.go:988-1028 -> shard_read.go:246-252) -- through
// the library's micro-batcher (wv_batcher_search) over an index the caller
// built.  Native threads, so the caller side is not the bottleneck.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/wvgpu.h"

extern "C" {

// out[0] QPS, out[1] p50 latency (us), out[2] p99 (us), out[3] mean batch
// size, out[4] requests, out[5] seconds measured
int wvl_concurrent(wv_index* ix, const float* queries, int nq, int dim, int k, int threads, double seconds,
                   int max_batch, int max_wait_us, double* out) {
    if (!ix || !queries || nq <= 0 || dim <= 0 || k <= 0 || threads <= 0 || seconds <= 0 || !out) return WV_EINVAL;
    wv_batcher* b = nullptr;
    int rc = wv_batcher_create(ix, dim, max_batch, max_wait_us, &b);
    if (rc) return rc;
    std::atomic<bool> go{false}, stop{false};
    std::atomic<int> failed{0};
    std::vector<std::vector<float>> lat(threads);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
        ts.emplace_back([&, t] {
            std::vector<uint64_t> ids(k);
            std::vector<float> ds(k);
            int32_t n = 0;
            lat[t].reserve(1 << 16);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (uint64_t i = 0; !stop.load(std::memory_order_relaxed); ++i) {
                const float* q = queries + (size_t)((t + i * threads) % nq) * dim;
                const auto a = std::chrono::steady_clock::now();
                if (wv_batcher_search(b, q, k, nullptr, 0, ids.data(), ds.data(), &n)) { failed = 1; return; }
                lat[t].push_back(std::chrono::duration<float, std::micro>(std::chrono::steady_clock::now() - a).count());
            }
        });
    }
    uint64_t r0 = 0, b0 = 0;
    // warm-up: a quarter second of traffic, then the measured window
    go = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(250));
    std::vector<size_t> mark(threads);
    for (int t = 0; t < threads; ++t) mark[t] = 0;
    wv_batcher_stats(b, &r0, &b0);
    const auto t0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    uint64_t r1 = 0, b1 = 0;
    wv_batcher_stats(b, &r1, &b1);
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    stop = true;
    for (auto& t : ts) t.join();
    wv_batcher_destroy(b);
    if (failed) return WV_EDEVICE;
    std::vector<float> all;
    for (auto& v : lat) {
        const size_t skip = v.size() / 8;   // (drop each thread's warm-up share)
        all.insert(all.end(), v.begin() + skip, v.end());
    }
    if (all.empty()) return WV_ESTATE;
    std::sort(all.begin(), all.end());
    out[0] = (double)(r1 - r0) / el;
    out[1] = all[all.size() / 2];
    out[2] = all[std::min(all.size() - 1, all.size() * 99 / 100)];
    out[3] = b1 > b0 ? (double)(r1 - r0) / (double)(b1 - b0) : 0.0;
    out[4] = (double)(r1 - r0);
    out[5] = el;
    return WV_OK;
}

}  // extern "C"
