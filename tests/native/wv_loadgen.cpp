// wv_loadgen.cpp -- measurement infrastructure (libwvload.so, loaded by
// bench.py): T concurrent single-query callers, the way Weaviate calls
// SearchByVector -- once per request, from many goroutines
// (adapters/repos/db/index.go:988-1028 -> shard_read.go:246-252) -- through
// the library's micro-batcher (wv_batcher_search) over an index the caller
// built.  Native threads, so the caller side is not the bottleneck.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <random>
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

// T concurrent SearchByVectorDistance callers (search.go:90-158) through the
// micro-batcher (wv_batcher_search_distance_ids), each query with its own
// target (targets[i]), maxLimit -1, unfiltered.  out[0] QPS, out[1] p50 (us),
// out[2] p99, out[3] mean batch size, out[4] requests, out[5] seconds, out[6]
// mean results per call.
int wvl_concurrent_distance(wv_index* ix, const float* queries, const float* targets, int nq, int dim, int threads,
                            double seconds, int max_batch, double* out) {
    if (!ix || !queries || !targets || nq <= 0 || dim <= 0 || threads <= 0 || seconds <= 0 || !out) return WV_EINVAL;
    wv_batcher* b = nullptr;
    int rc = wv_batcher_create(ix, dim, max_batch, 0, &b);
    if (rc) return rc;
    std::atomic<bool> go{false}, stop{false};
    std::atomic<int> failed{0};
    std::atomic<uint64_t> results{0}, calls{0};
    std::vector<std::vector<float>> lat(threads);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
        ts.emplace_back([&, t] {
            const int64_t cap = 4096;
            std::vector<uint64_t> ids(cap);
            std::vector<float> ds(cap);
            int64_t n = 0;
            lat[t].reserve(1 << 14);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (uint64_t i = 0; !stop.load(std::memory_order_relaxed); ++i) {
                const size_t qi = (size_t)((t + i * threads) % nq);
                const auto a = std::chrono::steady_clock::now();
                if (wv_batcher_search_distance_ids(b, queries + qi * dim, targets[qi], -1, 0, nullptr, 0, ids.data(),
                                                   ds.data(), cap, &n)) {
                    failed = 1;
                    return;
                }
                lat[t].push_back(std::chrono::duration<float, std::micro>(std::chrono::steady_clock::now() - a).count());
                results += (uint64_t)n;
                calls++;
            }
        });
    }
    uint64_t r0 = 0, b0 = 0, r1 = 0, b1 = 0;
    go = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(250));
    wv_batcher_stats(b, &r0, &b0);
    const uint64_t res0 = results.load(), c0 = calls.load();
    const auto t0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    wv_batcher_stats(b, &r1, &b1);
    const uint64_t res1 = results.load(), c1 = calls.load();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    stop = true;
    for (auto& t : ts) t.join();
    wv_batcher_destroy(b);
    if (failed) return WV_EDEVICE;
    std::vector<float> all;
    for (auto& v : lat) all.insert(all.end(), v.begin() + v.size() / 8, v.end());
    if (all.empty()) return WV_ESTATE;
    std::sort(all.begin(), all.end());
    out[0] = (double)(r1 - r0) / el;
    out[1] = all[all.size() / 2];
    out[2] = all[std::min(all.size() - 1, all.size() * 99 / 100)];
    out[3] = b1 > b0 ? (double)(r1 - r0) / (double)(b1 - b0) : 0.0;
    out[4] = (double)(r1 - r0);
    out[5] = el;
    out[6] = c1 > c0 ? (double)(res1 - res0) / (double)(c1 - c0) : 0.0;
    return WV_OK;
}

// Open loop: requests arrive at Poisson times of rate `rate` (seed 7) for
// `seconds`, each issued at its time by one of `pool` threads (a pool larger
// than rate x latency keeps arrivals independent of completions); latency is
// measured from the scheduled arrival, so a request that waits for a free
// thread is charged for it.  out[0] achieved QPS, out[1] p50 (us), out[2] p99,
// out[3] p99.9, out[4] max, out[5] mean batch size, out[6] requests, out[7]
// requests that started > 50 us late (pool saturated).
int wvl_open_loop(wv_index* ix, const float* queries, int nq, int dim, int k, double rate, double seconds,
                  int max_batch, int pool, double* out) {
    if (!ix || !queries || nq <= 0 || dim <= 0 || k <= 0 || rate <= 0 || seconds <= 0 || pool <= 0 || !out)
        return WV_EINVAL;
    wv_batcher* b = nullptr;
    int rc = wv_batcher_create(ix, dim, max_batch, 0, &b);
    if (rc) return rc;
    using clk = std::chrono::steady_clock;
    const size_t n = (size_t)std::max(1.0, std::ceil(rate * seconds));
    std::vector<double> at(n);   // arrival offsets (s)
    std::mt19937_64 rng(7);
    std::exponential_distribution<double> gap(rate);
    double t = 0.0;
    for (size_t i = 0; i < n; ++i) { t += gap(rng); at[i] = t; }
    std::vector<float> lat(n, 0.f);
    std::atomic<size_t> next{0};
    std::atomic<int> failed{0}, late{0};
    uint64_t r0 = 0, b0 = 0, r1 = 0, b1 = 0;
    wv_batcher_stats(b, &r0, &b0);
    const auto t0 = clk::now() + std::chrono::milliseconds(20);
    std::vector<std::thread> ts;
    for (int w = 0; w < pool; ++w) {
        ts.emplace_back([&] {
            std::vector<uint64_t> ids(k);
            std::vector<float> ds(k);
            int32_t cnt = 0;
            for (;;) {
                const size_t i = next.fetch_add(1);
                if (i >= n || failed.load()) return;
                const auto due = t0 + std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(at[i]));
                // sleep to just before the arrival, then spin
                if (due - clk::now() > std::chrono::microseconds(200))
                    std::this_thread::sleep_until(due - std::chrono::microseconds(100));
                while (clk::now() < due) std::this_thread::yield();
                if (clk::now() - due > std::chrono::microseconds(50)) late++;
                const float* q = queries + (i % (size_t)nq) * dim;
                if (wv_batcher_search(b, q, k, nullptr, 0, ids.data(), ds.data(), &cnt)) { failed = 1; return; }
                lat[i] = std::chrono::duration<float, std::micro>(clk::now() - due).count();
            }
        });
    }
    for (auto& th : ts) th.join();
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    wv_batcher_stats(b, &r1, &b1);
    wv_batcher_destroy(b);
    if (failed) return WV_EDEVICE;
    const size_t skip = n / 10;   // (warm-up)
    std::vector<float> all(lat.begin() + skip, lat.end());
    if (all.empty()) return WV_ESTATE;
    std::sort(all.begin(), all.end());
    auto pct = [&](double f) { return (double)all[std::min(all.size() - 1, (size_t)(f * (double)all.size()))]; };
    out[0] = (double)n / el;
    out[1] = pct(0.5);
    out[2] = pct(0.99);
    out[3] = pct(0.999);
    out[4] = (double)all.back();
    out[5] = b1 > b0 ? (double)(r1 - r0) / (double)(b1 - b0) : 0.0;
    out[6] = (double)n;
    out[7] = (double)late.load();
    return WV_OK;
}

}  // extern "C"
