// cpu_index.cpp -- test infrastructure: a CPU stand-in for the wv_index_*
// entry points the host runtime calls (wv_mirror.cpp, wv_batcher.cpp), so
// that those files and wv_commitlog.cpp build under ThreadSanitizer in a
// container without a GPU (the reference runs `go test -race` over all of its
// packages, test/run.sh:101-109).  Exact search over the stored rows with
// tombstones and allow lists; one internal mutex, as the library's index
// serialises its own state.  Never linked into libwvgpu.so.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/wvgpu.h"

namespace {
thread_local std::string g_err;
int fail(int code, const char* m) {
    g_err = m;
    return code;
}
}  // namespace

struct wv_index {
    std::mutex mu;
    int dim = 0, metric = 0;
    wv_config cfg{};
    uint64_t cap = 0, n_rows = 0, graph_n = 0;
    std::vector<float> rows;
    std::vector<uint8_t> has, tomb;
    bool compressed = false;
    float dist(const float* a, const float* b) const {
        float s = 0.f;
        if (metric == WV_L2_SQUARED) {
            for (int j = 0; j < dim; ++j) s += (a[j] - b[j]) * (a[j] - b[j]);
            return s;
        }
        for (int j = 0; j < dim; ++j) s += a[j] * b[j];
        return metric == WV_DOT ? -s : 1.f - s;
    }
    void grow(uint64_t c) {
        if (c <= cap) return;
        rows.resize(c * (size_t)dim, 0.f);
        has.resize(c, 0);
        tomb.resize(c, 0);
        cap = c;
    }
};

extern "C" {

void wv_config_default(wv_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->max_connections = 64;
    c->ef = -1;
    c->dynamic_ef_min = 100;
    c->dynamic_ef_max = 500;
    c->dynamic_ef_factor = 8;
    c->flat_search_cutoff = 40000;
}
const char* wv_last_error(void) { return g_err.c_str(); }
void wv_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }

int wv_index_create(int dim, int metric, const wv_config* cfg, uint64_t capacity, wv_index** out) {
    if (dim <= 0 || !out) return fail(WV_EINVAL, "create");
    auto* x = new wv_index();
    x->dim = dim;
    x->metric = metric;
    if (cfg) x->cfg = *cfg;
    x->grow(std::max<uint64_t>(capacity, 1));
    *out = x;
    return WV_OK;
}
int wv_index_destroy(wv_index* x) {
    delete x;
    return WV_OK;
}
int wv_index_update_config(wv_index* x, const wv_config* c) {
    std::lock_guard<std::mutex> l(x->mu);
    x->cfg = *c;
    return WV_OK;
}
int wv_index_upload_graph(wv_index* x, uint64_t n, const int8_t*, const uint32_t*, int, const uint32_t*,
                          const uint32_t*, uint64_t, int, int, uint64_t) {
    std::lock_guard<std::mutex> l(x->mu);
    x->graph_n = n;
    return WV_OK;
}
int wv_index_build_graph(wv_index* x, int, uint64_t, int) {
    std::lock_guard<std::mutex> l(x->mu);
    x->graph_n = x->n_rows;
    return WV_OK;
}
int wv_index_graph_info(wv_index* x, uint64_t* n, int* deg0, int* degU, int* max_level, uint64_t* n_upper,
                        uint64_t* ep) {
    std::lock_guard<std::mutex> l(x->mu);
    if (n) *n = x->graph_n;
    if (deg0) *deg0 = 2 * x->cfg.max_connections;
    if (degU) *degU = x->cfg.max_connections;
    if (max_level) *max_level = 0;
    if (n_upper) *n_upper = 0;
    if (ep) *ep = 0;
    return WV_OK;
}
int wv_index_set_tombstones(wv_index* x, const uint64_t* bits, uint64_t nbits) {
    std::lock_guard<std::mutex> l(x->mu);
    if (nbits > x->cap) return fail(WV_EINVAL, "set_tombstones: past the capacity");
    std::fill(x->tomb.begin(), x->tomb.end(), 0);
    for (uint64_t i = 0; i < nbits; ++i) x->tomb[i] = (bits[i >> 6] >> (i & 63)) & 1;
    return WV_OK;
}
int wv_index_add(wv_index* x, const uint64_t* ids, const float* rows, uint64_t n) {
    std::lock_guard<std::mutex> l(x->mu);
    for (uint64_t i = 0; i < n; ++i) {
        if (ids[i] >= x->cap) return fail(WV_EINVAL, "add: id past the capacity");
        std::memcpy(&x->rows[ids[i] * x->dim], rows + i * x->dim, sizeof(float) * x->dim);
        x->has[ids[i]] = 1;
        x->n_rows = std::max(x->n_rows, ids[i] + 1);
    }
    return WV_OK;
}
int wv_index_add_tombstones(wv_index* x, const uint64_t* ids, uint64_t n) {
    std::lock_guard<std::mutex> l(x->mu);
    for (uint64_t i = 0; i < n; ++i)
        if (ids[i] < x->cap) x->tomb[ids[i]] = 1;
    return WV_OK;
}
int wv_index_reserve(wv_index* x, uint64_t capacity) {
    std::lock_guard<std::mutex> l(x->mu);
    x->grow(capacity);
    return WV_OK;
}
int wv_index_capacity(const wv_index* x, uint64_t* capacity, uint64_t* n_rows) {
    auto* m = const_cast<wv_index*>(x);
    std::lock_guard<std::mutex> l(m->mu);
    if (capacity) *capacity = x->cap;
    if (n_rows) *n_rows = x->n_rows;
    return WV_OK;
}
int wv_index_set_pq(wv_index* x, int, int, int, int, const float*) { return x ? WV_OK : WV_EINVAL; }
int wv_index_pq_encode(wv_index* x) { return x ? WV_OK : WV_EINVAL; }
int wv_index_set_compressed(wv_index* x, int on) {
    std::lock_guard<std::mutex> l(x->mu);
    x->compressed = on;
    return WV_OK;
}

int wv_search_batch(wv_index* x, const float* qs, int nq, int k, int, const uint64_t* allow, uint64_t nbits,
                    uint64_t stride, int, uint64_t* out_ids, float* out_d, int32_t* out_n) {
    std::lock_guard<std::mutex> l(x->mu);
    std::vector<std::pair<float, uint64_t>> c;
    for (int q = 0; q < nq; ++q) {
        c.clear();
        const uint64_t* a = allow ? allow + (size_t)q * stride : nullptr;
        for (uint64_t i = 0; i < x->n_rows; ++i) {
            if (!x->has[i] || x->tomb[i]) continue;
            if (a && (i >= nbits || !((a[i >> 6] >> (i & 63)) & 1))) continue;
            c.emplace_back(x->dist(qs + (size_t)q * x->dim, &x->rows[i * x->dim]), i);
        }
        const size_t kk = std::min<size_t>(k, c.size());
        std::partial_sort(c.begin(), c.begin() + kk, c.end());
        for (size_t j = 0; j < kk; ++j) {
            out_ids[(size_t)q * k + j] = c[j].second + x->cfg.id_base;
            out_d[(size_t)q * k + j] = c[j].first;
        }
        out_n[q] = (int32_t)kk;
    }
    return WV_OK;
}
int wv_search_by_vector_distance(wv_index* x, const float* v, float target, int64_t max_limit, const uint64_t* allow,
                                 uint64_t nbits, uint64_t* out_ids, float* out_d, int64_t out_cap, int64_t* out_n) {
    std::lock_guard<std::mutex> l(x->mu);
    std::vector<std::pair<float, uint64_t>> c;
    for (uint64_t i = 0; i < x->n_rows; ++i) {
        if (!x->has[i] || x->tomb[i]) continue;
        if (allow && (i >= nbits || !((allow[i >> 6] >> (i & 63)) & 1))) continue;
        const float d = x->dist(v, &x->rows[i * x->dim]);
        if (d <= target) c.emplace_back(d, i);
    }
    std::sort(c.begin(), c.end());
    if (max_limit >= 0 && (int64_t)c.size() > max_limit) c.resize(max_limit);
    for (int64_t j = 0; j < (int64_t)c.size() && j < out_cap; ++j) {
        out_ids[j] = c[j].second;
        out_d[j] = c[j].first;
    }
    *out_n = (int64_t)c.size();
    return WV_OK;
}
int wv_search_by_vector_distance_batch(wv_index* x, const float* qs, int nq, const float* targets, int64_t max_limit,
                                       const uint64_t* allow, uint64_t nbits, uint64_t stride, uint64_t* out_ids,
                                       float* out_d, int64_t out_cap, int64_t* out_n) {
    for (int q = 0; q < nq; ++q) {
        const uint64_t* a = allow ? allow + (stride ? (size_t)q * stride : 0) : nullptr;
        const int rc = wv_search_by_vector_distance(x, qs + (size_t)q * x->dim, targets[q], max_limit, a, nbits,
                                                    out_ids + (size_t)q * out_cap, out_d + (size_t)q * out_cap,
                                                    out_cap, out_n + q);
        if (rc) return rc;
    }
    return WV_OK;
}
int wv_group_search_batch(wv_group*, const float*, int, int, int, const uint64_t*, uint64_t, uint64_t, int, uint64_t*,
                          float*, int32_t*) {
    return fail(WV_EINVAL, "no groups in the TSAN stand-in");
}
int wv_group_search_by_vector_distance_batch(wv_group*, const float*, int, const float*, int64_t, const uint64_t*,
                                             uint64_t, uint64_t, uint64_t*, float*, int64_t, int64_t*) {
    return fail(WV_EINVAL, "no groups in the TSAN stand-in");
}

}  // extern "C"
