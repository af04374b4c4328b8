/*
 * wv_oracle.c -- CPU restatement of Weaviate's HNSW / flat vector search.
 *
 * TEST INFRASTRUCTURE ONLY (see wv_oracle.h): the parity checker and the CPU
 * baseline.  Never linked into, or called by, the product path.
 *
 * Reference paths below are relative to
 * /root/reference/adapters/repos/db/vector/hnsw/ unless stated otherwise.
 * Compiled with -ffp-contract=off so every float operation is rounded as the
 * Go code / assembly rounds it (fmaf only where the assembly uses VFMADD).
 */
#define _GNU_SOURCE
#include "wv_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define NIL_ID 0xFFFFFFFFu

/* ======================================================================== */
/* Distancers                                                               */
/* ======================================================================== */

/* asm.L2 -- distancer/asm/l2_amd64.s:7-64.
 * Four 8-lane accumulators over 32-float blocks (:20-38), a scalar FMA tail
 * (:40-52), then the reduction tree (:54-64):
 *   s = (acc0+acc1)+(acc2+acc3); v[l] = s[l]+s[l+4]; v += [t,0,0,0];
 *   r = (v0+v1)+(v2+v3)   (two VHADDPS). */
float wvo_asm_l2(const float *x, const float *y, int n) {
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    int i = 0;
    for (; n - i >= 32; i += 32) {
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++) {
                float d = x[i + 8 * j + l] - y[i + 8 * j + l]; /* VSUBPS */
                acc[j][l] = fmaf(d, d, acc[j][l]);              /* VFMADD231PS */
            }
    }
    float t = 0.0f;
    for (; i < n; i++) {
        float d = x[i] - y[i];
        t = fmaf(d, d, t); /* VFMADD231SS */
    }
    float s[8], v[4];
    for (int l = 0; l < 8; l++) s[l] = (acc[0][l] + acc[1][l]) + (acc[2][l] + acc[3][l]);
    for (int l = 0; l < 4; l++) v[l] = s[l] + s[l + 4];
    v[0] = t + v[0];
    v[1] = 0.0f + v[1];
    v[2] = 0.0f + v[2];
    v[3] = 0.0f + v[3];
    return (v[0] + v[1]) + (v[2] + v[3]);
}

/* asm.Dot -- distancer/asm/dot_amd64.s:7-55: identical structure with
 * acc = fma(x, y, acc) (:16-30) and tail t = fma(x, y, t) (:36-43). */
float wvo_asm_dot(const float *x, const float *y, int n) {
    float acc[4][8];
    memset(acc, 0, sizeof(acc));
    int i = 0;
    for (; n - i >= 32; i += 32) {
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < 8; l++)
                acc[j][l] = fmaf(x[i + 8 * j + l], y[i + 8 * j + l], acc[j][l]);
    }
    float t = 0.0f;
    for (; i < n; i++) t = fmaf(x[i], y[i], t);
    float s[8], v[4];
    for (int l = 0; l < 8; l++) s[l] = (acc[0][l] + acc[1][l]) + (acc[2][l] + acc[3][l]);
    for (int l = 0; l < 4; l++) v[l] = s[l] + s[l + 4];
    v[0] = t + v[0];
    v[1] = 0.0f + v[1];
    v[2] = 0.0f + v[2];
    v[3] = 0.0f + v[3];
    return (v[0] + v[1]) + (v[2] + v[3]);
}

#if defined(__x86_64__)
/* Instruction-by-instruction mirror of l2_amd64.s / dot_amd64.s.  Used as the
 * fast distance on AVX2+FMA hosts and to cross-check the scalar emulation. */
__attribute__((target("avx2,fma"))) static float avx2_l2(const float *x, const float *y, int n) {
    __m256 y0 = _mm256_setzero_ps(), y2 = _mm256_setzero_ps();
    __m256 y4 = _mm256_setzero_ps(), y6 = _mm256_setzero_ps();
    while (n >= 32) {
        __m256 y1 = _mm256_loadu_ps(x), y3 = _mm256_loadu_ps(x + 8);
        __m256 y5 = _mm256_loadu_ps(x + 16), y7 = _mm256_loadu_ps(x + 24);
        y1 = _mm256_sub_ps(y1, _mm256_loadu_ps(y));
        y3 = _mm256_sub_ps(y3, _mm256_loadu_ps(y + 8));
        y5 = _mm256_sub_ps(y5, _mm256_loadu_ps(y + 16));
        y7 = _mm256_sub_ps(y7, _mm256_loadu_ps(y + 24));
        y0 = _mm256_fmadd_ps(y1, y1, y0);
        y2 = _mm256_fmadd_ps(y3, y3, y2);
        y4 = _mm256_fmadd_ps(y5, y5, y4);
        y6 = _mm256_fmadd_ps(y7, y7, y6);
        x += 32; y += 32; n -= 32;
    }
    __m128 x1 = _mm_setzero_ps();
    while (n > 0) {
        __m128 x3 = _mm_sub_ss(_mm_load_ss(x), _mm_load_ss(y));
        x1 = _mm_fmadd_ss(x3, x3, x1);
        x++; y++; n--;
    }
    y0 = _mm256_add_ps(y2, y0);
    y4 = _mm256_add_ps(y6, y4);
    y0 = _mm256_add_ps(y4, y0);
    __m128 x2 = _mm256_extractf128_ps(y0, 1);
    __m128 x0 = _mm_add_ps(x2, _mm256_castps256_ps128(y0));
    x0 = _mm_add_ps(x1, x0);
    x0 = _mm_hadd_ps(x0, x0);
    x0 = _mm_hadd_ps(x0, x0);
    return _mm_cvtss_f32(x0);
}

__attribute__((target("avx2,fma"))) static float avx2_dot(const float *x, const float *y, int n) {
    __m256 y0 = _mm256_setzero_ps(), y1 = _mm256_setzero_ps();
    __m256 y2 = _mm256_setzero_ps(), y3 = _mm256_setzero_ps();
    while (n >= 32) {
        y0 = _mm256_fmadd_ps(_mm256_loadu_ps(x), _mm256_loadu_ps(y), y0);
        y1 = _mm256_fmadd_ps(_mm256_loadu_ps(x + 8), _mm256_loadu_ps(y + 8), y1);
        y2 = _mm256_fmadd_ps(_mm256_loadu_ps(x + 16), _mm256_loadu_ps(y + 16), y2);
        y3 = _mm256_fmadd_ps(_mm256_loadu_ps(x + 24), _mm256_loadu_ps(y + 24), y3);
        x += 32; y += 32; n -= 32;
    }
    __m128 x4 = _mm_setzero_ps();
    while (n > 0) {
        x4 = _mm_fmadd_ss(_mm_load_ss(x), _mm_load_ss(y), x4);
        x++; y++; n--;
    }
    y0 = _mm256_add_ps(y1, y0);
    y2 = _mm256_add_ps(y3, y2);
    y0 = _mm256_add_ps(y2, y0);
    __m128 x1 = _mm256_extractf128_ps(y0, 1);
    __m128 x0 = _mm_add_ps(x1, _mm256_castps256_ps128(y0));
    x0 = _mm_add_ps(x4, x0);
    x0 = _mm_hadd_ps(x0, x0);
    x0 = _mm_hadd_ps(x0, x0);
    return _mm_cvtss_f32(x0);
}
#endif

static int g_have_avx2 = -1;
static int have_avx2(void) {
    if (g_have_avx2 < 0) {
#if defined(__x86_64__)
        __builtin_cpu_init();
        g_have_avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
#else
        g_have_avx2 = 0;
#endif
    }
    return g_have_avx2;
}

static inline float raw_l2(const float *a, const float *b, int n) {
#if defined(__x86_64__)
    if (g_have_avx2 > 0) return avx2_l2(a, b, n);
#endif
    return wvo_asm_l2(a, b, n);
}
static inline float raw_dot(const float *a, const float *b, int n) {
#if defined(__x86_64__)
    if (g_have_avx2 > 0) return avx2_dot(a, b, n);
#endif
    return wvo_asm_dot(a, b, n);
}

/* L2Squared (l2.go:33-41), DotProduct distance = -dot (dot_product.go:36-44),
 * CosineDistance = 1 - dot over normalized vectors (cosine_dist.go:22-30). */
static inline float metric_dist(int metric, const float *a, const float *b, int n) {
    switch (metric) {
    case WVO_L2: return raw_l2(a, b, n);
    case WVO_DOT: return -raw_dot(a, b, n);
    default: return 1.0f - raw_dot(a, b, n);
    }
}

float wvo_distance(int metric, const float *a, const float *b, int n) {
    switch (metric) {
    case WVO_L2: return wvo_asm_l2(a, b, n);
    case WVO_DOT: return -wvo_asm_dot(a, b, n);
    default: return 1.0f - wvo_asm_dot(a, b, n);
    }
}

float wvo_distance_avx2(int metric, const float *a, const float *b, int n) {
#if defined(__x86_64__)
    if (have_avx2()) {
        switch (metric) {
        case WVO_L2: return avx2_l2(a, b, n);
        case WVO_DOT: return -avx2_dot(a, b, n);
        default: return 1.0f - avx2_dot(a, b, n);
        }
    }
#endif
    return wvo_distance(metric, a, b, n);
}

/* l2.go:16-25 and dot_product.go:23-31: sequential, not FMA-fused (Go 1.19,
 * GOAMD64=v1 does not fuse). */
float wvo_distance_purego(int metric, const float *a, const float *b, int n) {
    float sum = 0.0f;
    if (metric == WVO_L2) {
        for (int i = 0; i < n; i++) {
            float d = a[i] - b[i];
            float sq = d * d;
            sum = sum + sq;
        }
        return sum;
    }
    for (int i = 0; i < n; i++) {
        float p = a[i] * b[i];
        sum = sum + p;
    }
    return metric == WVO_DOT ? -sum : 1.0f - sum;
}

/* distancer/normalize.go:16-32 */
void wvo_normalize(const float *in, float *out, int n) {
    float norm = 0.0f;
    for (int i = 0; i < n; i++) {
        float p = in[i] * in[i];
        norm = norm + p;
    }
    if (norm == 0.0f) {
        for (int i = 0; i < n; i++) out[i] = 0.0f;
        return;
    }
    norm = (float)sqrt((double)norm);
    for (int i = 0; i < n; i++) out[i] = in[i] / norm;
}

void wvo_normalize_rows(const float *in, float *out, uint64_t rows, int dim) {
    for (uint64_t r = 0; r < rows; r++) wvo_normalize(in + r * (uint64_t)dim, out + r * (uint64_t)dim, dim);
}

/* ======================================================================== */
/* priorityqueue.Queue clone -- priorityqueue/queue.go:14-111               */
/* ======================================================================== */
typedef struct { uint64_t id; float dist; } pq_item;
typedef struct { pq_item *it; size_t len, cap; int is_max; } pq_t;

static void pq_init(pq_t *q, int is_max, size_t cap) {
    q->is_max = is_max;
    q->len = 0;
    q->cap = cap < 4 ? 4 : cap;
    q->it = (pq_item *)malloc(q->cap * sizeof(pq_item));
}
static void pq_free(pq_t *q) { free(q->it); q->it = NULL; q->len = q->cap = 0; }
static inline int pq_less(const pq_t *q, size_t i, size_t j) {
    return q->is_max ? (q->it[i].dist > q->it[j].dist) : (q->it[i].dist < q->it[j].dist);
}
static inline void pq_swap(pq_t *q, size_t i, size_t j) {
    pq_item t = q->it[i]; q->it[i] = q->it[j]; q->it[j] = t;
}
/* heapify (queue.go:58-74), recursion unrolled into a loop with the same swaps */
static void pq_heapify(pq_t *q, size_t i) {
    for (;;) {
        size_t left = 2 * i + 1, right = 2 * i + 2, smallest = i;
        if (left < q->len && pq_less(q, left, i)) smallest = left;
        if (right < q->len && pq_less(q, right, smallest)) smallest = right;
        if (smallest == i) return;
        pq_swap(q, i, smallest);
        i = smallest;
    }
}
/* Insert (queue.go:76-83) */
static void pq_insert(pq_t *q, uint64_t id, float dist) {
    if (q->len == q->cap) {
        q->cap *= 2;
        q->it = (pq_item *)realloc(q->it, q->cap * sizeof(pq_item));
    }
    q->it[q->len] = (pq_item){id, dist};
    size_t i = q->len++;
    while (i != 0 && pq_less(q, i, (i - 1) / 2)) {
        pq_swap(q, i, (i - 1) / 2);
        i = (i - 1) / 2;
    }
}
/* Pop (queue.go:85-91) */
static pq_item pq_pop(pq_t *q) {
    pq_item out = q->it[0];
    q->it[0] = q->it[q->len - 1];
    q->len--;
    pq_heapify(q, 0);
    return out;
}

int wvo_pq_script(int is_max, int nops, const int *op, const uint64_t *ids,
                  const float *dists, uint64_t *out_ids, float *out_d) {
    pq_t q;
    pq_init(&q, is_max, 8);
    int n = 0;
    for (int i = 0; i < nops; i++) {
        if (op[i] == 0) pq_insert(&q, ids[i], dists[i]);
        else if (q.len > 0) {
            pq_item it = pq_pop(&q);
            out_ids[n] = it.id;
            out_d[n] = it.dist;
            n++;
        }
    }
    pq_free(&q);
    return n;
}

/* QueueWithIndex (priorityqueue/queue_with_index.go:14-111), min variant */
typedef struct { uint64_t id, index; float dist; } pqi_item;
typedef struct { pqi_item *it; size_t len, cap; } pqi_t;
static void pqi_insert(pqi_t *q, uint64_t id, uint64_t index, float dist) {
    if (q->len == q->cap) {
        q->cap = q->cap ? q->cap * 2 : 16;
        q->it = (pqi_item *)realloc(q->it, q->cap * sizeof(pqi_item));
    }
    q->it[q->len] = (pqi_item){id, index, dist};
    size_t i = q->len++;
    while (i != 0 && q->it[i].dist < q->it[(i - 1) / 2].dist) {
        pqi_item t = q->it[i]; q->it[i] = q->it[(i - 1) / 2]; q->it[(i - 1) / 2] = t;
        i = (i - 1) / 2;
    }
}
static pqi_item pqi_pop(pqi_t *q) {
    pqi_item out = q->it[0];
    q->it[0] = q->it[q->len - 1];
    q->len--;
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = 2 * i + 2, s = i;
        if (l < q->len && q->it[l].dist < q->it[i].dist) s = l;
        if (r < q->len && q->it[r].dist < q->it[s].dist) s = r;
        if (s == i) break;
        pqi_item t = q->it[i]; q->it[i] = q->it[s]; q->it[s] = t;
        i = s;
    }
    return out;
}

/* ======================================================================== */
/* searchTimeEF / autoEfFromK -- search.go:30-62                            */
/* ======================================================================== */
int wvo_search_time_ef(int64_t ef64, int64_t ef_min, int64_t ef_max,
                       int64_t ef_factor, int k) {
    int ef = (int)ef64;
    if (ef < 1) {
        int factor = (int)ef_factor, mn = (int)ef_min, mx = (int)ef_max;
        ef = k * factor;
        if (ef > mx) ef = mx;
        else if (ef < mn) ef = mn;
        if (k > ef) ef = k;
        return ef;
    }
    if (ef < k) ef = k;
    return ef;
}

/* ======================================================================== */
/* Product quantization -- ssdhelpers/product_quantization.go, kmeans.go    */
/* (paths relative to adapters/repos/db/vector/)                            */
/* ======================================================================== */

/* NewProductQuantizer (product_quantization.go:116-179): bits = int(log2(ks)),
 * bytes = int(log2(ks-1))/8 + 1, and the code accessor pair by (bytes, bits,
 * useBitsEncoding).  kind: 8/16/24/32 = plain big-endian accessor of that
 * width; 0 = extractBitsCode / putBitsCode over the `inner` accessor. */
typedef struct { int bits, bytes, kind, inner, sharp; uint64_t mask; } pq_layout;

static int pq_layout_of(int ks, int use_bits, pq_layout *L) {
    if (ks < 2 || ks > (1 << 24)) return -1;
    L->bits = (int)log2((double)ks);
    L->bytes = (int)log2((double)(ks - 1)) / 8 + 1;
    L->sharp = L->bits % 8 == 0;
    L->mask = (L->bits >= 64) ? ~0ull : ((1ull << L->bits) - 1);   /* uint64(2^bits) - 1 */
    switch (L->bytes) {
    case 1: if (L->bits == 8 || !use_bits) { L->kind = 8; } else { L->kind = 0; L->inner = 16; } break;
    case 2: if (L->bits == 16 || !use_bits) { L->kind = 16; } else { L->kind = 0; L->inner = 24; } break;
    case 3: if (L->bits == 32 || !use_bits) { L->kind = 24; } else { L->kind = 0; L->inner = 32; } break;
    default: return -1;
    }
    return 0;
}

/* extractCode8/16/24/32 (:191-205), big endian */
static uint64_t pq_get(int width, const uint8_t *p) {
    switch (width) {
    case 8: return p[0];
    case 16: return ((uint64_t)p[0] << 8) | p[1];
    case 24: return (((uint64_t)p[0] << 24) | ((uint64_t)p[1] << 16) | ((uint64_t)p[2] << 8) | p[3]) >> 8;
    default: return ((uint64_t)p[0] << 24) | ((uint64_t)p[1] << 16) | ((uint64_t)p[2] << 8) | p[3];
    }
}

/* putCode8/16/24/32 (:207-221) */
static void pq_set(int width, uint64_t code, uint8_t *p) {
    switch (width) {
    case 8: p[0] = (uint8_t)code; break;
    case 16: p[0] = (uint8_t)(code >> 8); p[1] = (uint8_t)code; break;
    case 24: {
        uint32_t v = (uint32_t)(code << 8);
        p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
        break;
    }
    default: {
        uint32_t v = (uint32_t)code;
        p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
    }
    }
}

/* ProductQuantizer.ExtractCode: plain accessor or extractBitsCode (:223-237) */
static uint64_t pq_extract(const pq_layout *L, const uint8_t *enc, int index) {
    if (L->kind) return pq_get(L->kind, enc + (size_t)index * (L->kind / 8));
    const int ci = index * L->bits / 8;
    uint64_t code = pq_get(L->inner, enc + ci);
    if (L->sharp) return code;
    const int rest = (index + 1) * L->bits % 8;
    const int rfs = index * L->bits % 8;
    if (rfs < rest) code >>= 16 - rest;
    else code >>= 8 - rest;
    return code & L->mask;
}

/* ProductQuantizer.PutCode: plain accessor, putBitsCode (:239-258), or --
 * for 3-byte codes with bit encoding -- the plain putCode32 (:174) */
static void pq_put(const pq_layout *L, uint64_t code, uint8_t *enc, int index) {
    if (L->kind) { pq_set(L->kind, code, enc + (size_t)index * (L->kind / 8)); return; }
    if (L->inner == 32) { pq_set(32, code, enc + (size_t)index * 4); return; }
    const int ci = index * L->bits / 8;
    if (L->sharp) { pq_set(L->inner, code, enc + ci); return; }
    const int rest = (index + 1) * L->bits % 8;
    const int rfs = index * L->bits % 8;
    if (rfs < rest) code <<= 16 - rest;
    else code <<= 8 - rest;
    code |= (uint64_t)enc[ci] << (L->bytes * 8);
    pq_set(L->inner, code, enc + ci);
}

int wvo_pq_layout(int ks, int use_bits, int *bits, int *bytes) {
    pq_layout L;
    if (pq_layout_of(ks, use_bits, &L)) return -1;
    *bits = L.bits;
    *bytes = L.bytes;
    return 0;
}

int wvo_pq_extract(const uint8_t *enc, int n_codes, int ks, int use_bits, uint64_t *out) {
    pq_layout L;
    if (pq_layout_of(ks, use_bits, &L)) return -1;
    for (int i = 0; i < n_codes; i++) out[i] = pq_extract(&L, enc, i);
    return 0;
}

int wvo_pq_put(const uint64_t *codes, int n_codes, int ks, int use_bits, uint8_t *enc) {
    pq_layout L;
    if (pq_layout_of(ks, use_bits, &L)) return -1;
    for (int i = 0; i < n_codes; i++) pq_put(&L, codes[i], enc, i);
    return 0;
}

/* L2SquaredProvider.Step / DotProductProvider.Step / CosineDistanceProvider.Step
 * (distancer/l2.go:63-72, dot_product.go:80-87, cosine_dist.go:57-64): pure Go,
 * sequential, not fused. */
static float pq_step(int metric, const float *x, const float *y, int n) {
    float sum = 0.0f;
    if (metric == WVO_L2) {
        for (int i = 0; i < n; i++) {
            float d = x[i] - y[i];
            float sq = d * d;
            sum = sum + sq;
        }
    } else {
        for (int i = 0; i < n; i++) {
            float p = x[i] * y[i];
            sum = sum + p;
        }
    }
    return sum;
}

/* Wrap (l2.go:74-76, dot_product.go:89-91, cosine_dist.go:66-68) */
static float pq_wrap(int metric, float x) {
    return metric == WVO_L2 ? x : metric == WVO_DOT ? -x : 1.0f - x;
}

/* DistanceBetweenCompressedAndUncompressedVectors (:284-291); the lookup
 * table (:56-75) caches exactly these Step values and sums them in the same
 * segment order, so PQDistancer.Distance returns the same float. */
static float pq_distance(int metric, const pq_layout *L, const float *x, const uint8_t *enc,
                         const float *cent, int m, int ks, int ds) {
    float dist = 0.0f;
    for (int i = 0; i < m; i++) {
        const uint64_t c = pq_extract(L, enc, i);
        dist = dist + pq_step(metric, x + (size_t)i * ds, cent + ((size_t)i * ks + c) * ds, ds);
    }
    return pq_wrap(metric, dist);
}

float wvo_pq_distance(int metric, const float *x, const uint8_t *enc, const float *cent, int m, int ks, int dim,
                      int use_bits) {
    pq_layout L;
    if (pq_layout_of(ks, use_bits, &L) || m <= 0 || dim % m) return NAN;
    return pq_distance(metric, &L, x, enc, cent, m, ks, dim / m);
}

/* KMeans.Nearest / nNearest with n = 1 (kmeans.go:78-110): asm.L2 over the
 * segment; a candidate replaces the best when best >= d, so among equal
 * distances the last centroid wins. */
static uint64_t kmeans_nearest(const float *seg, const float *centers, int ks, int ds) {
    uint64_t best = 0;
    float bd = FLT_MAX;
    for (int c = 0; c < ks; c++) {
        const float d = raw_l2(seg, centers + (size_t)c * ds, ds);
        if (!(bd < d)) { bd = d; best = (uint64_t)c; }
    }
    return best;
}

/* ProductQuantizer.Encode (:348-354) with KMeans encoders: enc[n][m*bytes] */
int wvo_pq_encode_kmeans(const float *vecs, uint64_t n, int dim, int m, int ks, const float *cent, int use_bits,
                         uint8_t *enc) {
    pq_layout L;
    if (pq_layout_of(ks, use_bits, &L) || m <= 0 || dim % m) return -1;
    have_avx2();
    const int ds = dim / m;
    const size_t len = (size_t)m * L.bytes;
    uint8_t *tmp = (uint8_t *)calloc(len + 8, 1);
    for (uint64_t r = 0; r < n; r++) {
        memset(tmp, 0, len + 8);
        for (int i = 0; i < m; i++)
            pq_put(&L, kmeans_nearest(vecs + r * (uint64_t)dim + (size_t)i * ds, cent + (size_t)i * ks * ds, ks, ds),
                   tmp, i);
        memcpy(enc + r * len, tmp, len);
    }
    free(tmp);
    return 0;
}

/* ======================================================================== */
/* Index                                                                    */
/* ======================================================================== */
typedef struct { uint32_t len, cap; uint32_t *ids; } conn_list;

struct wvo_index {
    int dim, metric, M, M0, efC;
    uint64_t cap;
    uint64_t seed;
    double level_normalizer;
    float *vecs;
    uint8_t *has_vec;
    int8_t *level;       /* -1: nil node (index.go:91 nodes[id] == nil) */
    uint8_t *maint;      /* vertex.maintenance (vertex.go:18-45) */
    conn_list **conns;   /* conns[id][level] */
    uint8_t *tomb;       /* tombstones map (delete.go:546-566) */
    pthread_mutex_t *node_lock;
    pthread_rwlock_t glock;  /* h.RWMutex guarding entrypoint / max layer */
    pthread_mutex_t init_lock;
    int threaded;
    uint64_t ep;
    int max_layer;
    atomic_uint_fast64_t n_nodes;
    int initial_done;
    int next_level; /* test hook, -1 = draw */
    /* search config (index.go:79-87) */
    int64_t ef, ef_min, ef_max, ef_factor, flat_cutoff;
    int forbid_flat;
    /* commit log (commitlog/logger.go), written where the reference writes it */
    int log_on;
    uint8_t *log;
    size_t log_len, log_cap;
    pthread_mutex_t log_lock;
    /* product quantization: h.compressed / h.pq / compressedVectorsCache
     * (compress.go:39-89); codes kept in the reference's encoded layout */
    int compressed;
    int pq_m, pq_ks, pq_ds, pq_use_bits;
    uint64_t pq_code_len;
    float *pq_cent;      /* [m][ks][ds] = kms[i].Centroid(c) */
    uint8_t *pq_codes;   /* [cap][code_len] */
    uint8_t *pq_has;     /* [cap] */
};

/* ---- commit log records -- commitlog/logger.go:28-215 (little endian) ---- */
enum { CL_ADD_NODE = 0, CL_SET_EP = 1, CL_ADD_LINK = 2, CL_REPLACE_LINKS = 3, CL_ADD_TOMB = 4,
       CL_REMOVE_TOMB = 5, CL_CLEAR_LINKS = 6, CL_DELETE_NODE = 7, CL_RESET = 8, CL_CLEAR_LINKS_AT_LEVEL = 9,
       CL_ADD_LINKS = 10 };

static void log_bytes(wvo_index *h, const uint8_t *b, size_t n) {
    if (h->log_len + n > h->log_cap) {
        size_t c = h->log_cap ? h->log_cap * 2 : 1 << 16;
        while (c < h->log_len + n) c *= 2;
        h->log = (uint8_t *)realloc(h->log, c);
        h->log_cap = c;
    }
    memcpy(h->log + h->log_len, b, n);
    h->log_len += n;
}
static void put64(uint8_t *p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }
static void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

/* AddNode / SetEntryPointWithMaxLayer / AddLinkAtLevel / AddTombstone /
 * ClearLinksAtLevel (logger.go:59-75,98-106,170-176,194-201) */
static void log_id_level(wvo_index *h, int type, uint64_t id, int level) {
    if (!h->log_on) return;
    uint8_t b[11];
    b[0] = (uint8_t)type;
    put64(b + 1, id);
    put16(b + 9, (uint16_t)level);
    pthread_mutex_lock(&h->log_lock);
    log_bytes(h, b, 11);
    pthread_mutex_unlock(&h->log_lock);
}
static void log_add_link(wvo_index *h, uint64_t id, int level, uint64_t target) {
    if (!h->log_on) return;
    uint8_t b[19];
    b[0] = CL_ADD_LINK;
    put64(b + 1, id);
    put16(b + 9, (uint16_t)level);
    put64(b + 11, target);
    pthread_mutex_lock(&h->log_lock);
    log_bytes(h, b, 19);
    pthread_mutex_unlock(&h->log_lock);
}
/* ReplaceLinksAtLevel (logger.go:125-168): 13-byte header + 8 bytes per target */
static void log_replace_links(wvo_index *h, uint64_t id, int level, const uint32_t *t, uint32_t n) {
    if (!h->log_on) return;
    uint8_t hd[13];
    hd[0] = CL_REPLACE_LINKS;
    put64(hd + 1, id);
    put16(hd + 9, (uint16_t)level);
    put16(hd + 11, (uint16_t)n);
    pthread_mutex_lock(&h->log_lock);
    log_bytes(h, hd, 13);
    for (uint32_t i = 0; i < n; i++) {
        uint8_t v[8];
        put64(v, t[i]);
        log_bytes(h, v, 8);
    }
    pthread_mutex_unlock(&h->log_lock);
}
static void log_id(wvo_index *h, int type, uint64_t id) {
    if (!h->log_on) return;
    uint8_t b[9];
    b[0] = (uint8_t)type;
    put64(b + 1, id);
    pthread_mutex_lock(&h->log_lock);
    log_bytes(h, b, 9);
    pthread_mutex_unlock(&h->log_lock);
}

void wvo_log_enable(wvo_index *h, int on) { h->log_on = on; }
uint64_t wvo_log_size(wvo_index *h) { return h->log_len; }
uint64_t wvo_log_copy(wvo_index *h, uint8_t *out, uint64_t cap) {
    uint64_t n = h->log_len < cap ? h->log_len : cap;
    if (n) memcpy(out, h->log, n);
    return n;
}

/* per-thread search context: the visited.ListSet (visited/list_set.go:23-64)
 * restated as an epoch array; a fresh epoch == a freshly borrowed list. */
typedef struct {
    uint32_t *vis;
    uint64_t vis_n;
    uint32_t epoch;
    uint64_t vis_count;
    pq_t cand;
    uint32_t *nbuf;
    size_t nbuf_cap;
    wvo_stats st;
} ctx_t;

static void ctx_init(ctx_t *c, uint64_t n) {
    memset(c, 0, sizeof(*c));
    c->vis_n = n + 1;
    c->vis = (uint32_t *)calloc(c->vis_n, sizeof(uint32_t));
    c->epoch = 0;
    pq_init(&c->cand, 0, 256);
    c->nbuf_cap = 256;
    c->nbuf = (uint32_t *)malloc(c->nbuf_cap * sizeof(uint32_t));
}
static void ctx_free(ctx_t *c) {
    free(c->vis);
    pq_free(&c->cand);
    free(c->nbuf);
}
static void ctx_reset_visited(ctx_t *c) {
    c->epoch++;
    c->vis_count = 0;
    if (c->epoch == 0) {
        memset(c->vis, 0, c->vis_n * sizeof(uint32_t));
        c->epoch = 1;
    }
}
static inline int ctx_visited(ctx_t *c, uint64_t id) { return id < c->vis_n && c->vis[id] == c->epoch; }
static inline void ctx_visit(ctx_t *c, uint64_t id) {
    if (id < c->vis_n) { c->vis[id] = c->epoch; c->vis_count++; }
}

static inline int allow_contains(const uint64_t *bits, uint64_t nbits, uint64_t id) {
    return id < nbits && ((bits[id >> 6] >> (id & 63)) & 1u);
}

wvo_index *wvo_create(int dim, int metric, int max_connections,
                      int ef_construction, uint64_t capacity, uint64_t seed) {
    have_avx2();
    wvo_index *h = (wvo_index *)calloc(1, sizeof(wvo_index));
    h->dim = dim;
    h->metric = metric;
    h->M = max_connections;
    h->M0 = 2 * max_connections; /* index.go:223 */
    h->efC = ef_construction;
    h->cap = capacity;
    h->seed = seed;
    h->level_normalizer = 1.0 / log((double)max_connections); /* index.go:226 */
    h->vecs = (float *)calloc(capacity * (uint64_t)dim, sizeof(float));
    h->has_vec = (uint8_t *)calloc(capacity, 1);
    h->level = (int8_t *)malloc(capacity);
    memset(h->level, -1, capacity);
    h->maint = (uint8_t *)calloc(capacity, 1);
    h->conns = (conn_list **)calloc(capacity, sizeof(conn_list *));
    h->tomb = (uint8_t *)calloc(capacity, 1);
    h->node_lock = (pthread_mutex_t *)malloc(capacity * sizeof(pthread_mutex_t));
    for (uint64_t i = 0; i < capacity; i++) pthread_mutex_init(&h->node_lock[i], NULL);
    pthread_rwlock_init(&h->glock, NULL);
    pthread_mutex_init(&h->init_lock, NULL);
    pthread_mutex_init(&h->log_lock, NULL);
    h->next_level = -1;
    /* entities/vectorindex/hnsw/config.go:33-50 defaults */
    h->ef = -1; h->ef_min = 100; h->ef_max = 500; h->ef_factor = 8;
    h->flat_cutoff = 40000;
    return h;
}

void wvo_destroy(wvo_index *h) {
    if (!h) return;
    for (uint64_t i = 0; i < h->cap; i++) {
        if (h->conns[i]) {
            for (int l = 0; l <= h->level[i]; l++) free(h->conns[i][l].ids);
            free(h->conns[i]);
        }
        pthread_mutex_destroy(&h->node_lock[i]);
    }
    free(h->conns); free(h->vecs); free(h->has_vec); free(h->level);
    free(h->maint); free(h->tomb); free(h->node_lock); free(h->log);
    free(h->pq_cent); free(h->pq_codes); free(h->pq_has);
    free(h);
}

void wvo_set_search_config(wvo_index *h, int64_t ef, int64_t ef_min,
                           int64_t ef_max, int64_t ef_factor,
                           int64_t flat_search_cutoff, int forbid_flat) {
    h->ef = ef; h->ef_min = ef_min; h->ef_max = ef_max; h->ef_factor = ef_factor;
    h->flat_cutoff = flat_search_cutoff; h->forbid_flat = forbid_flat;
}

static inline void nlock(wvo_index *h, uint64_t id) { if (h->threaded) pthread_mutex_lock(&h->node_lock[id]); }
static inline void nunlock(wvo_index *h, uint64_t id) { if (h->threaded) pthread_mutex_unlock(&h->node_lock[id]); }

int wvo_set_vector(wvo_index *h, uint64_t id, const float *vec) {
    if (id >= h->cap) return -1;
    float *dst = h->vecs + id * (uint64_t)h->dim;
    if (h->metric == WVO_COSINE) wvo_normalize(vec, dst, h->dim);
    else memcpy(dst, vec, sizeof(float) * h->dim);
    h->has_vec[id] = 1;
    return 0;
}

/* The object behind id left the object store (the shard deleted it): reads
 * through VectorForIDThunk now fail (shard_read.go:155-158). */
int wvo_clear_vector(wvo_index *h, uint64_t id) {
    if (id >= h->cap) return -1;
    h->has_vec[id] = 0;
    return 0;
}

static inline const float *vec_of(wvo_index *h, uint64_t id) { return h->vecs + id * (uint64_t)h->dim; }

/* distanceToFloatNode / distBetweenNodeAndVec (search.go:420-441,
 * index.go:492-538): ok=0 when the object store has no vector, after which a
 * tombstone is attached (handleDeletedNode, search.go:446-458). */
static inline int dist_node_vec(wvo_index *h, ctx_t *c, uint64_t id, const float *q, float *out) {
    if (h->compressed) {
        /* distanceToByteNode (search.go:403-418) / distBetweenNodeAndVec
         * compressed branch (index.go:493-511): a node without a code is
         * handled like a deleted one */
        if (id >= h->cap || !h->pq_has[id]) {
            if (id < h->cap) h->tomb[id] = 1;
            return 0;
        }
        if (c) c->st.dist_evals++;
        pq_layout L;
        pq_layout_of(h->pq_ks, h->pq_use_bits, &L);
        *out = pq_distance(h->metric, &L, q, h->pq_codes + id * h->pq_code_len, h->pq_cent, h->pq_m, h->pq_ks,
                           h->pq_ds);
        return 1;
    }
    if (id >= h->cap || !h->has_vec[id]) {
        if (id < h->cap) h->tomb[id] = 1;
        return 0;
    }
    if (c) c->st.dist_evals++;
    *out = metric_dist(h->metric, vec_of(h, id), q, h->dim);
    return 1;
}

/* Compress (compress.go:39-89) with a fitted quantizer: every later search
 * uses the PQ distance.  cent = kms[i].Centroid(c) for c < ks, i < m;
 * codes[n][code_len] in ProductQuantizer.Encode's layout for ids 0..n-1
 * (has[id] = 0 marks an id with no stored code). */
int wvo_compress(wvo_index *h, int m, int ks, int use_bits, const float *cent, const uint8_t *codes,
                 const uint8_t *has, uint64_t n) {
    pq_layout L;
    if (pq_layout_of(ks, use_bits, &L) || m <= 0 || h->dim % m || n > h->cap) return -1;
    h->pq_m = m; h->pq_ks = ks; h->pq_ds = h->dim / m; h->pq_use_bits = use_bits;
    h->pq_code_len = (uint64_t)m * L.bytes;
    free(h->pq_cent); free(h->pq_codes); free(h->pq_has);
    h->pq_cent = (float *)malloc(sizeof(float) * (size_t)m * ks * h->pq_ds);
    memcpy(h->pq_cent, cent, sizeof(float) * (size_t)m * ks * h->pq_ds);
    h->pq_codes = (uint8_t *)calloc(h->cap * h->pq_code_len + 8, 1);
    memcpy(h->pq_codes, codes, n * h->pq_code_len);
    h->pq_has = (uint8_t *)calloc(h->cap, 1);
    for (uint64_t i = 0; i < n; i++) h->pq_has[i] = has ? has[i] : 1;
    h->compressed = 1;
    return 0;
}

static conn_list *alloc_levels(int level, int M, int M0) {
    conn_list *cl = (conn_list *)calloc((size_t)level + 1, sizeof(conn_list));
    for (int l = 0; l <= level; l++) {
        cl[l].cap = (uint32_t)(l == 0 ? M0 : M);
        cl[l].ids = (uint32_t *)malloc(sizeof(uint32_t) * (cl[l].cap ? cl[l].cap : 1));
    }
    return cl;
}

static void conn_set(conn_list *cl, const uint32_t *ids, uint32_t n) {
    if (n > cl->cap) {
        cl->cap = n;
        cl->ids = (uint32_t *)realloc(cl->ids, sizeof(uint32_t) * n);
    }
    memcpy(cl->ids, ids, sizeof(uint32_t) * n);
    cl->len = n;
}
static void conn_append(conn_list *cl, uint32_t id) {
    if (cl->len == cl->cap) {
        cl->cap = cl->cap ? cl->cap * 2 : 4;
        cl->ids = (uint32_t *)realloc(cl->ids, sizeof(uint32_t) * cl->cap);
    }
    cl->ids[cl->len++] = id;
}

static int side_diag = 0;
void wvo_set_side_diag(int on) { side_diag = on; }

/* ---- searchLayerByVector -- search.go:160-327 ---------------------------- */
/* entrypoints: min-heap consumed; results: caller-initialised max heap. */
static void search_layer(wvo_index *h, ctx_t *c, const float *q, pq_t *eps,
                         int ef, int level, const uint64_t *allow,
                         uint64_t allow_nbits, pq_t *results) {
    ctx_reset_visited(c);
    pq_t *cand = &c->cand;
    cand->len = 0;
    results->len = 0;
    /* insertViableEntrypointsAsCandidatesAndResults (search.go:329-353) */
    while (eps->len > 0) {
        pq_item ep = pq_pop(eps);
        ctx_visit(c, ep.id);
        pq_insert(cand, ep.id, ep.dist);
        if (level == 0 && allow && !allow_contains(allow, allow_nbits, ep.id)) continue;
        if (ep.id < h->cap && h->tomb[ep.id]) continue;
        pq_insert(results, ep.id, ep.dist);
    }
    /* currentWorstResultDistanceToFloat (search.go:355-377) */
    float worst;
    if (results->len > 0) {
        float d;
        if (!dist_node_vec(h, NULL, results->it[0].id, q, &d)) worst = FLT_MAX;
        else worst = d;
    } else {
        worst = FLT_MAX;
    }

    uint64_t side_exp = 0;
    while (cand->len > 0) {
        if (cand->len > c->st.max_cand) c->st.max_cand = cand->len;
        if (side_diag && level == 0) {
            uint64_t live = 0;
            for (size_t i = 0; i < cand->len; i++) {
                const uint64_t id = cand->it[i].id;
                const int inel = (allow && !allow_contains(allow, allow_nbits, id)) || (id < h->cap && h->tomb[id]);
                if (inel && (cand->it[i].dist <= worst || (int)results->len < ef)) live++;
            }
            if (live > c->st.side_live_max) c->st.side_live_max = live;
        }
        /* :192-215 -- the top's distance is recomputed by the reference; it is
         * bit-identical to the stored value, so the stored one is used. */
        uint64_t top = cand->it[0].id;
        float dist;
        if (top >= h->cap || !h->has_vec[top]) {
            if (top < h->cap) h->tomb[top] = 1;
            pq_pop(cand);
            continue;
        }
        dist = cand->it[0].dist;
        if (dist > worst) break;
        pq_item candidate = pq_pop(cand);
        uint64_t cid = candidate.id;
        /* diagnostics only: an equal-distance candidate left on the heap means
         * the expansion order depends on heap layout */
        if (cand->len > 0 && cand->it[0].dist == candidate.dist) c->st.ties++;
        /* :217-254 */
        nlock(h, cid);
        if (h->level[cid] < 0 || h->conns[cid] == NULL) { nunlock(h, cid); continue; }
        if (h->level[cid] < level) { nunlock(h, cid); continue; }
        conn_list *cl = &h->conns[cid][level];
        if (cl->len > c->nbuf_cap) {
            c->nbuf_cap = cl->len;
            c->nbuf = (uint32_t *)realloc(c->nbuf, sizeof(uint32_t) * c->nbuf_cap);
        }
        uint32_t nn = cl->len;
        memcpy(c->nbuf, cl->ids, sizeof(uint32_t) * nn);
        nunlock(h, cid);
        c->st.expansions++;
        c->st.nbr_slots += nn;
        if (side_diag && level == 0 &&
            ((allow && !allow_contains(allow, allow_nbits, cid)) || (cid < h->cap && h->tomb[cid])))
            side_exp++;

        /* :256-315 */
        for (uint32_t i = 0; i < nn; i++) {
            uint64_t nb = c->nbuf[i];
            if (ctx_visited(c, nb)) continue;
            ctx_visit(c, nb);
            float d;
            if (!dist_node_vec(h, c, nb, q, &d)) continue;
            if (d == worst && (int)results->len >= ef) c->st.ties++;
            if (d < worst || (int)results->len < ef) {
                pq_insert(cand, nb, d);
                if (level == 0 && allow && !allow_contains(allow, allow_nbits, nb)) continue;
                if (nb < h->cap && h->tomb[nb]) continue;
                pq_insert(results, nb, d);
                if ((int)results->len > ef) pq_pop(results);
                if (results->len > 0) worst = results->it[0].dist;
            }
        }
    }
    c->st.side_exp += side_exp;
    if (side_exp > c->st.side_exp_max) c->st.side_exp_max = side_exp;
    c->st.visited += c->vis_count;
    if (level == 0 && c->vis_count > c->st.layer0_visited_max) c->st.layer0_visited_max = c->vis_count;
}

/* ---- knnSearchByVector -- search.go:460-550 -------------------------------- */
static int knn_search(wvo_index *h, ctx_t *c, const float *q, int k, int ef,
                      const uint64_t *allow, uint64_t allow_nbits,
                      uint64_t *out_ids, float *out_d, int *out_n) {
    *out_n = 0;
    if (atomic_load(&h->n_nodes) == 0) return 0; /* isEmpty -> nil, nil, nil */
    if (h->threaded) pthread_rwlock_rdlock(&h->glock);
    uint64_t ep = h->ep;
    int max_layer = h->max_layer;
    if (h->threaded) pthread_rwlock_unlock(&h->glock);
    float epd;
    if (!dist_node_vec(h, c, ep, q, &epd)) return -2; /* entrypoint deleted */
    pq_t eps, res;
    pq_init(&eps, 0, 10);
    pq_init(&res, 1, (size_t)ef + 1);
    for (int level = max_layer; level >= 1; level--) {
        eps.len = 0;
        pq_insert(&eps, ep, epd);
        search_layer(h, c, q, &eps, 1, level, NULL, 0, &res);
        while (res.len > 0) {
            pq_item cand = pq_pop(&res);
            if (cand.id >= h->cap || h->level[cand.id] < 0) {
                if (cand.id < h->cap) h->tomb[cand.id] = 1;
                continue;
            }
            if (!h->maint[cand.id]) {
                ep = cand.id;
                epd = cand.dist;
                break;
            }
        }
    }
    eps.len = 0;
    pq_insert(&eps, ep, epd);
    search_layer(h, c, q, &eps, ef, 0, allow, allow_nbits, &res);
    while ((int)res.len > k) pq_pop(&res);
    int n = (int)res.len;
    for (int i = n - 1; i >= 0; i--) {
        pq_item it = pq_pop(&res);
        out_ids[i] = it.id;
        out_d[i] = it.dist;
    }
    *out_n = n;
    pq_free(&eps);
    pq_free(&res);
    return 0;
}

/* ---- flatSearch -- flat_search.go:19-74 ------------------------------------ */
static int flat_search(wvo_index *h, const float *q, int limit, const uint64_t *allow,
                       uint64_t allow_nbits, uint64_t *out_ids, float *out_d, int *out_n) {
    pq_t res;
    pq_init(&res, 1, (size_t)limit + 1);
    for (uint64_t w = 0; w < (allow_nbits + 63) / 64; w++) {
        uint64_t word = allow[w];
        while (word) {
            int b = __builtin_ctzll(word);
            word &= word - 1;
            uint64_t cand = w * 64 + (uint64_t)b;
            if (cand >= allow_nbits) break;
            if (cand >= h->cap) continue;            /* :29-35 */
            if (h->level[cand] < 0 || h->tomb[cand]) continue; /* :36-40 */
            float d;
            if (!dist_node_vec(h, NULL, cand, q, &d)) continue;
            if ((int)res.len < limit) pq_insert(&res, cand, d);
            else if (res.it[0].dist > d) {
                pq_pop(&res);
                pq_insert(&res, cand, d);
            }
        }
    }
    int n = (int)res.len;
    for (int i = n - 1; i >= 0; i--) {
        pq_item it = pq_pop(&res);
        out_ids[i] = it.id;
        out_d[i] = it.dist;
    }
    *out_n = n;
    pq_free(&res);
    return 0;
}

static uint64_t popcount_bits(const uint64_t *bits, uint64_t nbits) {
    uint64_t c = 0, nw = nbits / 64;
    for (uint64_t w = 0; w < nw; w++) c += (uint64_t)__builtin_popcountll(bits[w]);
    if (nbits & 63) c += (uint64_t)__builtin_popcountll(bits[nw] & ((1ull << (nbits & 63)) - 1));
    return c;
}

/* ---- SearchByVector -- search.go:64-79 ------------------------------------ */
static int search_by_vector(wvo_index *h, ctx_t *c, const float *qin, int k,
                            const uint64_t *allow, uint64_t allow_nbits,
                            uint64_t *out_ids, float *out_d, int *out_n) {
    float qbuf[4096];
    float *qn = NULL;
    const float *q = qin;
    if (h->metric == WVO_COSINE) {
        qn = h->dim <= 4096 ? qbuf : (float *)malloc(sizeof(float) * h->dim);
        wvo_normalize(qin, qn, h->dim);
        q = qn;
    }
    int rc;
    if (allow && !h->forbid_flat && (int64_t)popcount_bits(allow, allow_nbits) < h->flat_cutoff)
        rc = flat_search(h, q, k, allow, allow_nbits, out_ids, out_d, out_n);
    else
        rc = knn_search(h, c, q, k,
                        wvo_search_time_ef(h->ef, h->ef_min, h->ef_max, h->ef_factor, k),
                        allow, allow_nbits, out_ids, out_d, out_n);
    if (qn && qn != qbuf) free(qn);
    return rc;
}

int wvo_search_by_vector(wvo_index *h, const float *q, int k,
                         const uint64_t *allow_bits, uint64_t allow_nbits,
                         uint64_t *out_ids, float *out_d, int *out_n, wvo_stats *st) {
    ctx_t c;
    ctx_init(&c, h->cap);
    int rc = search_by_vector(h, &c, q, k, allow_bits, allow_nbits, out_ids, out_d, out_n);
    if (st) *st = c.st;
    ctx_free(&c);
    return rc;
}

int wvo_knn_search(wvo_index *h, const float *q, int k, int ef,
                   const uint64_t *allow_bits, uint64_t allow_nbits,
                   uint64_t *out_ids, float *out_d, int *out_n, wvo_stats *st) {
    ctx_t c;
    ctx_init(&c, h->cap);
    int rc = knn_search(h, &c, q, k, ef, allow_bits, allow_nbits, out_ids, out_d, out_n);
    if (st) *st = c.st;
    ctx_free(&c);
    return rc;
}

int wvo_flat_search(wvo_index *h, const float *q, int k, const uint64_t *allow_bits,
                    uint64_t allow_nbits, uint64_t *out_ids, float *out_d, int *out_n) {
    return flat_search(h, q, k, allow_bits, allow_nbits, out_ids, out_d, out_n);
}

/* ---- SearchByVectorDistance -- search.go:90-158, 552-619 ------------------- */
int wvo_search_by_vector_distance(wvo_index *h, const float *q, float target,
                                  int64_t max_limit, const uint64_t *allow_bits,
                                  uint64_t allow_nbits, uint64_t *out_ids,
                                  float *out_d, int64_t out_cap, int64_t *out_n) {
    int64_t offset = 0, limit = 100, total = 100; /* DefaultSearchByDistInitialLimit */
    int64_t n_out = 0;
    ctx_t c;
    ctx_init(&c, h->cap);
    int rc = 0;
    for (int first = 1;; first = 0) {
        if (!first) {
            /* iterate (:607-611) and maxLimitReached (:613-619) */
            offset = total;
            limit *= 10; /* DefaultSearchByDistLimitMultiplier */
            total = offset + limit;
            if (max_limit >= 0 && total > max_limit) break;
        }
        uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)total);
        float *ds = (float *)malloc(sizeof(float) * (size_t)total);
        int n = 0;
        rc = search_by_vector(h, &c, q, (int)total, allow_bits, allow_nbits, ids, ds, &n);
        if (rc) { free(ids); free(ds); break; }
        int64_t lo = offset < n ? offset : n;   /* offsetCapacity */
        int64_t hi = total < n ? total : n;     /* totalLimitCapacity */
        int cont = 0;
        if (hi - lo > 0) {
            cont = ds[hi - 1] <= target;
            for (int64_t i = lo; i < hi; i++) {
                if (ds[i] <= target || fabs((double)ds[i] - (double)target) <= 1e-6) {
                    if (n_out < out_cap) { out_ids[n_out] = ids[i]; out_d[n_out] = ds[i]; }
                    n_out++;
                } else {
                    break;
                }
            }
        }
        free(ids); free(ds);
        if (!cont) break;
    }
    ctx_free(&c);
    *out_n = n_out;
    return rc;
}

/* ======================================================================== */
/* Graph construction -- insert.go, neighbor_connections.go, heuristic.go   */
/* ======================================================================== */

/* selectNeighborsHeuristic (heuristic.go:23-135); input is a max-heap that is
 * rewritten in place; denyList is always the empty allow list here. */
static void select_neighbors_heuristic(wvo_index *h, pq_t *input, int max) {
    if ((int)input->len < max) return;
    size_t n = input->len;
    uint64_t *ids = (uint64_t *)malloc(sizeof(uint64_t) * n);
    pqi_t closest = {0};
    uint64_t i = 0;
    while (input->len > 0) {
        pq_item e = pq_pop(input);
        pqi_insert(&closest, e.id, i, e.dist);
        ids[i] = e.id;
        i++;
    }
    pqi_item *ret = (pqi_item *)malloc(sizeof(pqi_item) * n);
    int nret = 0;
    while (closest.len > 0 && nret < max) {
        pqi_item curr = pqi_pop(&closest);
        float dq = curr.dist;
        const float *cv = vec_of(h, ids[curr.index]);
        int good = 1;
        for (int r = 0; r < nret; r++) {
            /* SingleDist(currVec, vecs[item.Index]) */
            float pd = metric_dist(h->metric, cv, vec_of(h, ids[ret[r].index]), h->dim);
            if (pd < dq) { good = 0; break; }
        }
        if (good) ret[nret++] = curr;
    }
    for (int r = 0; r < nret; r++) pq_insert(input, ret[r].id, ret[r].dist);
    free(closest.it);
    free(ret);
    free(ids);
}

/* connectNeighborAtLevel (neighbor_connections.go:134-209) */
static void connect_neighbor(wvo_index *h, uint64_t node, uint64_t nb, int level) {
    if (nb == node) return;                               /* skipNeighbor */
    if (nb >= h->cap || h->level[nb] < 0 || h->tomb[nb]) return;
    nlock(h, nb);
    if (level > h->level[nb]) {                           /* upgradeToLevelNoLock */
        conn_list *nl = alloc_levels(level, h->M, h->M0);
        for (int l = 0; l <= h->level[nb]; l++) {
            free(nl[l].ids);
            nl[l] = h->conns[nb][l];
        }
        free(h->conns[nb]);
        h->conns[nb] = nl;
        h->level[nb] = (int8_t)level;
    }
    conn_list *cl = &h->conns[nb][level];
    int maxc = level == 0 ? h->M0 : h->M;
    if ((int)cl->len < maxc) {
        conn_append(cl, (uint32_t)node);
        log_add_link(h, nb, level, node);                 /* :155 */
    } else {
        float d = metric_dist(h->metric, vec_of(h, node), vec_of(h, nb), h->dim);
        pq_t cands;
        pq_init(&cands, 1, cl->len + 1);
        pq_insert(&cands, node, d);
        for (uint32_t i = 0; i < cl->len; i++) {
            uint64_t ex = cl->ids[i];
            if (!h->has_vec[ex]) continue;
            float de = metric_dist(h->metric, vec_of(h, ex), vec_of(h, nb), h->dim);
            pq_insert(&cands, ex, de);
        }
        select_neighbors_heuristic(h, &cands, maxc);
        cl->len = 0;
        log_id_level(h, CL_CLEAR_LINKS_AT_LEVEL, nb, level);   /* :194-197 */
        while (cands.len > 0) {
            uint64_t id = pq_pop(&cands).id;
            conn_append(cl, (uint32_t)id);
            log_add_link(h, nb, level, id);                   /* :199-205 */
        }
        pq_free(&cands);
    }
    nunlock(h, nb);
}

/* findBestEntrypointForNode (index.go:371-408) */
static uint64_t find_best_entrypoint(wvo_index *h, ctx_t *c, int cur_max, int target,
                                     uint64_t ep, const float *vec) {
    pq_t eps, res;
    pq_init(&eps, 0, 4);
    pq_init(&res, 1, 4);
    for (int level = cur_max; level > target; level--) {
        float d;
        if (!dist_node_vec(h, c, ep, vec, &d)) continue;
        eps.len = 0;
        pq_insert(&eps, ep, d);
        search_layer(h, c, vec, &eps, 1, level, NULL, 0, &res);
        if (res.len > 0) {
            pq_item e = pq_pop(&res);
            if (e.id < h->cap && h->level[e.id] >= 0 && !h->maint[e.id]) ep = e.id;
        }
    }
    pq_free(&eps);
    pq_free(&res);
    return ep;
}

/* neighborFinderConnector (neighbor_connections.go:23-132, 229-307) */
static void find_and_connect(wvo_index *h, ctx_t *c, uint64_t node, uint64_t ep,
                             const float *vec, int target, int cur_max) {
    pq_t eps, res;
    pq_init(&eps, 0, 4);
    pq_init(&res, 1, (size_t)h->efC + 1);
    uint32_t *nbrs = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)h->efC + 1));
    int top = target < cur_max ? target : cur_max;
    for (int level = top; level >= 0; level--) {
        /* pickEntrypoint / tryEpCandidate (:236-307).  A candidate under
         * maintenance (only possible in a concurrent build) is replaced by
         * the global entrypoint, as findNewLocalEntrypoint does when the
         * global entrypoint differs (delete.go:480-489). */
        if (ep >= h->cap || h->level[ep] < 0 || h->maint[ep]) {
            if (h->threaded) pthread_rwlock_rdlock(&h->glock);
            ep = h->ep;
            if (h->threaded) pthread_rwlock_unlock(&h->glock);
        }
        float epd = FLT_MAX;
        dist_node_vec(h, c, ep, vec, &epd);
        eps.len = 0;
        pq_insert(&eps, ep, epd);
        search_layer(h, c, vec, &eps, h->efC, level, NULL, 0, &res);
        select_neighbors_heuristic(h, &res, h->M); /* max = maximumConnections */
        int nn = 0;
        while (res.len > 0) nbrs[nn++] = (uint32_t)pq_pop(&res).id;
        nlock(h, node);
        conn_set(&h->conns[node][level], nbrs, (uint32_t)nn); /* setConnectionsAtLevel */
        log_replace_links(h, node, level, nbrs, (uint32_t)nn); /* :111 */
        nunlock(h, node);
        for (int i = 0; i < nn; i++) connect_neighbor(h, node, nbrs[i], level);
        if (nn > 0) {
            uint64_t next = nbrs[nn - 1];
            if (next == node) break;
            ep = next;
        }
    }
    free(nbrs);
    pq_free(&eps);
    pq_free(&res);
}

static uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

/* insert (insert.go:103-217) with insertInitialElement (:67-101) */
static int insert_node(wvo_index *h, ctx_t *c, uint64_t id, int forced_level) {
    const float *vec = vec_of(h, id);
    int was_first = 0;
    pthread_mutex_lock(&h->init_lock);
    if (!h->initial_done) {
        h->initial_done = 1;
        if (atomic_load(&h->n_nodes) == 0) {
            was_first = 1;
            log_id_level(h, CL_SET_EP, id, 0);                /* insertInitialElement :71 */
            h->conns[id] = alloc_levels(0, h->M, h->M0);
            h->level[id] = 0;
            log_id_level(h, CL_ADD_NODE, id, 0);              /* :81 */
            if (h->threaded) pthread_rwlock_wrlock(&h->glock);
            h->ep = id;
            h->max_layer = 0;
            if (h->threaded) pthread_rwlock_unlock(&h->glock);
            atomic_fetch_add(&h->n_nodes, 1);
        }
    }
    pthread_mutex_unlock(&h->init_lock);
    if (was_first) return 0;

    h->maint[id] = 1;
    if (h->threaded) pthread_rwlock_rdlock(&h->glock);
    uint64_t ep = h->ep;
    int cur_max = h->max_layer;
    if (h->threaded) pthread_rwlock_unlock(&h->glock);

    int target;
    if (forced_level >= 0) {
        target = forced_level;
    } else {
        /* targetLevel = floor(-ln(U) * levelNormalizer), U ~ rand.Float64 */
        uint64_t r = mix64(h->seed * 0xD1B54A32D192ED03ull + id * 0x9E3779B97F4A7C15ull + 1);
        double u = ((double)(r >> 11) + 0.5) * (1.0 / 9007199254740992.0);
        target = (int)floor(-log(u) * h->level_normalizer);
    }
    if (target > 126) target = 126;
    conn_list *cl = alloc_levels(target, h->M, h->M0);
    nlock(h, id);
    h->conns[id] = cl;
    h->level[id] = (int8_t)target;
    nunlock(h, id);
    log_id_level(h, CL_ADD_NODE, id, target);             /* insert.go:148 */
    atomic_fetch_add(&h->n_nodes, 1);

    ep = find_best_entrypoint(h, c, cur_max, target, ep, vec);
    find_and_connect(h, c, id, ep, vec, target, cur_max);
    h->maint[id] = 0;

    if (h->threaded) pthread_rwlock_wrlock(&h->glock);
    if (target > h->max_layer) {
        log_id_level(h, CL_SET_EP, id, target);           /* insert.go:206 */
        h->ep = id;
        h->max_layer = target;
    }
    if (h->threaded) pthread_rwlock_unlock(&h->glock);
    return 0;
}

void wvo_set_next_level(wvo_index *h, int level) { h->next_level = level; }

int wvo_add(wvo_index *h, uint64_t id, const float *vec) {
    if (id >= h->cap) return -1;
    if (h->level[id] >= 0) return -3;
    wvo_set_vector(h, id, vec); /* Add normalizes for cosine (insert.go:56-60) */
    if (h->compressed) {
        /* insert.go:91-95: a compressed index stores the new node's code
         * (pq.Encode of the stored vector; KMeans encoders: the nearest centre
         * per segment, kmeans.go:78-110) */
        wvo_pq_encode_kmeans(vec_of(h, id), 1, h->dim, h->pq_m, h->pq_ks, h->pq_cent, h->pq_use_bits,
                             h->pq_codes + id * h->pq_code_len);
        h->pq_has[id] = 1;
    }
    ctx_t c;
    ctx_init(&c, h->cap);
    int lvl = h->next_level;
    h->next_level = -1;
    int rc = insert_node(h, &c, id, lvl);
    ctx_free(&c);
    return rc;
}

typedef struct {
    wvo_index *h;
    uint64_t first, n;
    atomic_uint_fast64_t *next;
} build_arg;

static void *build_worker(void *p) {
    build_arg *a = (build_arg *)p;
    ctx_t c;
    ctx_init(&c, a->h->cap);
    for (;;) {
        uint64_t i = atomic_fetch_add(a->next, 1);
        if (i >= a->n) break;
        insert_node(a->h, &c, a->first + i, -1);
    }
    ctx_free(&c);
    return NULL;
}

int wvo_add_batch(wvo_index *h, uint64_t first_id, const float *vecs, uint64_t n, int threads) {
    if (first_id + n > h->cap) return -1;
    for (uint64_t i = 0; i < n; i++) wvo_set_vector(h, first_id + i, vecs + i * (uint64_t)h->dim);
    if (threads <= 1) {
        ctx_t c;
        ctx_init(&c, h->cap);
        for (uint64_t i = 0; i < n; i++) insert_node(h, &c, first_id + i, -1);
        ctx_free(&c);
        return 0;
    }
    /* the first insert is done alone (initialInsertOnce) so every concurrent
     * insert sees a non-empty graph */
    uint64_t start = 0;
    if (atomic_load(&h->n_nodes) == 0 && n > 0) {
        ctx_t c;
        ctx_init(&c, h->cap);
        insert_node(h, &c, first_id, -1);
        ctx_free(&c);
        start = 1;
    }
    h->threaded = 1;
    atomic_uint_fast64_t next = start;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    build_arg a = {h, first_id, n, &next};
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, build_worker, &a);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    h->threaded = 0;
    return 0;
}

int wvo_add_tombstone(wvo_index *h, uint64_t id) {
    if (id >= h->cap) return -1;
    h->tomb[id] = 1;
    log_id(h, CL_ADD_TOMB, id);                           /* delete.go -> AddTombstone */
    return 0;
}
int wvo_remove_tombstone(wvo_index *h, uint64_t id) {
    if (id >= h->cap) return -1;
    h->tomb[id] = 0;
    return 0;
}

/* ---- graph import / export ------------------------------------------------ */
int wvo_import_node(wvo_index *h, uint64_t id, int level, const uint64_t *conns, const int *counts) {
    if (id >= h->cap || level < 0) return -1;
    conn_list *cl = (conn_list *)calloc((size_t)level + 1, sizeof(conn_list));
    size_t off = 0;
    for (int l = 0; l <= level; l++) {
        uint32_t n = (uint32_t)counts[l];
        uint32_t cap = (uint32_t)(l == 0 ? h->M0 : h->M);
        if (cap < n) cap = n;
        cl[l].cap = cap ? cap : 1;
        cl[l].ids = (uint32_t *)malloc(sizeof(uint32_t) * cl[l].cap);
        for (uint32_t i = 0; i < n; i++) cl[l].ids[i] = (uint32_t)conns[off + i];
        cl[l].len = n;
        off += n;
    }
    if (h->level[id] < 0) atomic_fetch_add(&h->n_nodes, 1);
    h->conns[id] = cl;
    h->level[id] = (int8_t)level;
    h->initial_done = 1;
    return 0;
}

/* Bulk restore from the fixed-degree CSR of wvo_export_layer0/_upper (the
 * bench's graph cache): vectors rows [0, n) and every node's lists in stored
 * order (NIL_ID pads dropped).  Equivalent to import_node per node. */
int wvo_import_csr(wvo_index *h, uint64_t n, const float *vecs, const int8_t *levels, const uint32_t *layer0,
                   int deg0, const uint32_t *upper_row, const uint32_t *upper, int degU, int max_level,
                   uint64_t entrypoint) {
    if (n > h->cap) return -1;
    uint64_t *buf = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)deg0 + (size_t)degU * (max_level + 1) + 1));
    int *counts = (int *)malloc(sizeof(int) * ((size_t)max_level + 2));
    for (uint64_t i = 0; i < n; i++) {
        wvo_set_vector(h, i, vecs + i * (uint64_t)h->dim);
        if (levels[i] < 0) continue;
        size_t off = 0;
        int c = 0;
        for (int j = 0; j < deg0; j++) {
            uint32_t v = layer0[i * (uint64_t)deg0 + j];
            if (v == NIL_ID) break;
            buf[off++] = v;
            c++;
        }
        counts[0] = c;
        for (int l = 1; l <= levels[i]; l++) {
            const uint32_t *row = upper + ((uint64_t)upper_row[i] * max_level + (l - 1)) * degU;
            c = 0;
            for (int j = 0; j < degU; j++) {
                if (row[j] == NIL_ID) break;
                buf[off++] = row[j];
                c++;
            }
            counts[l] = c;
        }
        wvo_import_node(h, i, levels[i], buf, counts);
    }
    free(buf);
    free(counts);
    wvo_set_entrypoint(h, entrypoint, max_level);
    return 0;
}

void wvo_set_entrypoint(wvo_index *h, uint64_t ep, int max_level) {
    h->ep = ep;
    h->max_layer = max_level;
}

void wvo_graph_info(wvo_index *h, uint64_t *n_slots, uint64_t *entrypoint, int *max_level,
                    uint64_t *n_upper_nodes) {
    uint64_t hi = 0, up = 0;
    for (uint64_t i = 0; i < h->cap; i++)
        if (h->level[i] >= 0) {
            hi = i + 1;
            if (h->level[i] >= 1) up++;
        }
    *n_slots = hi;
    *entrypoint = h->ep;
    *max_level = h->max_layer;
    *n_upper_nodes = up;
}

int wvo_export_layer0(wvo_index *h, int deg0, int8_t *levels, uint32_t *layer0, uint32_t *counts0) {
    uint64_t n, ep, up;
    int ml;
    wvo_graph_info(h, &n, &ep, &ml, &up);
    int over = 0;
    for (uint64_t i = 0; i < n; i++) {
        levels[i] = h->level[i];
        uint32_t *row = layer0 + i * (uint64_t)deg0;
        uint32_t len = 0;
        if (h->level[i] >= 0) {
            conn_list *cl = &h->conns[i][0];
            len = cl->len;
            if ((int)len > deg0) { len = (uint32_t)deg0; over = 1; }
            memcpy(row, cl->ids, sizeof(uint32_t) * len);
        }
        for (uint32_t j = len; j < (uint32_t)deg0; j++) row[j] = NIL_ID;
        counts0[i] = len;
    }
    return over ? 1 : 0;
}

int wvo_export_upper(wvo_index *h, int degU, int max_level, uint32_t *upper_row, uint32_t *upper,
                     uint64_t n_rows) {
    uint64_t n, ep, up;
    int ml;
    wvo_graph_info(h, &n, &ep, &ml, &up);
    uint64_t r = 0;
    int over = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (h->level[i] < 1) { upper_row[i] = NIL_ID; continue; }
        if (r >= n_rows) return -1;
        upper_row[i] = (uint32_t)r;
        uint32_t *base = upper + r * (uint64_t)max_level * degU;
        for (int l = 1; l <= max_level; l++) {
            uint32_t *row = base + (uint64_t)(l - 1) * degU;
            uint32_t len = 0;
            if (l <= h->level[i]) {
                conn_list *cl = &h->conns[i][l];
                len = cl->len;
                if ((int)len > degU) { len = (uint32_t)degU; over = 1; }
                memcpy(row, cl->ids, sizeof(uint32_t) * len);
            }
            for (uint32_t j = len; j < (uint32_t)degU; j++) row[j] = NIL_ID;
        }
        r++;
    }
    return over ? 1 : 0;
}

/* ---- batched search (ssdhelpers.Concurrently split) ------------------------ */
typedef struct {
    wvo_index *h;
    const float *qs;
    int q0, q1, k, ef, mode;
    const uint64_t *allow;
    uint64_t allow_nbits;
    uint64_t *out_ids;
    float *out_d;
    int *out_n;
    wvo_stats st;
} batch_arg;

static void *batch_worker(void *p) {
    batch_arg *a = (batch_arg *)p;
    wvo_index *h = a->h;
    ctx_t c;
    ctx_init(&c, h->cap);
    float *qn = (float *)malloc(sizeof(float) * h->dim);
    for (int qi = a->q0; qi < a->q1; qi++) {
        const float *q = a->qs + (uint64_t)qi * h->dim;
        if (h->metric == WVO_COSINE) { wvo_normalize(q, qn, h->dim); q = qn; }
        uint64_t *oi = a->out_ids + (uint64_t)qi * a->k;
        float *od = a->out_d + (uint64_t)qi * a->k;
        if (a->mode == 0)
            knn_search(h, &c, q, a->k, a->ef, a->allow, a->allow_nbits, oi, od, &a->out_n[qi]);
        else
            flat_search(h, q, a->k, a->allow, a->allow_nbits, oi, od, &a->out_n[qi]);
    }
    free(qn);
    a->st = c.st;
    ctx_free(&c);
    return NULL;
}

int wvo_search_batch(wvo_index *h, const float *qs, int nq, int k, int ef,
                     const uint64_t *allow_bits, uint64_t allow_nbits, int mode,
                     int threads, uint64_t *out_ids, float *out_d, int *out_n, wvo_stats *st) {
    if (threads < 1) threads = 1;
    if (threads > nq) threads = nq > 0 ? nq : 1;
    uint64_t *all = NULL;
    if (mode == 1 && !allow_bits) {
        /* exact search over every node: an allow list of all ids */
        allow_nbits = h->cap;
        all = (uint64_t *)malloc(sizeof(uint64_t) * ((h->cap + 63) / 64));
        memset(all, 0xFF, sizeof(uint64_t) * ((h->cap + 63) / 64));
        allow_bits = all;
    }
    batch_arg *args = (batch_arg *)calloc((size_t)threads, sizeof(batch_arg));
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    int chunk = (nq + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        int q0 = t * chunk, q1 = q0 + chunk;
        if (q1 > nq) q1 = nq;
        if (q0 > nq) q0 = nq;
        args[t] = (batch_arg){h, qs, q0, q1, k, ef, mode, allow_bits, allow_nbits,
                              out_ids, out_d, out_n, {0}};
        pthread_create(&th[t], NULL, batch_worker, &args[t]);
    }
    wvo_stats tot = {0};
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        tot.dist_evals += args[t].st.dist_evals;
        tot.expansions += args[t].st.expansions;
        tot.nbr_slots += args[t].st.nbr_slots;
        tot.visited += args[t].st.visited;
        tot.ties += args[t].st.ties;
        if (args[t].st.max_cand > tot.max_cand) tot.max_cand = args[t].st.max_cand;
        tot.side_exp += args[t].st.side_exp;
        if (args[t].st.side_exp_max > tot.side_exp_max) tot.side_exp_max = args[t].st.side_exp_max;
        if (args[t].st.side_live_max > tot.side_live_max) tot.side_live_max = args[t].st.side_live_max;
        if (args[t].st.layer0_visited_max > tot.layer0_visited_max)
            tot.layer0_visited_max = args[t].st.layer0_visited_max;
    }
    if (st) *st = tot;
    free(args); free(th); free(all);
    return 0;
}

/* ---- standalone flat scan -------------------------------------------------- */
typedef struct {
    int metric, dim, k;
    const float *base;
    uint64_t n;
    const float *qs;
    int q0, q1;
    const uint64_t *allow, *tomb;
    uint64_t *out_ids;
    float *out_d;
    int *out_n;
} scan_arg;

static void *scan_worker(void *p) {
    scan_arg *a = (scan_arg *)p;
    pq_t res;
    pq_init(&res, 1, (size_t)a->k + 1);
    for (int qi = a->q0; qi < a->q1; qi++) {
        const float *q = a->qs + (uint64_t)qi * a->dim;
        res.len = 0;
        for (uint64_t id = 0; id < a->n; id++) {
            if (a->allow && !((a->allow[id >> 6] >> (id & 63)) & 1u)) continue;
            if (a->tomb && ((a->tomb[id >> 6] >> (id & 63)) & 1u)) continue;
            float d = metric_dist(a->metric, a->base + id * (uint64_t)a->dim, q, a->dim);
            if ((int)res.len < a->k) pq_insert(&res, id, d);
            else if (res.it[0].dist > d) { pq_pop(&res); pq_insert(&res, id, d); }
        }
        int n = (int)res.len;
        for (int i = n - 1; i >= 0; i--) {
            pq_item it = pq_pop(&res);
            a->out_ids[(uint64_t)qi * a->k + i] = it.id;
            a->out_d[(uint64_t)qi * a->k + i] = it.dist;
        }
        a->out_n[qi] = n;
    }
    pq_free(&res);
    return NULL;
}

int wvo_flat_scan(int metric, const float *base, uint64_t n, int dim, const float *qs, int nq,
                  int k, const uint64_t *allow_bits, const uint64_t *tomb_bits, int threads,
                  uint64_t *out_ids, float *out_d, int *out_n) {
    have_avx2();
    if (threads < 1) threads = 1;
    if (threads > nq) threads = nq > 0 ? nq : 1;
    scan_arg *args = (scan_arg *)calloc((size_t)threads, sizeof(scan_arg));
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    int chunk = (nq + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        int q0 = t * chunk, q1 = q0 + chunk;
        if (q1 > nq) q1 = nq;
        if (q0 > nq) q0 = nq;
        args[t] = (scan_arg){metric, dim, k, base, n, qs, q0, q1, allow_bits, tomb_bits,
                             out_ids, out_d, out_n};
        pthread_create(&th[t], NULL, scan_worker, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(args); free(th);
    return 0;
}
