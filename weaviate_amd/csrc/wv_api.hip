// wv_api.hip -- host side of the C ABI declared in include/wvgpu.h.
//
// Owns device memory for one index (vectors, norms, CSR graph, bitmaps),
// dispatches SearchByVector the way the reference does (search.go:64-79) and
// runs the device pipelines of wv_bf.hip / wv_hnsw.hip.  No CPU search code:
// every distance and every selection happens on the GPU.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/wvgpu.h"
#include "wv_device.h"

#include "wv_params.h"

extern "C" {
hipError_t wv_launch_bf_mfma(const wv::BfParams* p, hipStream_t s);
hipError_t wv_launch_bf_finalize(const wv::BfFinParams* p, hipStream_t s);
hipError_t wv_launch_bf_finalize_wide(const wv::BfFinParams* p, hipStream_t s);
hipError_t wv_launch_exact_scan(const wv::ScanParams* p, hipStream_t s);
hipError_t wv_launch_fb(const wv::FbParams* p, hipStream_t s);
hipError_t wv_launch_fbd(const int32_t* flags, int nq, const wv::FbParams* fb, hipStream_t s);
hipError_t wv_launch_fbd_mark(const int32_t* status, int nq, int32_t* flags, float* thr, const float* out_d,
                              const int32_t* out_n, int k, hipStream_t s);
hipError_t wv_launch_hnsw_stats(const uint32_t* counters, int nq, unsigned long long* acc, hipStream_t s);
hipError_t wv_launch_rownorm(const float* X, uint64_t N, int D, int ldx, float* norm2, unsigned int* maxbits,
                             hipStream_t s);
hipError_t wv_launch_normalize(const float* in, float* out, uint64_t n, int D, int ld, hipStream_t s);
hipError_t wv_launch_scale(const float* in, float* out, uint64_t n, float scale, hipStream_t s);
hipError_t wv_launch_qnorm(const float* Q, int nq, int D, int ldq, int metric, float* out, float* absmax_part,
                           hipStream_t s);
hipError_t wv_launch_hnsw(const wv::HnswParams* p, int waves_per_block, hipStream_t s);
hipError_t wv_launch_hnsw_wg(const wv::HnswParams* p, hipStream_t s);
hipError_t wv_launch_build_search(const wv::BuildParams* b, int waves_per_block, hipStream_t s);
hipError_t wv_launch_build_select(const wv::BuildParams* b, hipStream_t s);
hipError_t wv_launch_build_link(const wv::BuildParams* b, hipStream_t s);
int wv_hnsw_per_wave_words(int dpad, int efc, int sc, int vc_log2, int xs_log2);
int wv_hnsw_side_per_wave_words(int dpad, int side_rows, int vc_log2, int xs_log2);
int wv_hnsw_reg_per_wave_words(int dpad, int vc_log2);
hipError_t wv_launch_hnsw_side(const wv::HnswParams* p, int waves_per_block, int ev, hipStream_t s);
hipError_t wv_launch_sbd_scan(const wv::SbdParams* p, hipStream_t s);
hipError_t wv_sbd_sort(unsigned long long* keys, unsigned long long* tmp, const unsigned int* cnt, int nq, int cap,
                       int* offsets, void** scratch, size_t* scratch_cap, hipStream_t s);
hipError_t wv_launch_pq_encode(const float* X, int ldx, const uint64_t* ids, uint64_t n_rows, const wv::PqParams* pq,
                               uint8_t* codes, hipStream_t s);
hipError_t wv_launch_pq_scan(const wv::PqScanParams* p, hipStream_t s);
hipError_t wv_launch_split_rows(const float* in, int ld_in, const uint64_t* ids, uint64_t n, uint64_t n_valid, int D,
                                float scale, void* out, int ld_out, uint64_t out_row0, hipStream_t s);
hipError_t wv_launch_h16_rows(const float* in, int ld_in, const uint64_t* ids, uint64_t n, int D, int ns, float sign,
                              float scale, const unsigned int* scale_from_max, void* out, uint64_t out_row0,
                              unsigned int* res_max_bits, float* res_out, int wide_layout, hipStream_t s);
hipError_t wv_launch_h16_rows_gather(const float* in, int ld_in, const uint32_t* gather, uint64_t n, uint64_t n_pad,
                                     int D, int ns, float scale, void* out, hipStream_t s);
hipError_t wv_launch_h16_compact_aux(const float* xnorm, const uint32_t* rowidx, uint64_t n, const uint32_t* n_dev,
                                     float* cxnorm, uint64_t* excl, uint64_t excl_words, hipStream_t s);
hipError_t wv_launch_remap_ids(uint32_t* ids, int nq, int n_slots, int per_slot, int bq, uint64_t ntiles,
                               uint64_t units_per_block, const uint32_t* rowidx, uint64_t n_rows, const uint32_t* n_dev,
                               hipStream_t s);
hipError_t wv_launch_absmax(const float* in, int ld, uint64_t n, int D, unsigned int* max_bits, hipStream_t s);
hipError_t wv_launch_h16_qscale(const float* part, int nparts, unsigned int* max_bits, float bsign, float* qscale,
                                hipStream_t s);
hipError_t wv_launch_h16_xns(const float* xnorm, uint64_t n, float sx, const float* qscale, float* xns, hipStream_t s);
hipError_t wv_launch_bf_h16(const wv::H16Params* p, int ns, int seed, hipStream_t s);
hipError_t wv_launch_bf_h16w(const wv::H16Params* p, hipStream_t s);
hipError_t wv_launch_h16_seed(const wv::H16SeedParams* p, hipStream_t s);
hipError_t wv_launch_h16_margin(int metric, int D, const float* qnorm, const float* qres, float xnorm_max,
                                float ex_max, float sx, const float* qscale, int nq, float* marg, hipStream_t s);
hipError_t wv_launch_h16_gtau(const unsigned int* gtau, int nq, float sx, const float* qscale, float* tau,
                              hipStream_t s);
float wv_h16_pow2_scale(float maxabs);
hipError_t wv_launch_pq_topk(const float* skey, const uint32_t* sval, const float* dist, const uint32_t* rows,
                             uint64_t nr, int q0, int nqc, int k, uint64_t id_base, uint64_t* out_ids, float* out_d,
                             int32_t* out_n, hipStream_t s);
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail(_e == hipErrorOutOfMemory ? WV_EOOM : WV_EDEVICE,                      \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                   \
    } while (0)
// record timing event i of the current batch's set (wv_index::ev)
#define TREC(i)                                                                     \
    do {                                                                            \
        if (ix->timing && ix->ev) {                                                 \
            HIP_TRY(hipEventRecord(ix->ev[i], s));                                  \
            ix->ev_mask[ix->ev_used - 1] |= (uint8_t)(1u << (i));                   \
        }                                                                           \
    } while (0)

// growable device scratch buffer
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        // batches may still be queued that read the old buffer (several in
        // flight on the index's stream, wv_search_batch): drain the device
        // before it goes
        size_t want = std::max<size_t>(bytes, 256);
        // scratch that grows with the batch: geometric steps (bounded), so a
        // stream of growing batches does not reallocate -- and drain -- each time
        if (cap) want = std::max(want, std::min(cap + cap / 2, bytes + ((size_t)256 << 20)));
        if (p) { (void)hipDeviceSynchronize(); (void)hipFree(p); }
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

__global__ void gather_rows_kernel(const float* src, int ld_src, const int32_t* idx, int n, int D, float* dst,
                                   int ld_dst) {
    const int r = blockIdx.x;
    if (r >= n) return;
    const float* s = src + (size_t)idx[r] * ld_src;
    float* d = dst + (size_t)r * ld_dst;
    for (int i = threadIdx.x; i < ld_dst; i += blockDim.x) d[i] = i < D ? s[i] : 0.f;
}

// copy rows [n][ld_src] into the padded layout [n][ld_dst], zero-filling D..ld_dst
__global__ void pad_rows_kernel(const float* src, uint64_t ld_src, uint64_t n, int D, float* dst, int ld_dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t r = i / ld_dst;
    const int c = (int)(i % ld_dst);
    if (r >= n) return;
    dst[r * ld_dst + c] = c < D ? src[r * ld_src + c] : 0.f;
}

hipError_t launch_pad_rows(const float* src, uint64_t ld_src, uint64_t n, int D, float* dst, int ld_dst, hipStream_t s) {
    const uint64_t total = n * (uint64_t)ld_dst;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, src, ld_src, n, D, dst,
                       ld_dst);
    return hipGetLastError();
}

__global__ void gather_words_kernel(const uint64_t* src, uint64_t stride, const int32_t* idx, int n, uint64_t* dst) {
    const int r = blockIdx.x;
    if (r >= n) return;
    for (uint64_t i = threadIdx.x; i < stride; i += blockDim.x) dst[r * stride + i] = src[(uint64_t)idx[r] * stride + i];
}

__global__ void scatter_results_kernel(const uint64_t* ids, const float* ds, const int32_t* ns, const int32_t* idx,
                                       int n, int k, uint64_t* out_ids, float* out_d, int32_t* out_n) {
    const int r = blockIdx.x;
    if (r >= n) return;
    const int q = idx[r];
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
        out_ids[(size_t)q * k + i] = ids[(size_t)r * k + i];
        out_d[(size_t)q * k + i] = ds[(size_t)r * k + i];
    }
    if (threadIdx.x == 0) out_n[q] = ns[r];
}

__global__ void copy_topk_kernel(const float* sd, const uint32_t* si, uint64_t n_eligible_cap, int k, uint64_t id_base,
                                 uint64_t* out_ids, float* out_d, int32_t* out_n) {
    // first k of a sorted (dist, id) array; +inf marks ineligible rows
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
        if ((uint64_t)i < n_eligible_cap && sd[i] != __builtin_inff()) {
            out_ids[i] = id_base + si[i];
            out_d[i] = sd[i];
            atomicAdd(&cnt, 1);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *out_n = cnt;
}

__global__ void merge_shards_kernel(const float* in_d, const uint64_t* in_ids, const int32_t* in_n, int n_shards,
                                    int nq, int k, float* out_d, uint64_t* out_ids, int32_t* out_n) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    int head[16];
    for (int s = 0; s < n_shards; ++s) head[s] = 0;
    int n = 0;
    for (; n < k; ++n) {
        int best = -1;
        float bd = 0.f;
        uint64_t bi = 0;
        for (int s = 0; s < n_shards; ++s) {
            const int cnt = in_n[(size_t)s * nq + q];
            if (head[s] >= cnt) continue;
            const size_t off = ((size_t)s * nq + q) * k + head[s];
            const float d = in_d[off];
            const uint64_t id = in_ids[off];
            if (best < 0 || d < bd || (d == bd && id < bi)) { best = s; bd = d; bi = id; }
        }
        if (best < 0) break;
        head[best]++;
        out_d[(size_t)q * k + n] = bd;
        out_ids[(size_t)q * k + n] = bi;
    }
    out_n[q] = n;
}

// queries whose search reported an overflow (status != 0) into *acc
__global__ void count_nonzero_kernel(const int32_t* st, int n, unsigned long long* acc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool nz = i < n && st[i] != 0;
    const unsigned long long c = __popcll(__ballot(nz));
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(acc, c);
}

__global__ void popcount_rows_kernel(const uint64_t* bits, uint64_t words, uint64_t stride, int nrows,
                                     unsigned long long* out) {
    const int r = blockIdx.x;
    if (r >= nrows) return;
    unsigned long long c = 0;
    for (uint64_t i = threadIdx.x; i < words; i += blockDim.x) c += __popcll(bits[r * stride + i]);
    atomicAdd(&out[r], c);
}

}  // namespace

// rows of the corpus buffers: whole 128-row tiles of the brute-force passes
// and whole 256-row tiles of the wide f16 pass (wv_bf_h16w_kernel<.., 128>)
inline uint64_t align_rows(uint64_t n) { return (n + 255) / 256 * 256; }

struct wv_index {
    int dim = 0, dpad = 0, metric = 0;
    int ldx = 0;            // corpus row stride: D rounded up to 32 floats (whole 128-B lines, whole MFMA k-chunks) when D >= 32
    wv_config cfg{};
    uint64_t capacity = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // corpus
    DevBuf vecs;            // [capacity rounded to 128][ldx]
    // bf16 hi/lo image of vecs for the brute-force key pass (same bytes, in
    // the MFMA-native layout of split_hi_index), kept in step with every row write
    DevBuf xsplit;
    bool use_split = false;
    // f16 image of vecs for the f16 key pass (wv_h16.hip, the default for
    // D <= 128): f16(s_x x) in the layout of h16_index; h16_ex = max residual
    // norm |x - f16(s_x x) / s_x| over the rows (rounded up), both host-cached
    bool use_h16 = false;
    bool h16_wide = false;  // D > 128: wv_bf_h16w_kernel (both operands through LDS, 128-row tiles)
    int h16_ns = 0;
    float h16_sx = 0.f, h16_ex = 0.f;
    DevBuf ximg16, xns, qimg16, qres, qmax, qscale, tau, gtau, marg, allow_pad, ex_bits, gslot, seed_d, seed_id;
    // the f16 pass's block order (block_order), cached for its schedule
    DevBuf blk_order;
    std::vector<int> blk_order_host;
    uint64_t blk_key[4] = {0, 0, 0, 0};
    DevBuf qmax_part;       // per-block max |q_i| of the query-norm pass
    float maxnorm_host = 0.f;   // max |x| (rounded up), cached after every row write
    DevBuf xnorm;           // [capacity]
    DevBuf maxnorm;         // unsigned bits of max |x|
    std::vector<uint64_t> has_vec;   // host copy of uploaded rows
    uint64_t n_rows = 0;    // highest uploaded id + 1
    // graph
    bool has_graph = false;
    uint64_t gn = 0;
    int deg0 = 0, degU = 0, max_level = 0;
    uint64_t n_upper = 0, entrypoint = 0;
    std::vector<uint64_t> nil_host;   // graph nil nodes and ids >= gn, one bit per id
    DevBuf levels, layer0, upper_row, upper;
    // bitmaps
    std::vector<uint64_t> tomb_host;
    bool any_tomb = false, any_nil = false;   // any tombstone / nil node below gn
    uint64_t n_tomb = 0;                      // tombstones (sizes the side-register path's state)
    int last_side_rows = 0, last_side_xs = 0;  // the last side-register launch's LDS rows / spill capacity
    DevBuf side_vb, side_sp;                   // its visited bitmaps and spills (HBM scratch)
    DevBuf tomb;            // tombstones (HNSW eligibility)
    DevBuf excl;            // tombstone | nil node | no vector (flatSearch skips)
    uint64_t bm_words = 0;
    uint64_t clean_words = 0;   // leading exclusion words that are zero (refresh_bitmaps)
    bool bitmaps_dirty = true;
    // scratch
    DevBuf stage;           // contiguous host->device staging
    DevBuf q_in, q_norm, q_nrm2, q_scaled, cand_d, cand_id, fail, status, counters;
    // SearchByVectorDistance batches (wv_sbd.hip): targets, lists, counts, sort scratch
    DevBuf sbd_t, sbd_keys, sbd_tmp, sbd_cnt, sbd_off, sbd_q;
    void* sbd_scr = nullptr;
    size_t sbd_scr_cap = 0;
    DevBuf scan_d, scan_i, sort_d, sort_i, sort_tmp;
    DevBuf g_idx, g_q, g_allow, g_ids, g_d, g_n, g_cnt;
    DevBuf out_ids, out_d, out_n;
    DevBuf fail_thr, fb_idx, fb_d, fb_i, fb_n, fb_of;
    DevBuf ac_cnt, ac_off, rowidx;   // allow-list compaction
    // mutable-index sync: rows added since the last graph
    // upload are "pending"; those the graph does not hold are the delta set,
    // searched exactly beside the graph
    std::vector<uint64_t> pending_host;
    uint64_t delta_count = 0;
    DevBuf delta, dmask, dl_ids, dl_d, dl_n, dq_tmp;
    // graph construction scratch
    DevBuf b_tgt, b_ci, b_cd, b_cn, b_cnt0, b_cntu, b_rk, b_rn, b_rk2, b_rn2, b_uk, b_ul, b_uo, b_nr, b_tmp;
    // product quantization: h.pq / h.compressed
    // (compress.go:39-89).  Codes live on the device as u8 (ks <= 256) or u16
    // per segment, rows padded to whole words; has_code marks rows encoded.
    int pq_m = 0, pq_ks = 0, pq_ds = 0, pq_encoder = 0;
    bool pq_set = false, pq_on = false, pq_use_bits = false;
    uint64_t pq_stride = 0;
    std::vector<uint64_t> has_code;
    DevBuf pq_cent, pq_codes;
    DevBuf pk_key, pk_dist, pk_val, pk_skey, pk_sval, pk_off;
    // stats of the last batch: host-side counts plus device accumulators
    // (stat_acc: distance evaluations, expansions, device-resolved
    // fallbacks), read -- after a sync -- only when the stats are asked for
    uint64_t last_dist = 0, last_exp = 0, last_fallbacks = 0;
    DevBuf stat_acc;
    hipStream_t stat_stream = nullptr;
    // device-resolved certificate fallback (wv_launch_fbd): failed-query list
    // and count, survivors, overflow flags, full-scan slots
    DevBuf fbd_list, fbd_nf, fbd_over, fbd_cd, fbd_ci, fbd_cn, fbd_scr;
    // ordering of work on a caller's stream (wv_search_batch_device) against
    // the index's own stream: the call waits for ix->stream, and ix->stream
    // then waits for the call, so the scratch and state buffers the call reads
    // are never rewritten by a later call while it is still queued
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    hipEvent_t ev_null = nullptr;   // a NULL-stream call: the legacy default stream's work so far
    // optional kernel timing (hipEvents on the launch stream): each batch
    // records into its own event set (pairs 0-1 key pass, 2-3 finalize, 4-5
    // HNSW, 6-7 seed pass); the sets are read -- after a sync -- only when the
    // times are asked for, so timing adds no host round trip per batch
    bool timing = false;
    hipEvent_t* ev = nullptr;                    // the current batch's set
    std::vector<std::array<hipEvent_t, 8>> ev_pool;
    std::vector<uint8_t> ev_mask;                // pairs recorded per set
    size_t ev_used = 0;                          // sets recorded since the last read
    float t_mfma = 0.f, t_fin = 0.f, t_hnsw = 0.f, t_pre = 0.f;
    int n_cus = 256;
    // brute-force workgroups per launch: a whole number of resident waves of
    // workgroups (CUs x 2 per CU x WV_BF_ROUNDS)
    int bf_blocks = 512;
    // host staging of wv_search_batch: pinned slots, so a batch's copies are
    // asynchronous and the index mutex is released before the caller waits --
    // the next batch (another batcher worker) is staged and queued while this
    // one runs, and the GPU does not idle between batches
    struct HostSlot {
        void* pin = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;
        bool busy = false;
    };
    std::mutex slot_mu;
    std::condition_variable slot_cv;
    std::array<HostSlot, 3> slots;
    DevBuf allow_keep;   // per-query allow lists of an AUTO batch (the dispatch gathers into g_allow)
    // f16 key pass over a compacted shared allow list: the rows' image,
    // their |x|^2 and the scan's exclusion bits (the last tile's padding)
    DevBuf cimg16, cxnorm, cexcl;
};

namespace {

int refresh_bitmaps(wv_index* ix) {
    if (!ix->bitmaps_dirty) return WV_OK;
    const uint64_t words = ix->bm_words;
    std::vector<uint64_t> ex(words, 0);
    for (uint64_t w = 0; w < words; ++w) {
        uint64_t v = ~ix->has_vec[w];
        // compressed: a node whose code is missing is skipped like a deleted
        // one (distanceToByteNode, search.go:403-418)
        if (ix->pq_on) v |= ~ix->has_code[w];
        if (w < ix->tomb_host.size()) v |= ix->tomb_host[w];
        ex[w] = v;
    }
    std::vector<uint64_t> dl(words, 0);
    uint64_t dcount = 0;
    if (ix->has_graph) {
        // a nil node is skipped by flatSearch (flat_search.go:29-40) unless
        // it was added after the graph snapshot: then it is live (delta)
        for (uint64_t w = 0; w < words; ++w) {
            const uint64_t nil = ix->nil_host[w], pend = ix->pending_host[w];
            dl[w] = nil & pend & ix->has_vec[w] & ~ex[w];
            ex[w] |= nil & ~pend;
            dcount += (uint64_t)__builtin_popcountll(dl[w]);
        }
    }
    ix->delta_count = dcount;
    // the clean prefix: words (64-row tiles of the f16 pass) before the first
    // excluded row, which the key pass need not test
    ix->clean_words = 0;
    while (ix->clean_words < words && ex[ix->clean_words] == 0) ix->clean_words++;
    if (dcount) {
        HIP_TRY(ix->delta.ensure(words * 8));
        HIP_TRY(hipMemcpyAsync(ix->delta.p, dl.data(), words * 8, hipMemcpyHostToDevice, ix->stream));
    }
    std::vector<uint64_t> tb(words, 0);
    for (uint64_t w = 0; w < words && w < ix->tomb_host.size(); ++w) tb[w] = ix->tomb_host[w];
    HIP_TRY(hipMemcpyAsync(ix->excl.p, ex.data(), words * 8, hipMemcpyHostToDevice, ix->stream));
    HIP_TRY(hipMemcpyAsync(ix->tomb.p, tb.data(), words * 8, hipMemcpyHostToDevice, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    ix->bitmaps_dirty = false;
    return WV_OK;
}

int search_time_ef(const wv_config& c, int k) {
    int ef = (int)c.ef;
    if (ef < 1) {
        ef = k * (int)c.dynamic_ef_factor;
        if (ef > (int)c.dynamic_ef_max) ef = (int)c.dynamic_ef_max;
        else if (ef < (int)c.dynamic_ef_min) ef = (int)c.dynamic_ef_min;
        if (k > ef) ef = k;
        return ef;
    }
    if (ef < k) ef = k;
    return ef;
}

// Exact scan + stable radix sort, one query at a time (large k and certificate
// fallbacks).  q: device query (normalized if cosine).
int exact_full(wv_index* ix, const float* d_q, int k, const uint64_t* d_allow, uint64_t allow_nbits,
               uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s) {
    const uint64_t N = ix->n_rows;
    if (N == 0) {
        HIP_TRY(hipMemsetAsync(d_out_n, 0, sizeof(int32_t), s));
        return WV_OK;
    }
    HIP_TRY(ix->scan_d.ensure(N * 4));
    HIP_TRY(ix->scan_i.ensure(N * 4));
    HIP_TRY(ix->sort_d.ensure(N * 4));
    HIP_TRY(ix->sort_i.ensure(N * 4));
    wv::ScanParams sp{};
    sp.X = ix->vecs.as<float>();
    sp.q = d_q;
    sp.tomb = ix->excl.as<uint64_t>();
    sp.tomb_nbits = ix->capacity;
    sp.allow = d_allow;
    sp.allow_nbits = allow_nbits;
    sp.N = N;
    sp.D = ix->dim;
    sp.ldx = ix->ldx;
    sp.metric = ix->metric;
    sp.dist = ix->scan_d.as<float>();
    sp.ids = ix->scan_i.as<uint32_t>();
    HIP_TRY(wv_launch_exact_scan(&sp, s));
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, ix->scan_d.as<float>(), ix->sort_d.as<float>(),
                                               ix->scan_i.as<uint32_t>(), ix->sort_i.as<uint32_t>(), (int)N, 0, 32,
                                               s));
    HIP_TRY(ix->sort_tmp.ensure(tmp));
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(ix->sort_tmp.p, tmp, ix->scan_d.as<float>(), ix->sort_d.as<float>(),
                                               ix->scan_i.as<uint32_t>(), ix->sort_i.as<uint32_t>(), (int)N, 0, 32,
                                               s));
    hipLaunchKernelGGL(copy_topk_kernel, dim3(1), dim3(256), 0, s, ix->sort_d.as<float>(), ix->sort_i.as<uint32_t>(),
                       N, k, ix->cfg.id_base, d_out_ids, d_out_d, d_out_n);
    HIP_TRY(hipGetLastError());
    return WV_OK;
}

__global__ void allowed_count_kernel(const uint64_t* allow, uint64_t allow_words, const uint64_t* excl, uint64_t N,
                                     uint32_t* cnt) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t words = (N + 63) / 64;
    if (w >= words) return;
    uint64_t b = w < allow_words ? allow[w] & ~excl[w] : 0ull;
    if (w == words - 1 && (N & 63)) b &= (1ull << (N & 63)) - 1;
    cnt[w] = (uint32_t)__popcll(b);
}

__global__ void allowed_scatter_kernel(const uint64_t* allow, uint64_t allow_words, const uint64_t* excl, uint64_t N,
                                       const uint32_t* off, uint32_t* rowidx) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t words = (N + 63) / 64;
    if (w >= words) return;
    uint64_t b = w < allow_words ? allow[w] & ~excl[w] : 0ull;
    if (w == words - 1 && (N & 63)) b &= (1ull << (N & 63)) - 1;
    uint32_t o = off[w];
    while (b) {
        rowidx[o++] = (uint32_t)(w * 64 + __builtin_ctzll(b));
        b &= b - 1;
    }
}

__global__ void pad_rowidx_kernel(uint32_t* rowidx, uint64_t from, uint64_t to, const uint32_t* n_dev) {
    if (n_dev) {   // (the device's count: pad it to a whole tile)
        from = *n_dev;
        to = (from + wv::HW_BN - 1) / wv::HW_BN * wv::HW_BN;
    }
    const uint64_t i = from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < to) rowidx[i] = 0;   // padded tile rows read row 0 and are masked by the row count
}

// Ascending list of the rows a shared allow list keeps (allowed, not excluded,
// < N) into ix->rowidx, padded to whole tiles; *n_ok = its length.
// The f16 pass runs over a shared allow list's gathered rows when gathering
// costs less than masking the rest of the corpus: a gathered row moves ~6 D
// bytes once, a masked row costs the pass ~nq x D of MFMA work (measured at
// 10M x 768: 0.9 ns per gathered row, 1.6 ns per scanned row per 1000
// queries) and at least one read of its 2 D-byte image, so compacting pays
// below n_ok / N = max(1/3, nq / (nq + 560)) -- 64 % at configs[3]'s 1000
// queries (round 4's fixed rule, 50 %, left the 50 % leg a coin flip).
static bool worth_compacting(uint64_t n_ok, uint64_t N, int nq) {
    const double f = std::max(1.0 / 3.0, (double)nq / ((double)nq + 560.0));
    return (double)n_ok < (double)N * f;
}

int compact_allowed(wv_index* ix, const uint64_t* d_allow, uint64_t allow_nbits, uint64_t N, uint64_t* n_ok,
                    hipStream_t s, bool always = false, int nq = 1) {
    const uint64_t words = (N + 63) / 64;
    const uint64_t allow_words = (allow_nbits + 63) / 64;
    HIP_TRY(ix->ac_cnt.ensure((words + 1) * 4));
    HIP_TRY(ix->ac_off.ensure((words + 1) * 4));
    const unsigned blocks = (unsigned)((words + 255) / 256);
    hipLaunchKernelGGL(allowed_count_kernel, dim3(blocks), dim3(256), 0, s, d_allow, allow_words,
                       ix->excl.as<uint64_t>(), N, ix->ac_cnt.as<uint32_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemsetAsync(ix->ac_cnt.as<uint32_t>() + words, 0, 4, s));
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, ix->ac_cnt.as<uint32_t>(), ix->ac_off.as<uint32_t>(),
                                             (int)(words + 1), s));
    HIP_TRY(ix->sort_tmp.ensure(tmp));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ix->sort_tmp.p, tmp, ix->ac_cnt.as<uint32_t>(), ix->ac_off.as<uint32_t>(),
                                             (int)(words + 1), s));
    uint32_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, ix->ac_off.as<uint32_t>() + words, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_ok = total;
    // (the row list also serves the fp32 pass, which compacts below 1/2)
    if (total == 0 || (!worth_compacting(total, N, nq) && 2 * (uint64_t)total >= N && !always)) return WV_OK;
    // (whole 256-row tiles: the wide-D pass reads the list per tile)
    const uint64_t padded = (total + wv::HW_BN - 1) / wv::HW_BN * wv::HW_BN;
    HIP_TRY(ix->rowidx.ensure(padded * 4));
    hipLaunchKernelGGL(allowed_scatter_kernel, dim3(blocks), dim3(256), 0, s, d_allow, allow_words,
                       ix->excl.as<uint64_t>(), N, ix->ac_off.as<uint32_t>(), ix->rowidx.as<uint32_t>());
    HIP_TRY(hipGetLastError());
    if (padded > total)
        hipLaunchKernelGGL(pad_rowidx_kernel, dim3(1), dim3(256), 0, s, ix->rowidx.as<uint32_t>(), (uint64_t)total,
                           padded, nullptr);
    HIP_TRY(hipGetLastError());
    return WV_OK;
}

// The same list without reading its length back: ix->rowidx holds it, padded
// to whole tiles, and *n_dev (device memory) its length, which the compacted
// f16 wide-D pass reads itself (H16Params.n_dev) -- no host round trip
// between the allow list and the scan.
int compact_allowed_dev(wv_index* ix, const uint64_t* d_allow, uint64_t allow_nbits, uint64_t N, const uint32_t** n_dev,
                        hipStream_t s) {
    const uint64_t words = (N + 63) / 64;
    const uint64_t allow_words = (allow_nbits + 63) / 64;
    HIP_TRY(ix->ac_cnt.ensure((words + 1) * 4));
    HIP_TRY(ix->ac_off.ensure((words + 1) * 4));
    const unsigned blocks = (unsigned)((words + 255) / 256);
    hipLaunchKernelGGL(allowed_count_kernel, dim3(blocks), dim3(256), 0, s, d_allow, allow_words,
                       ix->excl.as<uint64_t>(), N, ix->ac_cnt.as<uint32_t>());
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemsetAsync(ix->ac_cnt.as<uint32_t>() + words, 0, 4, s));
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, ix->ac_cnt.as<uint32_t>(), ix->ac_off.as<uint32_t>(),
                                             (int)(words + 1), s));
    HIP_TRY(ix->sort_tmp.ensure(tmp));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ix->sort_tmp.p, tmp, ix->ac_cnt.as<uint32_t>(), ix->ac_off.as<uint32_t>(),
                                             (int)(words + 1), s));
    const uint64_t padded = (N + wv::HW_BN - 1) / wv::HW_BN * wv::HW_BN;
    HIP_TRY(ix->rowidx.ensure(padded * 4));
    hipLaunchKernelGGL(allowed_scatter_kernel, dim3(blocks), dim3(256), 0, s, d_allow, allow_words,
                       ix->excl.as<uint64_t>(), N, ix->ac_off.as<uint32_t>(), ix->rowidx.as<uint32_t>());
    HIP_TRY(hipGetLastError());
    *n_dev = ix->ac_off.as<uint32_t>() + words;
    hipLaunchKernelGGL(pad_rowidx_kernel, dim3(1), dim3(256), 0, s, ix->rowidx.as<uint32_t>(), 0ull, 0ull, *n_dev);
    HIP_TRY(hipGetLastError());
    return WV_OK;
}

// Brute force (flatSearch semantics) over a device batch of prepared queries.
// d_rowmask (nullable, with per-query allow lists only): a shared bitmap that
// contains every row any query may return (the delta set of wv_index_add);
// its rows are compacted and each query's own list is tested per row.
int run_pq_flat(wv_index* ix, const float* d_q, int nq, int k, const uint64_t* d_allow, uint64_t allow_nbits,
                uint64_t allow_stride, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s,
                const uint64_t* d_rowmask, uint64_t rowmask_nbits);

// f16 key pass (wv_h16.hip) over the whole corpus, optionally masked by a
// shared allow list: query image + scale, an optional seed pre-pass over every
// H_SAMPLE-th tile (its finalize yields per-query thresholds), the main pass
// seeded with them, and the certifying finalize.  Appends uncertified queries
// to `fails` (read back from the device).
// rowidx (nullable): the ascending row list of a compacted shared allow list
// (compact_allowed) -- the pass then runs over an f16 image of just those N
// rows (gathered here) and the candidate ids are mapped back to rows before
// the finalize; d_allow is then already applied
// Block order of an f16 pass: the blocks sorted by the corpus offset of their
// first tile, read by the kernels at their XCD-contiguous position (locality
// bit 1), so that each XCD runs the blocks of every query block over the same
// part of the corpus at the same time -- a tile then comes into that XCD's L2
// once per pass instead of once per query block.  nullptr: the identity
// (a single query block).
// rotated: the tiles of query block qb are rotated by qb ntiles mod U (the
// D <= 128 pass's locality bit 2), so a block's first tile is (slot U) mod ntiles.
int block_order(wv_index* ix, uint64_t nqb, const wv::BfSchedule& sch, hipStream_t s, const int** out,
                bool rotated = false) {
    *out = nullptr;
    if (nqb < 2 || sch.n_blocks < 16) return WV_OK;
    const uint64_t key[4] = {nqb, sch.ntiles, sch.units_per_block, rotated ? 1u : 0u};
    if (!std::equal(key, key + 4, ix->blk_key)) {
        const int nb = sch.n_blocks;
        const uint64_t U = sch.units_per_block, nt = sch.ntiles;
        auto first_tile = [&](int lb) -> uint64_t {
            if (!rotated) return (uint64_t)lb * U % nt;
            const uint64_t qb = (uint64_t)lb * U / nt;
            return ((uint64_t)lb - (uint64_t)wv::bf_first_block(qb, nt, U)) * U % nt;
        };
        std::vector<int>& ord = ix->blk_order_host;
        ord.resize(nb);
        for (int i = 0; i < nb; ++i) ord[i] = i;
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return first_tile(a) < first_tile(b); });
        HIP_TRY(ix->blk_order.ensure((size_t)nb * 4));
        HIP_TRY(hipMemcpyAsync(ix->blk_order.p, ord.data(), (size_t)nb * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));   // (pageable source; a later schedule rewrites it)
        std::copy(key, key + 4, ix->blk_key);
    }
    *out = ix->blk_order.as<int>();
    return WV_OK;
}

int run_h16(wv_index* ix, const float* d_q, int nq, int k, const uint64_t* d_allow, uint64_t allow_nbits, uint64_t N,
            uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s, std::vector<int32_t>& fails,
            const uint32_t* rowidx = nullptr, const uint32_t* n_dev = nullptr) {
    const int ns = ix->h16_ns;
    const bool wd = ix->h16_wide;   // D > 128: the wide-D kernel
    // D <= 128: 8-wave (512-query) workgroups, one per CU; D > 128: 256-row
    // tiles x 256-query blocks, one workgroup per CU
    const int wg_per_cu = 1;
    const int tile_rows = wd ? wv::HW_BN : wv::H_BN, bq = wd ? wv::HW_BQ : 512;
    // seed minima per query and slot; lists per query and slot, entries per list
    const int seed_prod = wd ? wv::HW_PROD : wv::H_PROD;
    const int prod = seed_prod;
    const int kp = wv::BF_KP;
    const uint64_t ntl = (N + tile_rows - 1) / tile_rows;
    const uint64_t words = ntl * (uint64_t)(tile_rows / 64);   // allow words the kernel reads
    const uint64_t* allow = d_allow;
    if (d_allow && (allow_nbits + 63) / 64 < words) {
        HIP_TRY(ix->allow_pad.ensure(words * 8));
        HIP_TRY(hipMemsetAsync(ix->allow_pad.p, 0, words * 8, s));
        if (allow_nbits)
            HIP_TRY(hipMemcpyAsync(ix->allow_pad.p, d_allow, (allow_nbits + 63) / 64 * 8, hipMemcpyDeviceToDevice, s));
        allow = ix->allow_pad.as<uint64_t>();
    }
    const int nqb = (nq + bq - 1) / bq;
    const size_t qbytes = (size_t)nqb * bq * ns * 16 * 2;
    HIP_TRY(ix->qimg16.ensure(qbytes));
    HIP_TRY(ix->qres.ensure((size_t)nq * 4));
    HIP_TRY(ix->tau.ensure((size_t)nq * 4));
    HIP_TRY(ix->gtau.ensure((size_t)nq * 4));
    HIP_TRY(ix->q_nrm2.ensure((size_t)nq * 4));
    HIP_TRY(ix->fail.ensure((size_t)nq * 4));
    HIP_TRY(ix->fail_thr.ensure((size_t)nq * 4));
    // |q|^2 and, in the same pass, the batch's max |q_i|; B = f16(s_q b),
    // b = -2q (L2) or -q, s_q from max |b|
    const float bsign = ix->metric == WV_L2_SQUARED ? -2.f : -1.f;
    HIP_TRY(ix->qmax_part.ensure((size_t)((nq + 3) / 4) * 4));
    HIP_TRY(wv_launch_qnorm(d_q, nq, ix->dim, ix->dpad, ix->metric, ix->q_nrm2.as<float>(), ix->qmax_part.as<float>(),
                            s));
    HIP_TRY(hipMemsetAsync(ix->qimg16.p, 0, qbytes, s));
    HIP_TRY(wv_launch_h16_qscale(ix->qmax_part.as<float>(), (nq + 3) / 4, ix->qmax.as<unsigned int>(), bsign,
                                 ix->qscale.as<float>(), s));
    HIP_TRY(wv_launch_h16_rows(d_q, ix->dpad, nullptr, nq, ix->dim, ns, bsign, 1.f, ix->qmax.as<unsigned int>(),
                               ix->qimg16.p, 0, nullptr, ix->qres.as<float>(), 0, s));
    const void* ximg = ix->ximg16.p;
    const float* xnorm = ix->xnorm.as<float>();
    const uint64_t* excl = ix->excl.as<uint64_t>();
    if (rowidx) {
        // the allowed rows' image in list order (whole tiles, zero padded),
        // their |x|^2, and exclusion bits set only past N
        const uint64_t rows = ntl * tile_rows, ew = rows / 64 + 2;
        HIP_TRY(ix->cxnorm.ensure(rows * 4));
        HIP_TRY(ix->cexcl.ensure(ew * 8));
        HIP_TRY(hipMemsetAsync(ix->cxnorm.p, 0, rows * 4, s));
        if (!wd) {   // (D > 128: the pass reads the row-major image through the list itself)
            const size_t ib = rows * (size_t)ns * 16 * 2;
            HIP_TRY(ix->cimg16.ensure(ib));
            HIP_TRY(wv_launch_h16_rows_gather(ix->vecs.as<float>(), ix->ldx, rowidx, N, rows, ix->dim, ns, ix->h16_sx,
                                              ix->cimg16.p, s));
            ximg = ix->cimg16.p;
        }
        HIP_TRY(wv_launch_h16_compact_aux(ix->xnorm.as<float>(), rowidx, N, n_dev, ix->cxnorm.as<float>(),
                                          ix->cexcl.as<uint64_t>(), ew, s));
        xnorm = ix->cxnorm.as<float>();
        excl = ix->cexcl.as<uint64_t>();
        allow = nullptr;
    }
    if (ix->metric == WV_L2_SQUARED)
        HIP_TRY(wv_launch_h16_xns(xnorm, ntl * tile_rows, ix->h16_sx, ix->qscale.as<float>(), ix->xns.as<float>(), s));
    wv::H16Params hp{};
    hp.X = ximg;
    hp.rowidx = wd ? rowidx : nullptr;
    hp.Q = ix->qimg16.p;
    hp.xns = ix->xns.as<float>();
    hp.excl = excl;
    hp.allow = allow;
    hp.qscale = ix->qscale.as<float>();
    hp.sx = ix->h16_sx;
    hp.N = N;
    hp.nq = nq;
    hp.metric = ix->metric;
    hp.n_qblocks = nqb;
    hp.wide_rows = 128;
    // 64-row tiles the pass need not mask: every row present and eligible
    // (no allow list; a compacted scan: the rows below N)
    hp.clean_tiles = wd ? 0 : rowidx ? N / wv::H_BN : allow ? 0 : std::min<uint64_t>(ix->clean_words, N / wv::H_BN);
    hp.locality = 1;   // XCD-contiguous workgroup ids
    wv::BfFinParams fp{};
    fp.X = ix->vecs.as<float>();
    fp.Q = d_q;
    fp.qnorm = ix->q_nrm2.as<float>();
    fp.xnorm_max = ix->maxnorm_host;
    fp.nq = nq;
    fp.D = ix->dim;
    fp.ldx = ix->ldx;
    fp.ldq = ix->dpad;
    fp.metric = ix->metric;
    fp.k = k;
    fp.id_base = ix->cfg.id_base;
    fp.out_ids = d_out_ids;
    fp.out_d = d_out_d;
    fp.out_n = d_out_n;
    fp.fail = ix->fail.as<int32_t>();
    fp.fail_thr = ix->fail_thr.as<float>();
    fp.bq = bq;
    fp.prod = prod;
    fp.kp = kp;
    fp.h16 = 1;
    hp.ns = ns;
    fp.qscale = ix->qscale.as<float>();
    fp.sx = ix->h16_sx;
    fp.ex_max = ix->h16_ex;
    fp.qres = ix->qres.as<float>();
    // seed pre-pass: the k-th exact distance over every H_SAMPLE-th tile bounds
    // each query's true k-th distance, hence the keys worth keeping
    // k > FIN_KF (the wide finalize): at least k slots per query block, i.e.
    // >= 2k lists of BF_KP per query, so that no list is likely to hold more
    // than BF_KP of the top k (which would leave its tail below the k-th key
    // and fail the certificate); the seed pass needs >= k minima likewise
    const bool wide = k > wv::FIN_KF;
    auto target = [&](uint64_t tiles) {
        uint64_t t = (uint64_t)ix->n_cus * wg_per_cu;
        if (wide) t = std::max<uint64_t>(t, (uint64_t)nqb * std::min<uint64_t>(tiles, (uint64_t)k + 2));
        return (int)std::min<uint64_t>(t, 1u << 30);
    };
    int sample = wv::H_SAMPLE;   // (WV_H16_SAMPLE: the seed's tile stride, for measurements)
    if (const char* e = std::getenv("WV_H16_SAMPLE")) sample = std::max(1, std::atoi(e));
    const bool seed = !wd && ntl >= 64 * (uint64_t)sample && !std::getenv("WV_H16_NO_SEED");
    // The seed pre-pass over 1 / sample of the tiles.  List mode
    // (WV_H16_SEED_LISTS, where its lists fit the seed kernel's one-wave
    // sort; measured slower, profiles/r06/h16_seed_list_mode.log): the
    // pre-pass scans the corpus's last nts tiles with full lists, the seed
    // kernel takes the thresholds from them and hands their 2 BF_KP smallest
    // to the finalize as one more slot, and the main pass scans only the
    // other tiles -- no tile is scanned twice.  Otherwise (minima mode) it
    // scans every sample-th tile keeping minima, and the main pass all tiles.
    const uint64_t nts = seed ? (ntl + sample - 1) / sample : 0;
    wv::BfSchedule ss{};
    if (seed) ss = wv::bf_schedule(nq, nts * wv::H_BN, target(nts), bq, wv::H_BN);
    const bool seed_lists = seed && !wide && !n_dev && k <= 64 &&
                            (uint64_t)ss.n_slots * wv::H_PROD * wv::BF_KP <= 256 && std::getenv("WV_H16_SEED_LISTS");
    const uint64_t ntl_main = seed_lists ? ntl - nts : ntl;
    // the wide pass: query blocks cut at the same tile offsets where that
    // costs no work (bf_schedule_aligned)
    wv::BfSchedule sch{};
    if (n_dev) {
        // a device-counted list (N its bound): S slots per query block, the
        // kernel sizes their runs (H16Params.n_dev); finalize and remap see
        // S one-tile slots, which index the lists the same way
        if (!wd || wide) return fail(WV_ESTATE, "run_h16: device-counted rows need the wide-D pass");
        const int S = std::max(1, target(ntl) / nqb);
        sch.bq = bq;
        sch.ntiles = (uint64_t)S;
        sch.units_per_block = 1;
        sch.n_blocks = nqb * S;
        sch.n_slots = S + 1;
    }
    if (wd && !wide && sch.n_blocks == 0) sch = wv::bf_schedule_aligned(nq, N, target(ntl), bq, tile_rows, false);
    if (sch.n_blocks == 0)
        sch = wv::bf_schedule(nq, seed_lists ? ntl_main * tile_rows : N, target(ntl_main), bq, tile_rows);
    if (wide && (uint64_t)sch.n_slots * prod * kp > (uint64_t)wv::FINW_NE)
        return fail(WV_ESTATE, "run_h16: too many lists for the wide finalize");
    // list slots per query: the main pass's, + the seed's slot (list mode)
    const int out_slots = sch.n_slots + (seed_lists ? 1 : 0);
    HIP_TRY(ix->cand_d.ensure((size_t)nq * out_slots * prod * kp * 4));
    HIP_TRY(ix->cand_id.ensure((size_t)nq * out_slots * prod * kp * 4));
    // a seed pre-pass: minima over every stride-th tile -> thresholds (tau)
    auto seed_minima = [&](int stride) -> int {
        const uint64_t nt = (ntl + stride - 1) / stride;
        const wv::BfSchedule ms = wv::bf_schedule(nq, nt * wv::H_BN, target(nt), bq, wv::H_BN);
        HIP_TRY(ix->cand_d.ensure((size_t)nq * std::max(ms.n_slots * seed_prod, out_slots * prod * kp) * 4));
        hp.ntiles = ms.ntiles;
        hp.ntiles_real = ms.ntiles;
        hp.units_per_block = ms.units_per_block;
        hp.n_slots = ms.n_slots;
        hp.tile_stride = stride;
        hp.tile_base = 0;
        hp.tau = nullptr;
        hp.out_d = ix->cand_d.as<float>();
        hp.out_id = nullptr;
        HIP_TRY(wv_launch_bf_h16(&hp, ns, 1, s));
        wv::H16SeedParams sp{};
        sp.minima = ix->cand_d.as<float>();
        sp.n_slots = ms.n_slots;
        sp.ntiles = ms.ntiles;
        sp.units_per_block = ms.units_per_block;
        sp.nq = nq;
        sp.k = k;
        sp.metric = ix->metric;
        sp.D = ix->dim;
        sp.qscale = ix->qscale.as<float>();
        sp.sx = ix->h16_sx;
        sp.qnorm = ix->q_nrm2.as<float>();
        sp.xnorm_max = ix->maxnorm_host;
        sp.ex_max = ix->h16_ex;
        sp.qres = ix->qres.as<float>();
        sp.tau = ix->tau.as<float>();
        sp.gtau = ix->gtau.as<unsigned int>();
        sp.bq = bq;
        sp.prod = seed_prod;
        if (seed_lists) {
            // list mode: the list pass over the corpus's last nts tiles,
            // keys above the minima's thresholds dropped; its lists give
            // tighter thresholds (min with the minima's) and the finalize's
            // extra slot
            HIP_TRY(wv_launch_h16_seed(&sp, s));
            HIP_TRY(ix->seed_d.ensure((size_t)nq * ss.n_slots * prod * kp * 4));
            HIP_TRY(ix->seed_id.ensure((size_t)nq * ss.n_slots * prod * kp * 4));
            hp.ntiles = ss.ntiles;
            hp.ntiles_real = ss.ntiles;
            hp.units_per_block = ss.units_per_block;
            hp.n_slots = ss.n_slots;
            hp.tile_stride = 1;
            hp.tile_base = ntl_main;
            hp.tau = ix->tau.as<float>();
            hp.out_d = ix->seed_d.as<float>();
            hp.out_id = ix->seed_id.as<uint32_t>();
            HIP_TRY(wv_launch_bf_h16(&hp, ns, 0, s));
            hp.tile_base = 0;
            hp.tau = nullptr;
            sp.minima = ix->seed_d.as<float>();
            sp.ids = ix->seed_id.as<uint32_t>();
            sp.n_slots = ss.n_slots;
            sp.ntiles = ss.ntiles;
            sp.units_per_block = ss.units_per_block;
            sp.prod = prod * kp;
            sp.out_d = ix->cand_d.as<float>();
            sp.out_id = ix->cand_id.as<uint32_t>();
            sp.out_slots = out_slots;
            sp.out_ntiles = sch.ntiles;
            sp.out_upb = sch.units_per_block;
        }
        HIP_TRY(wv_launch_h16_seed(&sp, s));
        return WV_OK;
    };
    if (seed) {
        TREC(6);
        // (list mode: minima over every 4 sample-th tile for the list pass;
        // WV_H16_LIST_MULT: that factor, for measurements)
        int mult = 4;
        if (const char* e = std::getenv("WV_H16_LIST_MULT")) mult = std::max(1, std::atoi(e));
        if (int rc = seed_minima(seed_lists ? mult * sample : sample)) return rc;
        TREC(7);
    }
    hp.ntiles = sch.ntiles;
    hp.ntiles_real = ntl_main;
    hp.out_slots = seed_lists ? out_slots : 0;
    hp.units_per_block = sch.units_per_block;
    hp.n_slots = sch.n_slots;
    hp.n_dev = n_dev;
    hp.tile_stride = 1;
    hp.tau = nullptr;
    // the running threshold (k <= 2 BF_KP), started at the seed's
    if (!seed) HIP_TRY(hipMemsetAsync(ix->gtau.p, 0xFF, (size_t)nq * 4, s));
    hp.gtau = ix->gtau.as<unsigned int>();
    // (with the seed's threshold the running one only adds work: measured
    // 3.048 vs 3.092 ms per 1M x 10k key pass; without a seed -- corpora below
    // 64 * H_SAMPLE tiles -- it cuts the pass 4.13 -> 3.43 ms at 1M)
    // (the wide-D pass publishes from a lane pair's two lists: k <= 2 BF_KP)
    hp.kth = k <= (wd ? 2 * kp : prod * kp) && !seed && !std::getenv("WV_H16_NO_RUNNING")
                 ? k
                 : 0;
    // cross-slot threshold (32x32x16 pass, <= 32 list heads per query; on
    // unless WV_H16_XSLOT=0): 2.87-2.91 vs 2.98-3.00 ms per 1M x 10k key pass
    const char* xe = std::getenv("WV_H16_XSLOT");
    const bool xs_on = !xe || std::atoi(xe) != 0;
    if (xs_on && !wd && 2 * sch.n_slots <= 32 && k <= 2 * sch.n_slots) {
        const size_t gb = (size_t)nq * 2 * sch.n_slots * 4;
        HIP_TRY(ix->gslot.ensure(gb));
        HIP_TRY(hipMemsetAsync(ix->gslot.p, 0x7F, gb, s));   // 3.4e38: no head yet
        hp.gslot = ix->gslot.as<float>();
        hp.xslot = 1;
        hp.kth = k;
    }
    if (hp.kth) {
        HIP_TRY(ix->marg.ensure((size_t)nq * 4));
        HIP_TRY(wv_launch_h16_margin(ix->metric, ix->dim, ix->q_nrm2.as<float>(), ix->qres.as<float>(),
                                     ix->maxnorm_host, ix->h16_ex, ix->h16_sx, ix->qscale.as<float>(), nq,
                                     ix->marg.as<float>(), s));
        hp.marg = ix->marg.as<float>();
    }
    hp.out_d = ix->cand_d.as<float>();
    hp.out_id = ix->cand_id.as<uint32_t>();
    // the 8-wave D <= 128 pass on the flat schedule: tiles rotated per query
    // block (locality bit 2): 2.73-2.75 -> 2.66-2.68 ms per 1M x 10k pass,
    // L2-miss bytes 5.23 -> 0.66 GB
    const bool rotate = !wd && nqb >= 2 && sch.ntiles == ntl_main;
    if (rotate) hp.locality |= 2;
    if (int rc = block_order(ix, (uint64_t)nqb, sch, s, &hp.block_order, rotate)) return rc;
    TREC(0);
    HIP_TRY(wd ? wv_launch_bf_h16w(&hp, s) : wv_launch_bf_h16(&hp, ns, 0, s));
    TREC(1);
    // compacted scan: the candidate positions map to rows -- inside the
    // finalize for its FIN_KF selected entries, or (the wide finalize) all
    // of them first
    if (rowidx && wide)
        HIP_TRY(wv_launch_remap_ids(ix->cand_id.as<uint32_t>(), nq, sch.n_slots, prod * kp, bq, sch.ntiles,
                                    sch.units_per_block, rowidx, N, n_dev, s));
    if (rowidx && !wide) {
        fp.rowidx = rowidx;
        fp.rowidx_n = N;
        fp.rowidx_ndev = n_dev;
    }
    fp.cand_d = ix->cand_d.as<float>();
    fp.cand_id = ix->cand_id.as<uint32_t>();
    fp.n_slots = out_slots;
    fp.extra_slot = seed_lists ? 1 : 0;
    fp.ntiles = sch.ntiles;
    fp.units_per_block = sch.units_per_block;
    HIP_TRY(wv_launch_h16_gtau(ix->gtau.as<unsigned int>(), nq, ix->h16_sx, ix->qscale.as<float>(), ix->tau.as<float>(),
                               s));
    fp.tau_in = ix->tau.as<float>();
    TREC(2);
    HIP_TRY(wide ? wv_launch_bf_finalize_wide(&fp, s) : wv_launch_bf_finalize(&fp, s));
    TREC(3);
    (void)fails;   // uncertified queries are resolved on the device (queue_fbd)
    return WV_OK;
}

// Queue the device-resolved fallback for the queries whose flag in ix->fail
// is set (threshold ix->fail_thr): no host round trip (wv_bf.hip, fbd kernels).
int queue_fbd(wv_index* ix, const float* d_q, int nq, int k, const uint64_t* d_allow, uint64_t allow_nbits,
              uint64_t allow_stride, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s) {
    const uint64_t N = ix->n_rows;
    HIP_TRY(ix->fbd_list.ensure((size_t)nq * 4));
    HIP_TRY(ix->fbd_nf.ensure(16));
    HIP_TRY(ix->fbd_over.ensure((size_t)nq * 4));
    HIP_TRY(ix->fbd_cd.ensure((size_t)nq * wv::FB_CAP * 4));
    HIP_TRY(ix->fbd_ci.ensure((size_t)nq * wv::FB_CAP * 4));
    HIP_TRY(ix->fbd_cn.ensure((size_t)nq * 4));
    HIP_TRY(ix->fbd_scr.ensure((size_t)wv::FBD_SCR * std::max<uint64_t>(N, 1) * 4));
    HIP_TRY(ix->stat_acc.ensure(48));
    wv::FbParams bp{};
    bp.X = ix->vecs.as<float>();
    bp.Q = d_q;
    bp.qidx = ix->fbd_list.as<int32_t>();
    bp.thr = ix->fail_thr.as<float>();
    bp.tomb = ix->excl.as<uint64_t>();
    bp.tomb_nbits = ix->capacity;
    bp.allow = d_allow;
    bp.allow_nbits = allow_nbits;
    bp.allow_stride = allow_stride;
    bp.N = N;
    bp.nf = nq;
    bp.D = ix->dim;
    bp.ldx = ix->ldx;
    bp.ldq = ix->dpad;
    bp.metric = ix->metric;
    bp.k = k;
    bp.id_base = ix->cfg.id_base;
    bp.cand_d = ix->fbd_cd.as<float>();
    bp.cand_id = ix->fbd_ci.as<uint32_t>();
    bp.cand_n = ix->fbd_cn.as<uint32_t>();
    bp.out_ids = d_out_ids;
    bp.out_d = d_out_d;
    bp.out_n = d_out_n;
    bp.overflow = ix->fbd_over.as<int32_t>();
    bp.d_nf = ix->fbd_nf.as<int32_t>();
    bp.scratch = ix->fbd_scr.as<float>();
    bp.n_scr = wv::FBD_SCR;
    bp.fb_total = ix->stat_acc.as<unsigned long long>() + 2;
#ifdef WV_ABLATION_BUILD
    if (std::getenv("WV_ABLATE_NO_FALLBACK")) return WV_OK;   // kernel ablations only (tools/h16_ablate.sh)
#endif
    HIP_TRY(wv_launch_fbd(ix->fail.as<int32_t>(), nq, &bp, s));
    return WV_OK;
}

int run_exact(wv_index* ix, const float* d_q, int nq, int k, const uint64_t* d_allow, uint64_t allow_nbits,
              uint64_t allow_stride, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s,
              const uint64_t* d_rowmask = nullptr, uint64_t rowmask_nbits = 0) {
    if (ix->pq_on)   // flatSearch on a compressed index ranks by PQ distance (index.go:493-511)
        return run_pq_flat(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s,
                           d_rowmask, rowmask_nbits);
    const uint64_t N = ix->n_rows;
    if (N == 0 || nq == 0) {
        if (nq) HIP_TRY(hipMemsetAsync(d_out_n, 0, sizeof(int32_t) * nq, s));
        return WV_OK;
    }
    std::vector<int32_t> fails;
    // the f16 pass (whole corpus or a shared allow list) serves k up to
    // BF_WIDE_KMAX; the other key passes k up to BF_FAST_KMAX
    const bool h16_ok = ix->use_h16 && !allow_stride && !d_rowmask;
    // the key pass + finalize ran: fail_thr holds each failed query's bound
    const bool keyed = k <= wv::BF_FAST_KMAX || (h16_ok && k <= wv::BF_WIDE_KMAX);
    if (keyed) {
        // A shared allow list that keeps under half the corpus is compacted
        // into a row list first: the contraction then runs over |allow| rows
        // (the reference's flatSearch also walks only the allow list,
        // flat_search.go:25-58) instead of masking N.
        uint64_t n_scan = N;
        const uint32_t* d_rowidx = nullptr;
        const uint64_t* cmask = d_allow && !allow_stride ? d_allow : d_rowmask;
        const uint64_t cbits = d_allow && !allow_stride ? allow_nbits : rowmask_nbits;
        // The wide-D f16 pass (k <= FIN_KF) compacts every shared list with
        // no host round trip: its per-lane fill reads a compacted tile at the
        // cost of a contiguous one, so the list's length need not steer the
        // scan (WV_BF_SYNC_COMPACT=1: the read-back rule below, measurements)
        if (cmask && !d_rowmask && h16_ok && ix->h16_wide && k <= wv::FIN_KF && !std::getenv("WV_BF_SYNC_COMPACT") &&
            !std::getenv("WV_BF_NO_COMPACT")) {
            const uint32_t* n_dev = nullptr;
            const uint64_t n_bound = std::min<uint64_t>(N, cbits);
            if (n_bound == 0) {
                HIP_TRY(hipMemsetAsync(d_out_n, 0, sizeof(int32_t) * nq, s));
                return WV_OK;
            }
            if (int rc = compact_allowed_dev(ix, cmask, cbits, N, &n_dev, s)) return rc;
            std::vector<int32_t> none;
            if (int rc = run_h16(ix, d_q, nq, k, nullptr, 0, n_bound, d_out_ids, d_out_d, d_out_n, s, none,
                                 ix->rowidx.as<uint32_t>(), n_dev))
                return rc;
            return queue_fbd(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
        }
        if (cmask) {
            uint64_t n_ok = 0;
            int rc = compact_allowed(ix, cmask, cbits, N, &n_ok, s, d_rowmask != nullptr, nq);
            if (rc) return rc;
            if (n_ok == 0) {
                HIP_TRY(hipMemsetAsync(d_out_n, 0, sizeof(int32_t) * nq, s));
                return WV_OK;
            }
            // a list worth compacting (worth_compacting): the scan runs over
            // its rows -- on the f16 pass over their gathered image (h16_ok),
            // else (below 1/2 or 1/8) on the fp32 pass over the row list
            const bool compact = (worth_compacting(n_ok, N, nq) && !std::getenv("WV_BF_NO_COMPACT")) || d_rowmask;
            if (compact && h16_ok) {
                std::vector<int32_t> none;
                int rc2 = run_h16(ix, d_q, nq, k, nullptr, 0, n_ok, d_out_ids, d_out_d, d_out_n, s, none,
                                  ix->rowidx.as<uint32_t>());
                if (rc2) return rc2;
                return queue_fbd(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
            }
            // (no gathered f16 pass: the f16 pass masks the whole corpus
            // unless the list keeps under 1/8 of it)
            const uint64_t frac = ix->use_h16 && !allow_stride ? 8 : 2;
            if (((frac * n_ok < N && !std::getenv("WV_BF_NO_COMPACT")) || d_rowmask) && k <= wv::BF_FAST_KMAX) {
                n_scan = n_ok;
                d_rowidx = ix->rowidx.as<uint32_t>();
            }
        }
        if (ix->use_h16 && !d_rowidx && !allow_stride) {
            const uint64_t* sh = d_allow && !allow_stride ? d_allow : nullptr;
            int rc = run_h16(ix, d_q, nq, k, sh, allow_nbits, N, d_out_ids, d_out_d, d_out_n, s, fails);
            if (rc) return rc;
            return queue_fbd(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
        }
        // bf16x3 key pass on native images (whole-corpus or shared allow list
        // scans, opt-in WV_BF_SPLIT=1): 256-query blocks, one 512-thread
        // workgroup per CU, two waves per SIMD (wv_bf_split_kernel)
        const bool split = ix->use_split && !d_rowidx && !allow_stride;
        const int bq = split ? 2 * wv::BF_BQ : wv::BF_BQ;
        const int prod = wv::BF_PROD;
        const int n_qblocks = (nq + bq - 1) / bq;
        const wv::BfSchedule sch =
            wv::bf_schedule(nq, n_scan, bq == wv::BF_BQ ? ix->bf_blocks : ix->bf_blocks / 2, bq);
        const size_t n_lists = (size_t)sch.n_slots * prod;
        HIP_TRY(ix->cand_d.ensure((size_t)nq * n_lists * wv::BF_KP * 4));
        HIP_TRY(ix->cand_id.ensure((size_t)nq * n_lists * wv::BF_KP * 4));
        HIP_TRY(ix->q_nrm2.ensure((size_t)nq * 4));
        HIP_TRY(ix->fail.ensure((size_t)nq * 4));
        HIP_TRY(wv_launch_qnorm(d_q, nq, ix->dim, ix->dpad, ix->metric, ix->q_nrm2.as<float>(), nullptr, s));
        // B operand in whole bq-row query blocks, zero rows past nq: -2q
        // (L2) or -q, as fp32 rows or (split key pass: whole-corpus or shared
        // allow list scans) as the native bf16 hi/lo image
        const size_t nq_pad = (size_t)n_qblocks * bq;
        const int ldb = split ? ix->ldx : ix->dpad;
        const float bscale = ix->metric == WV_L2_SQUARED ? -2.f : -1.f;
        HIP_TRY(ix->q_scaled.ensure(nq_pad * ldb * 4));
        if (split) {
            HIP_TRY(wv_launch_split_rows(d_q, ix->dpad, nullptr, nq_pad, nq, ix->dim, bscale, ix->q_scaled.p, ldb, 0, s));
        } else {
            if (nq_pad > (size_t)nq)
                HIP_TRY(hipMemsetAsync(ix->q_scaled.as<float>() + (size_t)nq * ldb, 0, (nq_pad - nq) * ldb * 4, s));
            HIP_TRY(wv_launch_scale(d_q, ix->q_scaled.as<float>(), (uint64_t)nq * ix->dpad, bscale, s));
        }
        wv::BfParams bp{};
        bp.split = split ? 1 : 0;
        bp.bq = bq;
        bp.prod = prod;
        bp.locality = 3;   // XCD-contiguous workgroups, aligned tile rotation
        bp.X = split ? ix->xsplit.as<float>() : ix->vecs.as<float>();
        bp.Q = ix->q_scaled.as<float>();
        bp.xnorm = ix->xnorm.as<float>();
        bp.tomb = d_rowidx ? nullptr : ix->excl.as<uint64_t>();
        bp.tomb_nbits = ix->capacity;
        // compacted rows carry the shared list already; per-query lists are
        // still tested (per gathered row)
        bp.allow = d_rowidx && !allow_stride ? nullptr : d_allow;
        bp.allow_nbits = allow_nbits;
        bp.allow_stride = allow_stride;
        bp.rowidx = d_rowidx;
        bp.N = n_scan;
        bp.nq = nq;
        bp.D = ix->dim;
        bp.ldx = ix->ldx;
        bp.ldq = ldb;
        bp.metric = ix->metric;
        bp.n_qblocks = n_qblocks;
        bp.n_slots = sch.n_slots;
        bp.ntiles = sch.ntiles;
        bp.units_per_block = sch.units_per_block;
        bp.out_d = ix->cand_d.as<float>();
        bp.out_id = ix->cand_id.as<uint32_t>();
        TREC(0);
        HIP_TRY(wv_launch_bf_mfma(&bp, s));
        TREC(1);
        const float maxn = ix->maxnorm_host;   // cached at every row write
        wv::BfFinParams fp{};
        fp.X = ix->vecs.as<float>();
        fp.Q = d_q;
        fp.cand_d = ix->cand_d.as<float>();
        fp.cand_id = ix->cand_id.as<uint32_t>();
        fp.qnorm = ix->q_nrm2.as<float>();
        fp.xnorm_max = maxn;
        fp.n_slots = sch.n_slots;
        fp.ntiles = sch.ntiles;
        fp.units_per_block = sch.units_per_block;
        fp.nq = nq;
        fp.D = ix->dim;
        fp.ldx = ix->ldx;
        fp.ldq = ix->dpad;
        fp.metric = ix->metric;
        fp.k = k;
        fp.id_base = ix->cfg.id_base;
        fp.out_ids = d_out_ids;
        fp.out_d = d_out_d;
        fp.out_n = d_out_n;
        fp.fail = ix->fail.as<int32_t>();
        HIP_TRY(ix->fail_thr.ensure((size_t)nq * 4));
        fp.fail_thr = ix->fail_thr.as<float>();
        fp.split = bp.split;
        fp.bq = bq;
        fp.prod = prod;
        TREC(2);
        HIP_TRY(wv_launch_bf_finalize(&fp, s));
        TREC(3);
        return queue_fbd(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    } else {
        for (int i = 0; i < nq; ++i) fails.push_back(i);
    }
    ix->last_fallbacks += fails.size();
#ifdef WV_ABLATION_BUILD
    if (!fails.empty() && std::getenv("WV_ABLATE_NO_FALLBACK")) fails.clear();   // kernel ablations only
#endif
    if (!fails.empty() && keyed) {
        // batched threshold filter over the corpus for every failed query
        std::vector<int32_t> rest;
        for (size_t b0 = 0; b0 < fails.size(); b0 += 256) {
            const int nf = (int)std::min<size_t>(256, fails.size() - b0);
            HIP_TRY(ix->fb_idx.ensure((size_t)nf * 4));
            HIP_TRY(ix->fb_d.ensure((size_t)nf * wv::FB_CAP * 4));
            HIP_TRY(ix->fb_i.ensure((size_t)nf * wv::FB_CAP * 4));
            HIP_TRY(ix->fb_n.ensure((size_t)nf * 4));
            HIP_TRY(ix->fb_of.ensure((size_t)nf * 4));
            HIP_TRY(hipMemcpyAsync(ix->fb_idx.p, fails.data() + b0, 4 * (size_t)nf, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemsetAsync(ix->fb_n.p, 0, 4 * (size_t)nf, s));
            wv::FbParams bp{};
            bp.X = ix->vecs.as<float>();
            bp.Q = d_q;
            bp.qidx = ix->fb_idx.as<int32_t>();
            bp.thr = ix->fail_thr.as<float>();
            bp.tomb = ix->excl.as<uint64_t>();
            bp.tomb_nbits = ix->capacity;
            bp.allow = d_allow;
            bp.allow_nbits = allow_nbits;
            bp.allow_stride = allow_stride;
            bp.N = N;
            bp.nf = nf;
            bp.D = ix->dim;
            bp.ldx = ix->ldx;
            bp.ldq = ix->dpad;
            bp.metric = ix->metric;
            bp.k = k;
            bp.id_base = ix->cfg.id_base;
            bp.cand_d = ix->fb_d.as<float>();
            bp.cand_id = ix->fb_i.as<uint32_t>();
            bp.cand_n = ix->fb_n.as<uint32_t>();
            bp.out_ids = d_out_ids;
            bp.out_d = d_out_d;
            bp.out_n = d_out_n;
            bp.overflow = ix->fb_of.as<int32_t>();
            HIP_TRY(wv_launch_fb(&bp, s));
            std::vector<int32_t> of(nf);
            HIP_TRY(hipMemcpyAsync(of.data(), ix->fb_of.p, 4 * (size_t)nf, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            for (int i = 0; i < nf; ++i)
                if (of[i]) rest.push_back(fails[b0 + i]);
        }
        fails.swap(rest);   // survivors overflowed: full scan + sort below
    }
    for (int q : fails) {
        const uint64_t* al = d_allow ? d_allow + (allow_stride ? (uint64_t)q * allow_stride : 0) : nullptr;
        int rc = ix->pq_on ? run_pq_flat(ix, d_q + (size_t)q * ix->dpad, 1, k, al, allow_nbits, 0,
                                         d_out_ids + (size_t)q * k, d_out_d + (size_t)q * k, d_out_n + q, s, nullptr, 0)
                           : exact_full(ix, d_q + (size_t)q * ix->dpad, k, al, allow_nbits, d_out_ids + (size_t)q * k,
                                        d_out_d + (size_t)q * k, d_out_n + q, s);
        if (rc) return rc;
    }
    return WV_OK;
}

wv::PqParams pq_params(const wv_index* ix) {
    wv::PqParams pq{};
    pq.codes = ix->pq_codes.as<uint8_t>();
    pq.cent = ix->pq_cent.as<float>();
    pq.stride = ix->pq_stride;
    pq.m = ix->pq_m;
    pq.ks = ix->pq_ks;
    pq.ds = ix->pq_ds;
    pq.wide = ix->pq_ks > 256;
    return pq;
}

__global__ void iota_stride_kernel(int32_t* off, int n, int64_t stride) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) off[i] = (int32_t)(i * stride);
}

// flatSearch over PQ codes: the rows a shared allow list (or the delta mask)
// keeps are compacted, every (query, row) distance is computed from the codes
// and a stable segmented radix sort orders each query's row list by
// (dist, id); queries go in chunks of at most 2^26 (query, row) pairs.
int run_pq_flat(wv_index* ix, const float* d_q, int nq, int k, const uint64_t* d_allow, uint64_t allow_nbits,
                uint64_t allow_stride, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s,
                const uint64_t* d_rowmask, uint64_t rowmask_nbits) {
    const uint64_t N = ix->n_rows;
    if (N == 0 || nq == 0) {
        if (nq) HIP_TRY(hipMemsetAsync(d_out_n, 0, sizeof(int32_t) * nq, s));
        return WV_OK;
    }
    const uint64_t* cmask = d_allow && !allow_stride ? d_allow : d_rowmask;
    const uint64_t cbits = d_allow && !allow_stride ? allow_nbits : rowmask_nbits;
    uint64_t nr = N;
    const uint32_t* rows = nullptr;
    if (cmask) {
        int rc = compact_allowed(ix, cmask, cbits, N, &nr, s, true);
        if (rc) return rc;
        if (nr == 0) {
            HIP_TRY(hipMemsetAsync(d_out_n, 0, sizeof(int32_t) * nq, s));
            return WV_OK;
        }
        rows = ix->rowidx.as<uint32_t>();
    }
    const uint64_t cap = 1ull << 26;
    const int qc = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)nq, cap / nr));
    const uint64_t items = (uint64_t)qc * nr;
    if (items > (uint64_t)INT32_MAX) return fail(WV_EINVAL, "flat PQ search: too many rows per query");
    HIP_TRY(ix->pk_key.ensure(items * 4));
    HIP_TRY(ix->pk_dist.ensure(items * 4));
    HIP_TRY(ix->pk_val.ensure(items * 4));
    HIP_TRY(ix->pk_skey.ensure(items * 4));
    HIP_TRY(ix->pk_sval.ensure(items * 4));
    HIP_TRY(ix->pk_off.ensure(((size_t)qc + 1) * 4));
    wv::PqScanParams sp{};
    sp.pq = pq_params(ix);
    sp.Q = d_q;
    sp.rows = rows;
    sp.excl = ix->excl.as<uint64_t>();
    sp.excl_nbits = ix->capacity;
    sp.allow = allow_stride ? d_allow : nullptr;   // a shared list is compacted already
    sp.allow_nbits = allow_nbits;
    sp.allow_stride = allow_stride;
    sp.nr = nr;
    sp.ldq = ix->dpad;
    sp.metric = ix->metric;
    sp.key = ix->pk_key.as<float>();
    sp.dist = ix->pk_dist.as<float>();
    sp.val = ix->pk_val.as<uint32_t>();
    for (int q0 = 0; q0 < nq; q0 += qc) {
        const int nqc = std::min(qc, nq - q0);
        sp.q0 = q0;
        sp.nqc = nqc;
        HIP_TRY(wv_launch_pq_scan(&sp, s));
        hipLaunchKernelGGL(iota_stride_kernel, dim3((nqc + 256) / 256), dim3(256), 0, s, ix->pk_off.as<int32_t>(), nqc,
                           (int64_t)nr);
        HIP_TRY(hipGetLastError());
        const int n_items = (int)((uint64_t)nqc * nr);
        size_t tmp = 0;
        HIP_TRY(hipcub::DeviceSegmentedRadixSort::SortPairs(
            nullptr, tmp, ix->pk_key.as<float>(), ix->pk_skey.as<float>(), ix->pk_val.as<uint32_t>(),
            ix->pk_sval.as<uint32_t>(), n_items, nqc, ix->pk_off.as<int32_t>(), ix->pk_off.as<int32_t>() + 1, 0, 32, s));
        HIP_TRY(ix->sort_tmp.ensure(tmp));
        HIP_TRY(hipcub::DeviceSegmentedRadixSort::SortPairs(
            ix->sort_tmp.p, tmp, ix->pk_key.as<float>(), ix->pk_skey.as<float>(), ix->pk_val.as<uint32_t>(),
            ix->pk_sval.as<uint32_t>(), n_items, nqc, ix->pk_off.as<int32_t>(), ix->pk_off.as<int32_t>() + 1, 0, 32, s));
        HIP_TRY(wv_launch_pq_topk(ix->pk_skey.as<float>(), ix->pk_sval.as<uint32_t>(), ix->pk_dist.as<float>(), rows,
                                  nr, q0, nqc, k, ix->cfg.id_base, d_out_ids, d_out_d, d_out_n, s));
    }
    return WV_OK;
}

// Visited-cache size (2^vc_log2 16-bit slots) for a per-wave LDS budget, and
// the tag width that makes slot + tag identify ids below n_nodes exactly
// (HnswParams.vc_tbits <= 15; a graph past 2^(vc_log2 + 15) nodes gets more
// slots than the budget would give).
int choose_vc_log2(int per_wave_budget_words, int fixed_words, uint64_t n_nodes, int* tbits) {
    int l = 13;
    while (l > 8 && fixed_words + ((1 << l) + 1) / 2 > per_wave_budget_words) --l;
    int hb = 1;
    while (hb < 32 && (1ull << hb) < n_nodes) ++hb;
    if (hb - l > 15) l = hb - 15;
    *tbits = hb > l ? hb - l : 0;
    return l;
}

int run_hnsw(wv_index* ix, const float* d_q, int nq, int k, int ef, const uint64_t* d_allow, uint64_t allow_nbits,
             uint64_t allow_stride, uint64_t* d_out_ids, float* d_out_d, int32_t* d_out_n, hipStream_t s) {
    if (!ix->has_graph || ix->gn == 0) return fail(WV_ESTATE, "no graph uploaded");
    const int efc = std::max(64, (ef + 63) / 64 * 64);
    // Side candidates S (traversed but ineligible: search.go:282-298) and the
    // exact set of expanded side candidates exist only under a filter,
    // tombstones or nil nodes.  Without them the wave state shrinks and more
    // queries are in flight (the search is latency-bound on its gathers).  A
    // stray ineligible node still ends in the exact fallback (status bit 0),
    // never in a wrong answer.
    const bool filtered = d_allow != nullptr || ix->any_tomb || ix->any_nil;
    const int sc = filtered ? 256 : 0;
    const int xs_log2 = filtered ? 9 : 0;
    // register results (unfiltered, ef <= 256): the wave's LDS is the query,
    // the batch and the visited cache only
    const bool reg = !filtered && efc <= 256;
    const int fixed = reg ? wv_hnsw_reg_per_wave_words(ix->dpad, 0) - 1
                          : wv_hnsw_per_wave_words(ix->dpad, efc, sc, 0, xs_log2) - 1;
    // per-wave LDS budget: 20 KiB filtered (8 waves per CU), 12 KiB otherwise
    int wave_kb = filtered ? 20 : 12;
    if (const char* e = std::getenv("WV_HNSW_WAVE_KB")) wave_kb = std::max(4, std::atoi(e));
    const int budget = wave_kb * 1024 / 4;
    int vc_tbits = 0;
    const int vc_log2 = choose_vc_log2(budget, fixed, ix->gn, &vc_tbits);
    int per_wave = reg ? wv_hnsw_reg_per_wave_words(ix->dpad, vc_log2)
                       : wv_hnsw_per_wave_words(ix->dpad, efc, sc, vc_log2, xs_log2);
    per_wave = (per_wave + 3) & ~3;
    int wpb = 4;
    while (wpb > 1 && (size_t)wpb * per_wave * 4 > 160 * 1024) --wpb;
    if ((size_t)per_wave * 4 > 160 * 1024) return fail(WV_EINVAL, "hnsw LDS footprint too large");
    HIP_TRY(ix->status.ensure((size_t)nq * 4));
    HIP_TRY(ix->counters.ensure((size_t)nq * 8));
    wv::HnswParams hp{};
    hp.X = ix->vecs.as<float>();
    hp.levels = ix->levels.as<int8_t>();
    hp.layer0 = ix->layer0.as<uint32_t>();
    hp.upper_row = ix->upper_row.as<uint32_t>();
    hp.upper = ix->upper.as<uint32_t>();
    hp.tomb = ix->any_tomb ? ix->tomb.as<uint64_t>() : nullptr;
    hp.tomb_nbits = ix->capacity;
    hp.allow = d_allow;
    hp.allow_nbits = allow_nbits;
    hp.allow_stride = allow_stride;
    hp.Q = d_q;
    hp.N = ix->gn;
    hp.id_base = ix->cfg.id_base;
    hp.entrypoint = (uint32_t)ix->entrypoint;
    hp.D = ix->dim;
    hp.ldx = ix->ldx;
    hp.ldq = ix->dpad;
    hp.metric = ix->metric;
    hp.deg0 = ix->deg0;
    hp.degU = ix->degU;
    hp.max_level = ix->max_level;
    hp.upper_levels = ix->max_level;
    hp.nq = nq;
    hp.k = k;
    hp.ef = ef;
    hp.efc = efc;
    hp.sc = sc;
    hp.vc_log2 = vc_log2;
    hp.vc_tbits = vc_tbits;
    hp.xs_log2 = xs_log2;
    hp.dpad = ix->dpad;
    hp.per_wave_words = per_wave;
    hp.out_ids = d_out_ids;
    hp.out_d = d_out_d;
    hp.out_n = d_out_n;
    hp.status = ix->status.as<int32_t>();
    hp.counters = ix->counters.as<uint32_t>();
    if (ix->pq_on) hp.pq = pq_params(ix);   // compressed: PQ distances (search.go:171-199)
    // diagnostic: exact per-query visited bitmaps for the evaluation counts
    // (a bounded sample: nq x N bits of scratch, freed after the launch)
    void* uniq = nullptr;
    // (bounded by bytes too: a 100M-node graph would take 51 GB at nq 4096)
    if (std::getenv("WV_HNSW_UNIQUE_COUNTS") && nq <= 4096 && (size_t)nq * ((ix->gn + 63) / 64) * 8 <= ((size_t)1 << 30)) {
        hp.uniq_words = (ix->gn + 63) / 64;
        HIP_TRY(hipMallocAsync(&uniq, (size_t)nq * hp.uniq_words * 8, s));
        HIP_TRY(hipMemsetAsync(uniq, 0, (size_t)nq * hp.uniq_words * 8, s));
        hp.uniq = static_cast<unsigned long long*>(uniq);
    }
    TREC(4);
    // Filtered / tombstoned / nil-node searches with ef <= 128 (round 6):
    // the side-register path.  Layer 0 has an exact visited bitmap per query
    // in HBM (nothing evaluated or queued twice) and a side set whose smallest
    // keys sit in LDS, sized from the eligible fraction p (the live side set
    // peaks near 1.4 ef (1-p)/p: oracle side diagnostics), the
    // rest spilled to HBM.  Only a spill past its capacity takes the exact
    // fallback.  WV_HNSW_NO_SIDE=1 keeps the LDS path.
    const bool side = filtered && !ix->pq_on && efc <= 128 && !std::getenv("WV_HNSW_NO_SIDE");
    if (side) {
        double p_el = 1.0;
        if (d_allow) {
            const int rows = allow_stride ? nq : 1;
            const uint64_t words = std::min<uint64_t>((allow_nbits + 63) / 64, (ix->gn + 63) / 64);
            HIP_TRY(ix->g_cnt.ensure((size_t)rows * 8));
            HIP_TRY(hipMemsetAsync(ix->g_cnt.p, 0, (size_t)rows * 8, s));
            hipLaunchKernelGGL(popcount_rows_kernel, dim3(rows), dim3(256), 0, s, d_allow, words,
                               allow_stride ? allow_stride : words, rows, ix->g_cnt.as<unsigned long long>());
            HIP_TRY(hipGetLastError());
            std::vector<unsigned long long> cnt(rows);
            HIP_TRY(hipMemcpyAsync(cnt.data(), ix->g_cnt.p, 8 * (size_t)rows, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            const unsigned long long mn = *std::min_element(cnt.begin(), cnt.end());
            p_el = (double)mn / (double)std::max<uint64_t>(1, ix->gn);
        }
        p_el *= 1.0 - std::min(1.0, (double)ix->n_tomb / (double)std::max<uint64_t>(1, ix->gn));
        p_el = std::max(p_el, 1e-5);
        const double side_need = 1.4 * ef * (1.0 - p_el) / p_el;
        // per-wave LDS: 13 KiB (12 waves per CU); the side array takes what a
        // 2K-slot visited cache leaves, up to the live-set estimate
        int side_kb = 13;
        if (const char* e = std::getenv("WV_HNSW_SIDE_KB")) side_kb = std::max(4, std::atoi(e));
        const int xl = 8;   // the upper levels' expanded set
        const int budget_words = side_kb * 256;
        const int base_words = wv_hnsw_side_per_wave_words(ix->dpad, 0, 11, xl);
        const int max_rows = std::max(4, (budget_words - base_words) / 128);
        int side_rows = std::min(max_rows, std::max(4, (int)std::ceil((side_need + 64.0) / 64.0)));
        if (const char* e = std::getenv("WV_HNSW_SIDE_ROWS")) side_rows = std::max(4, std::atoi(e));
        wv::HnswParams hs = hp;
        hs.sc = 0;
        hs.side_rows = side_rows;
        hs.xs_log2 = xl;
        const int fixed = wv_hnsw_side_per_wave_words(ix->dpad, side_rows, 0, xl) - 1;
        hs.vc_log2 = std::max(10, choose_vc_log2(std::max(budget_words, fixed + 512), fixed, ix->gn, &hs.vc_tbits));
        int pw = (wv_hnsw_side_per_wave_words(ix->dpad, side_rows, hs.vc_log2, xl) + 3) & ~3;
        while (pw * 4 > 160 * 1024 && hs.vc_log2 > 8) {
            --hs.vc_log2;
            pw = (wv_hnsw_side_per_wave_words(ix->dpad, side_rows, hs.vc_log2, xl) + 3) & ~3;
        }
        if (pw * 4 > 160 * 1024) return fail(WV_EINVAL, "hnsw side state too large");
        hs.per_wave_words = pw;
        int wpb = 4;
        while (wpb > 1 && (size_t)wpb * pw * 4 > 160 * 1024) --wpb;
        // HBM scratch per query: the visited bitmap and the spill, in chunks
        // of at most WV_HNSW_SIDE_SCRATCH_MB (4 GiB) -- a 10M-row graph takes
        // 1.25 MB of bitmap a query
        hs.vwords = (ix->gn + 31) / 32;
        double cap = std::ceil(8.0 * side_need) + 4096.0;
        if (const char* e = std::getenv("WV_HNSW_SPILL_CAP")) cap = std::max(64, std::atoi(e));
        hs.spill_cap = (int)std::min(cap, (double)(1 << 22));
        const size_t per_q = hs.vwords * 4 + (size_t)hs.spill_cap * 8;
        size_t budget_b = (size_t)4 << 30;
        if (const char* e = std::getenv("WV_HNSW_SIDE_SCRATCH_MB")) budget_b = (size_t)std::max(1, std::atoi(e)) << 20;
        const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)nq, budget_b / per_q));
        HIP_TRY(ix->side_vb.ensure((size_t)chunk * hs.vwords * 4));
        HIP_TRY(ix->side_sp.ensure((size_t)chunk * hs.spill_cap * 8));
        hs.vbits = ix->side_vb.as<uint32_t>();
        hs.spill = ix->side_sp.as<uint32_t>();
        ix->last_side_rows = side_rows;
        ix->last_side_xs = hs.spill_cap;
        // Layer 0 with the exact bitmap below WV_HNSW_EV_BELOW (0.4) of the
        // rows eligible; above it (light filters, a few tombstones) the lossy
        // cache + expanded set, whose rare overflow re-runs exactly (redo).
        // Small batches (<= WV_HNSW_WG_MAX, 512): a workgroup per query.
        double ev_below = 0.4;
        if (const char* e = std::getenv("WV_HNSW_EV_BELOW")) ev_below = std::atof(e);
        const bool ev_first = p_el < ev_below;
        int wg_max = 512;
        if (const char* e = std::getenv("WV_HNSW_WG_MAX")) wg_max = std::atoi(e);
        hs.wg_helpers = nq <= wg_max ? 3 : 0;
        HIP_TRY(ix->stat_acc.ensure(48));
        hs.side_acc = ix->stat_acc.as<unsigned long long>();
        hs.ev_spec = std::getenv("WV_HNSW_EV_SPEC") ? 1 : 0;
        const int passes = ev_first ? 1 : 2;
        for (int pass = 0; pass < passes; ++pass) {
            for (int c0 = 0; c0 < nq; c0 += chunk) {
                const int cn = std::min(chunk, nq - c0);
                wv::HnswParams hc = hs;
                hc.nq = cn;
                hc.Q = d_q + (size_t)c0 * hp.ldq;
                if (hc.allow && allow_stride) hc.allow = d_allow + (size_t)c0 * allow_stride;
                hc.out_ids = d_out_ids + (size_t)c0 * k;
                hc.out_d = d_out_d + (size_t)c0 * k;
                hc.out_n = d_out_n + c0;
                hc.status = hp.status + c0;
                hc.counters = hp.counters + 2 * (size_t)c0;
                hc.redo = pass ? hc.status : nullptr;
                hc.vb_host_clear = std::getenv("WV_HNSW_VB_MEMSET") ? 1 : 0;
                if (hc.vb_host_clear && (ev_first || pass))
                    HIP_TRY(hipMemsetAsync(hs.vbits, 0, (size_t)cn * hs.vwords * 4, s));
                HIP_TRY(wv_launch_hnsw_side(&hc, wpb, ev_first || pass, s));
            }
        }
    } else {
    // small unfiltered batches (the batcher's callers): a workgroup per
    // query, whose three helper waves take the distance batches' other rows
    // -- while every workgroup is resident (up to 3 per CU at 158 VGPRs; a
    // 256-query batch 898 -> 705 us p50, profiles/r05/wg_latency.log).
    // WV_HNSW_WG_MAX: the largest such batch; 0 turns it off.
    int wg_max = 512;
    if (const char* e = std::getenv("WV_HNSW_WG_MAX")) wg_max = std::atoi(e);
    const bool wg = !filtered && !ix->pq_on && reg && nq <= wg_max;
    if (wg) {
        hp.wg_helpers = 3;
        HIP_TRY(wv_launch_hnsw_wg(&hp, s));
    } else {
        HIP_TRY(wv_launch_hnsw(&hp, wpb, s));
    }
    if (filtered && !std::getenv("WV_HNSW_NO_WIDE_SIDE")) {
        // second pass for the queries whose side set or expanded-set table
        // overflowed (status != 0; the others' waves exit at once): the same
        // search with a 2048-entry side set and a 2048-slot expanded set --
        // selective filters traverse many ineligible nodes (search.go:282-298:
        // at 10 % of the rows the reference's candidate heap reaches ~1.8k).
        // Only what still overflows here takes the exact fallback.
        wv::HnswParams h2 = hp;
        h2.redo = ix->status.as<int32_t>();
        h2.sc = 2048;
        h2.xs_log2 = 11;
        const int fixed2 = wv_hnsw_per_wave_words(ix->dpad, efc, h2.sc, 0, h2.xs_log2) - 1;
        h2.vc_log2 = choose_vc_log2(fixed2 + 1024, fixed2, ix->gn, &h2.vc_tbits);
        int pw2 = (wv_hnsw_per_wave_words(ix->dpad, efc, h2.sc, h2.vc_log2, h2.xs_log2) + 3) & ~3;
        h2.per_wave_words = pw2;
        int wpb2 = 4;
        while (wpb2 > 1 && (size_t)wpb2 * pw2 * 4 > 160 * 1024) --wpb2;
        if ((size_t)pw2 * 4 <= 160 * 1024) HIP_TRY(wv_launch_hnsw(&h2, wpb2, s));
    }
    }
    TREC(5);
    if (uniq) HIP_TRY(hipFreeAsync(uniq, s));
    HIP_TRY(ix->stat_acc.ensure(48));
    HIP_TRY(wv_launch_hnsw_stats(ix->counters.as<uint32_t>(), nq, ix->stat_acc.as<unsigned long long>(), s));
    if (!ix->pq_on) {
        // queries whose side state outgrew LDS: exact answer on the device
        HIP_TRY(ix->fail.ensure((size_t)nq * 4));
        HIP_TRY(ix->fail_thr.ensure((size_t)nq * 4));
        HIP_TRY(wv_launch_fbd_mark(ix->status.as<int32_t>(), nq, ix->fail.as<int32_t>(), ix->fail_thr.as<float>(),
                                   d_out_d, d_out_n, k, s));
        return queue_fbd(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    }
    std::vector<int32_t> st(nq);
    HIP_TRY(hipMemcpyAsync(st.data(), ix->status.p, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // Queries whose side-candidate set outgrew LDS are answered exactly
    // (flatSearch over the same allow list: a superset in quality).
    for (int q = 0; q < nq; ++q) {
        if (!st[q]) continue;
        ix->last_fallbacks++;
        const uint64_t* al = d_allow ? d_allow + (allow_stride ? (uint64_t)q * allow_stride : 0) : nullptr;
        int rc = ix->pq_on ? run_pq_flat(ix, d_q + (size_t)q * ix->dpad, 1, k, al, allow_nbits, 0,
                                         d_out_ids + (size_t)q * k, d_out_d + (size_t)q * k, d_out_n + q, s, nullptr, 0)
                           : exact_full(ix, d_q + (size_t)q * ix->dpad, k, al, allow_nbits, d_out_ids + (size_t)q * k,
                                        d_out_d + (size_t)q * k, d_out_n + q, s);
        if (rc) return rc;
    }
    return WV_OK;
}

// out[r][w] = a[r or 0][w] & b[w]  (rows x words; a_stride 0 = one shared row)
__global__ void and_bits_kernel(const uint64_t* a, uint64_t a_words, uint64_t a_stride, const uint64_t* b,
                                uint64_t words, int rows, uint64_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= words * (uint64_t)rows) return;
    const uint64_t r = i / words, w = i % words;
    const uint64_t av = a ? (w < a_words ? a[r * a_stride + w] : 0ull) : ~0ull;
    out[i] = av & b[w];
}

// knnSearchByVector over the uploaded graph, plus an exact pass over the
// delta set (rows added since the graph snapshot), merged by
// (dist, id): added rows are findable at once, as in the reference where
// Add inserts into the live graph (insert.go:43-65).  Exact over the delta is
// a superset in quality of a graph search.
int run_hnsw_delta(wv_index* ix, const float* d_q, int nq, int k, int ef, const uint64_t* d_allow,
                   uint64_t allow_nbits, uint64_t allow_stride, uint64_t* d_out_ids, float* d_out_d,
                   int32_t* d_out_n, hipStream_t s) {
    if (ix->delta_count == 0 || nq == 0)
        return run_hnsw(ix, d_q, nq, k, ef, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    const size_t nk = (size_t)nq * k;
    HIP_TRY(ix->dl_ids.ensure(2 * nk * 8));
    HIP_TRY(ix->dl_d.ensure(2 * nk * 4));
    HIP_TRY(ix->dl_n.ensure(2 * (size_t)nq * 4));
    uint64_t* ids = ix->dl_ids.as<uint64_t>();
    float* ds = ix->dl_d.as<float>();
    int32_t* ns = ix->dl_n.as<int32_t>();
    int rc = run_hnsw(ix, d_q, nq, k, ef, d_allow, allow_nbits, allow_stride, ids, ds, ns, s);
    if (rc) return rc;
    const uint64_t words = ix->bm_words;
    const int rows = d_allow && allow_stride ? nq : 1;
    HIP_TRY(ix->dmask.ensure((size_t)rows * words * 8));
    hipLaunchKernelGGL(and_bits_kernel, dim3((unsigned)((rows * words + 255) / 256)), dim3(256), 0, s, d_allow,
                       (allow_nbits + 63) / 64, allow_stride ? allow_stride : 0, ix->delta.as<uint64_t>(), words, rows,
                       ix->dmask.as<uint64_t>());
    HIP_TRY(hipGetLastError());
    const uint64_t st = d_allow && allow_stride ? words : 0;
    const uint64_t e = ix->last_dist, x = ix->last_exp, f = ix->last_fallbacks;
    rc = run_exact(ix, d_q, nq, k, ix->dmask.as<uint64_t>(), ix->capacity, st, ids + nk, ds + nk, ns + nq, s,
                   st ? ix->delta.as<uint64_t>() : nullptr, ix->capacity);
    if (rc) return rc;
    ix->last_dist = e;
    ix->last_exp = x;
    ix->last_fallbacks += f;
    hipLaunchKernelGGL(merge_shards_kernel, dim3((nq + 127) / 128), dim3(128), 0, s, ds, ids, ns, 2, nq, k, d_out_d,
                       d_out_ids, d_out_n);
    HIP_TRY(hipGetLastError());
    return WV_OK;
}

// Core: device queries already padded to dpad and normalized (cosine).
int search_core(wv_index* ix, const float* d_q, int nq, int k, int ef, const uint64_t* d_allow,
                uint64_t allow_nbits, uint64_t allow_stride, int mode, uint64_t* d_out_ids, float* d_out_d,
                int32_t* d_out_n, hipStream_t s) {
    int rc = refresh_bitmaps(ix);
    if (rc) return rc;
    ix->last_dist = ix->last_exp = ix->last_fallbacks = 0;
    ix->last_side_rows = ix->last_side_xs = 0;
    HIP_TRY(ix->stat_acc.ensure(48));
    HIP_TRY(hipMemsetAsync(ix->stat_acc.p, 0, 48, s));
    ix->stat_stream = s;
    if (ix->timing) {
        if (ix->ev_used == ix->ev_pool.size()) {
            std::array<hipEvent_t, 8> e{};
            for (auto& x : e) HIP_TRY(hipEventCreate(&x));
            ix->ev_pool.push_back(e);
            ix->ev_mask.push_back(0);
        }
        ix->ev = ix->ev_pool[ix->ev_used].data();
        ix->ev_mask[ix->ev_used] = 0;
        ix->ev_used++;
    }
    if (ef <= 0) ef = search_time_ef(ix->cfg, k);
    if (mode == WV_MODE_EXACT)
        return run_exact(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    if (mode == WV_MODE_HNSW) {
        if (ef > wv::HNSW_EF_MAX)
            return run_exact(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
        return run_hnsw_delta(ix, d_q, nq, k, ef, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    }
    // AUTO: search.go:74-78
    const bool can_hnsw = ix->has_graph && ef <= wv::HNSW_EF_MAX;
    if (!d_allow || ix->cfg.forbid_flat) {
        if (can_hnsw)
            return run_hnsw_delta(ix, d_q, nq, k, ef, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
        return run_exact(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    }
    // allowList.Len() < flatSearchCutoff decides per query
    const int rows = allow_stride ? nq : 1;
    const uint64_t words = (allow_nbits + 63) / 64;
    HIP_TRY(ix->g_cnt.ensure((size_t)rows * 8));
    HIP_TRY(hipMemsetAsync(ix->g_cnt.p, 0, (size_t)rows * 8, s));
    hipLaunchKernelGGL(popcount_rows_kernel, dim3(rows), dim3(256), 0, s, d_allow, words,
                       allow_stride ? allow_stride : words, rows, ix->g_cnt.as<unsigned long long>());
    HIP_TRY(hipGetLastError());
    std::vector<unsigned long long> cnt(rows);
    HIP_TRY(hipMemcpyAsync(cnt.data(), ix->g_cnt.p, 8 * (size_t)rows, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<int32_t> flat, knn;
    for (int q = 0; q < nq; ++q) {
        const unsigned long long c = cnt[allow_stride ? q : 0];
        if ((int64_t)c < ix->cfg.flat_search_cutoff || !can_hnsw) flat.push_back(q);
        else knn.push_back(q);
    }
    if (knn.empty())
        return run_exact(ix, d_q, nq, k, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    if (flat.empty())
        return run_hnsw_delta(ix, d_q, nq, k, ef, d_allow, allow_nbits, allow_stride, d_out_ids, d_out_d, d_out_n, s);
    // split the batch: gather each group, run, scatter back
    for (int pass = 0; pass < 2; ++pass) {
        const std::vector<int32_t>& sel = pass == 0 ? flat : knn;
        const int n = (int)sel.size();
        HIP_TRY(ix->g_idx.ensure((size_t)n * 4));
        HIP_TRY(ix->g_q.ensure((size_t)n * ix->dpad * 4));
        HIP_TRY(ix->g_ids.ensure((size_t)n * k * 8));
        HIP_TRY(ix->g_d.ensure((size_t)n * k * 4));
        HIP_TRY(ix->g_n.ensure((size_t)n * 4));
        HIP_TRY(hipMemcpyAsync(ix->g_idx.p, sel.data(), 4 * (size_t)n, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(gather_rows_kernel, dim3(n), dim3(128), 0, s, d_q, ix->dpad, ix->g_idx.as<int32_t>(), n,
                           ix->dpad, ix->g_q.as<float>(), ix->dpad);
        const uint64_t* al = d_allow;
        uint64_t ast = 0;
        if (allow_stride) {
            HIP_TRY(ix->g_allow.ensure((size_t)n * allow_stride * 8));
            hipLaunchKernelGGL(gather_words_kernel, dim3(n), dim3(256), 0, s, d_allow, allow_stride,
                               ix->g_idx.as<int32_t>(), n, ix->g_allow.as<uint64_t>());
            al = ix->g_allow.as<uint64_t>();
            ast = allow_stride;
        }
        HIP_TRY(hipGetLastError());
        int rc2 = pass == 0 ? run_exact(ix, ix->g_q.as<float>(), n, k, al, allow_nbits, ast, ix->g_ids.as<uint64_t>(),
                                        ix->g_d.as<float>(), ix->g_n.as<int32_t>(), s)
                            : run_hnsw_delta(ix, ix->g_q.as<float>(), n, k, ef, al, allow_nbits, ast,
                                       ix->g_ids.as<uint64_t>(), ix->g_d.as<float>(), ix->g_n.as<int32_t>(), s);
        if (rc2) return rc2;
        hipLaunchKernelGGL(scatter_results_kernel, dim3(n), dim3(64), 0, s, ix->g_ids.as<uint64_t>(),
                           ix->g_d.as<float>(), ix->g_n.as<int32_t>(), ix->g_idx.as<int32_t>(), n, k, d_out_ids,
                           d_out_d, d_out_n);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(s));
    }
    return WV_OK;
}

// host queries -> device, padded, normalized for cosine (search.go:68-72)
int stage_queries(wv_index* ix, const float* q, int nq, const float** d_out, hipStream_t s) {
    HIP_TRY(ix->q_in.ensure((size_t)nq * ix->dpad * 4));
    if (ix->dpad == ix->dim) {
        HIP_TRY(hipMemcpyAsync(ix->q_in.p, q, (size_t)nq * ix->dim * 4, hipMemcpyHostToDevice, s));
    } else {
        HIP_TRY(ix->stage.ensure((size_t)nq * ix->dim * 4));
        HIP_TRY(hipMemcpyAsync(ix->stage.p, q, (size_t)nq * ix->dim * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(launch_pad_rows(ix->stage.as<float>(), ix->dim, nq, ix->dim, ix->q_in.as<float>(), ix->dpad, s));
    }
    if (ix->metric == WV_COSINE_DOT)
        HIP_TRY(wv_launch_normalize(ix->q_in.as<float>(), ix->q_in.as<float>(), nq, ix->dim, ix->dpad, s));
    *d_out = ix->q_in.as<float>();
    return WV_OK;
}

int check(wv_index* ix) {
    if (!ix) return fail(WV_EINVAL, "null index");
    return WV_OK;
}

}  // namespace

extern "C" {

void wv_config_default(wv_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->device = 0;
    c->max_connections = 64;
    c->ef = -1;
    c->dynamic_ef_min = 100;
    c->dynamic_ef_max = 500;
    c->dynamic_ef_factor = 8;
    c->flat_search_cutoff = 40000;
    c->forbid_flat = 0;
    c->id_base = 0;
}

const char* wv_last_error(void) { return g_err.c_str(); }
// for wv_batcher.cpp: a request's error is reported on its caller's thread
void wv_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }
const char* wv_version(void) { return "wvgpu 0.1 (gfx950)"; }

int wv_index_create(int dim, int metric, const wv_config* cfg, uint64_t capacity, wv_index** out) {
    if (!out || dim <= 0 || metric < 0 || metric > 2 || capacity == 0 || capacity >= (1ull << 31))
        return fail(WV_EINVAL, "wv_index_create: bad argument");
    auto* ix = new wv_index();
    ix->dim = dim;
    ix->dpad = (dim + 3) & ~3;
    ix->ldx = dim >= 32 ? (dim + 31) & ~31 : ix->dpad;
    ix->metric = metric;
    if (cfg) ix->cfg = *cfg; else wv_config_default(&ix->cfg);
    ix->capacity = capacity;
    hipError_t e = hipSetDevice(ix->cfg.device);
    if (e != hipSuccess) { delete ix; return fail(WV_EDEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e)); }
    e = hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete ix; return fail(WV_EDEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e)); }
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->cfg.device) != hipSuccess || cus <= 0)
            cus = 256;
        ix->bf_blocks = cus * 2;
        ix->n_cus = cus;
    }
    ix->bm_words = (capacity + 63) / 64;
    // whole brute-force tiles (wv_bf.hip layout contract) and whole 256-row
    // tiles of the wide f16 pass: zero rows past capacity
    const uint64_t cap_rows = align_rows(capacity);
    const size_t vbytes = cap_rows * (size_t)ix->ldx * 4;
    if (ix->vecs.ensure(vbytes) != hipSuccess || ix->xnorm.ensure(cap_rows * 4) != hipSuccess ||
        ix->maxnorm.ensure(4) != hipSuccess || ix->tomb.ensure(ix->bm_words * 8) != hipSuccess ||
        ix->excl.ensure((ix->bm_words + 4) * 8) != hipSuccess) {   // + the words of a last 256-row tile
        wv_index_destroy(ix);
        return fail(WV_EOOM, "wv_index_create: device allocation failed");
    }
    // bf16x3 key pass (wv_bf_split_kernel): whole 32-float chunks, stride <= 128
    // (the query block image stays resident in LDS); WV_BF_FP32=1 keeps the
    // fp32 MFMA pass for every scan
    // f16 key pass (wv_bf_h16_kernel) for D <= 128 unless an ablation switch
    // asks for the bf16x3 (WV_BF_SPLIT=1) or the fp32 (WV_BF_FP32=1) pass
    ix->use_h16 = dim <= 16 * wv::HW_NS_MAX && !std::getenv("WV_BF_FP32") && !std::getenv("WV_BF_SPLIT");
    if (ix->use_h16) {
        // D > 128: the wide-D kernel, whose chunks are HW_KC 16-k steps
        ix->h16_wide = dim > 16 * wv::H_NS_MAX;
        ix->h16_ns = ix->h16_wide ? (dim + 16 * wv::HW_KC - 1) / (16 * wv::HW_KC) * wv::HW_KC : (dim + 15) / 16;
        const size_t ibytes = cap_rows * (size_t)ix->h16_ns * 16 * 2;
        if (ix->ximg16.ensure(ibytes) != hipSuccess || ix->xns.ensure(cap_rows * 4) != hipSuccess ||
            ix->ex_bits.ensure(4) != hipSuccess || ix->qmax.ensure(4) != hipSuccess ||
            ix->qscale.ensure(4) != hipSuccess) {
            wv_index_destroy(ix);
            return fail(WV_EOOM, "wv_index_create: device allocation failed");
        }
        (void)hipMemsetAsync(ix->ximg16.p, 0, ibytes, ix->stream);
        (void)hipMemsetAsync(ix->xns.p, 0, cap_rows * 4, ix->stream);
        (void)hipMemsetAsync(ix->ex_bits.p, 0, 4, ix->stream);
    }
    ix->use_split = !ix->use_h16 && ix->ldx % wv::BF_BK == 0 && ix->ldx <= 128 && !std::getenv("WV_BF_FP32");
    if (ix->use_split && ix->xsplit.ensure(vbytes) != hipSuccess) {
        wv_index_destroy(ix);
        return fail(WV_EOOM, "wv_index_create: device allocation failed");
    }
    if (ix->use_split) (void)hipMemsetAsync(ix->xsplit.p, 0, vbytes, ix->stream);
    (void)hipMemsetAsync(ix->vecs.p, 0, vbytes, ix->stream);
    (void)hipMemsetAsync(ix->xnorm.p, 0, cap_rows * 4, ix->stream);
    (void)hipMemsetAsync(ix->maxnorm.p, 0, 4, ix->stream);
    (void)hipStreamSynchronize(ix->stream);
    ix->has_vec.assign(ix->bm_words, 0);
    ix->tomb_host.assign(ix->bm_words, 0);
    ix->pending_host.assign(ix->bm_words, 0);
    *out = ix;
    return WV_OK;
}

int wv_index_destroy(wv_index* ix) {
    if (!ix) return WV_OK;
    (void)hipSetDevice(ix->cfg.device);
    for (DevBuf* b : {&ix->vecs, &ix->xsplit, &ix->xnorm, &ix->maxnorm, &ix->levels, &ix->layer0, &ix->upper_row, &ix->upper,
                      &ix->tomb, &ix->excl, &ix->q_in, &ix->q_norm, &ix->q_nrm2, &ix->q_scaled, &ix->cand_d, &ix->cand_id,
                      &ix->fail, &ix->status, &ix->counters, &ix->scan_d, &ix->scan_i, &ix->sort_d, &ix->sort_i,
                      &ix->sort_tmp, &ix->g_idx, &ix->g_q, &ix->g_allow, &ix->g_ids, &ix->g_d, &ix->g_n, &ix->g_cnt,
                      &ix->out_ids, &ix->out_d, &ix->out_n, &ix->stage, &ix->fail_thr, &ix->fb_idx, &ix->fb_d, &ix->fb_i, &ix->fb_n, &ix->fb_of,
                      &ix->ac_cnt, &ix->ac_off, &ix->rowidx, &ix->pq_cent, &ix->pq_codes, &ix->pk_key,
                      &ix->pk_dist, &ix->pk_val, &ix->pk_skey, &ix->pk_sval, &ix->pk_off, &ix->ximg16, &ix->qmax_part, &ix->xns,
                      &ix->qimg16, &ix->qres, &ix->qmax, &ix->qscale, &ix->tau, &ix->gtau, &ix->marg, &ix->allow_pad, &ix->ex_bits, &ix->gslot, &ix->blk_order,
                      &ix->delta, &ix->dmask, &ix->dl_ids, &ix->dl_d, &ix->dl_n, &ix->dq_tmp, &ix->b_tgt, &ix->b_ci,
                      &ix->b_cd, &ix->b_cn, &ix->b_cnt0, &ix->b_cntu, &ix->b_rk, &ix->b_rn, &ix->b_rk2, &ix->b_rn2,
                      &ix->b_uk, &ix->b_ul, &ix->b_uo, &ix->b_nr, &ix->b_tmp, &ix->stat_acc, &ix->fbd_list,
                      &ix->fbd_nf, &ix->fbd_over, &ix->fbd_cd, &ix->fbd_ci, &ix->fbd_cn, &ix->fbd_scr})
        b->release();
    if (ix->stream) (void)hipStreamSynchronize(ix->stream);
    ix->allow_keep.release();
    for (DevBuf* b : {&ix->sbd_t, &ix->sbd_keys, &ix->sbd_tmp, &ix->sbd_cnt, &ix->sbd_off, &ix->sbd_q}) b->release();
    if (ix->sbd_scr) (void)hipFree(ix->sbd_scr);
    ix->sbd_scr = nullptr;
    ix->cimg16.release();
    ix->cxnorm.release();
    ix->cexcl.release();
    for (auto& sl : ix->slots) {
        if (sl.pin) (void)hipHostFree(sl.pin);
        if (sl.done) (void)hipEventDestroy(sl.done);
    }
    for (auto& set : ix->ev_pool)
        for (auto e : set)
            if (e) (void)hipEventDestroy(e);
    if (ix->ev_in) (void)hipEventDestroy(ix->ev_in);
    if (ix->ev_out) (void)hipEventDestroy(ix->ev_out);
    if (ix->ev_null) (void)hipEventDestroy(ix->ev_null);
    if (ix->stream) (void)hipStreamDestroy(ix->stream);
    delete ix;
    return WV_OK;
}

int wv_index_update_config(wv_index* ix, const wv_config* cfg) {
    if (check(ix) || !cfg) return fail(WV_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    const int dev = ix->cfg.device;
    const uint64_t base = ix->cfg.id_base;
    ix->cfg = *cfg;
    ix->cfg.device = dev;   // the device and id base are fixed at creation
    ix->cfg.id_base = base;
    return WV_OK;
}

// After rows were written to vecs (rownorm updated maxnorm; the stream is
// synchronised): cache max |x| on the host (the finalize's eps needs it, and
// reading it per batch would cost a host round trip), and keep the f16 image
// in step.  s_x is fixed by the first write and only ever lowered (then the
// whole image is rebuilt) so that no element overflows f16.
static int rows_written(wv_index* ix, const uint64_t* d_ids, uint64_t n, uint64_t first_id) {
    unsigned int mb = 0;
    HIP_TRY(hipMemcpyAsync(&mb, ix->maxnorm.p, 4, hipMemcpyDeviceToHost, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    std::memcpy(&ix->maxnorm_host, &mb, 4);
    if (!ix->use_h16 || n == 0) return WV_OK;
    const float sx = wv_h16_pow2_scale(ix->maxnorm_host);
    const bool rebuild = ix->h16_sx != 0.f && sx < ix->h16_sx;
    if (ix->h16_sx == 0.f || rebuild) ix->h16_sx = sx;
    unsigned int* exb = ix->ex_bits.as<unsigned int>();
    if (rebuild) HIP_TRY(hipMemsetAsync(exb, 0, 4, ix->stream));
    {
        void* img = ix->ximg16.p;
        const int wide_layout = ix->h16_wide ? 1 : 0;   // (the wide-D kernel's h16w_index image)
        if (rebuild) {
            HIP_TRY(wv_launch_h16_rows(ix->vecs.as<float>(), ix->ldx, nullptr, ix->n_rows, ix->dim, ix->h16_ns, 1.f,
                                       ix->h16_sx, nullptr, img, 0, exb, nullptr, wide_layout, ix->stream));
        } else if (d_ids) {
            HIP_TRY(wv_launch_h16_rows(ix->vecs.as<float>(), ix->ldx, d_ids, n, ix->dim, ix->h16_ns, 1.f, ix->h16_sx,
                                       nullptr, img, 0, exb, nullptr, wide_layout, ix->stream));
        } else {
            HIP_TRY(wv_launch_h16_rows(ix->vecs.as<float>() + first_id * ix->ldx, ix->ldx, nullptr, n, ix->dim,
                                       ix->h16_ns, 1.f, ix->h16_sx, nullptr, img, first_id, exb, nullptr, wide_layout,
                                       ix->stream));
        }
    }
    unsigned int eb = 0;
    HIP_TRY(hipMemcpyAsync(&eb, exb, 4, hipMemcpyDeviceToHost, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    std::memcpy(&ix->h16_ex, &eb, 4);
    return WV_OK;
}

// Rows written while a quantizer is set: with KMeans encoders the device
// encodes them as hnsw.Add does on a compressed index (insert.go:91-95,
// 166-170); codes of other encoders come from the host, so the rows are
// unsearchable on a compressed index until wv_index_upload_pq_codes.
static int pq_rows_written(wv_index* ix, const uint64_t* d_ids, const uint64_t* ids, uint64_t n, uint64_t first_id) {
    if (!ix->pq_set || n == 0) return WV_OK;
    if (ix->pq_encoder == WV_PQ_KMEANS) {
        wv::PqParams pq = pq_params(ix);
        if (d_ids) {
            HIP_TRY(wv_launch_pq_encode(ix->vecs.as<float>(), ix->ldx, d_ids, n, &pq, ix->pq_codes.as<uint8_t>(),
                                        ix->stream));
        } else {
            HIP_TRY(wv_launch_pq_encode(ix->vecs.as<float>() + first_id * ix->ldx, ix->ldx, nullptr, n, &pq,
                                        ix->pq_codes.as<uint8_t>() + first_id * ix->pq_stride, ix->stream));
        }
        HIP_TRY(hipStreamSynchronize(ix->stream));
    }
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t id = ids ? ids[i] : first_id + i;
        if (ix->pq_encoder == WV_PQ_KMEANS) ix->has_code[id >> 6] |= 1ull << (id & 63);
        else ix->has_code[id >> 6] &= ~(1ull << (id & 63));
    }
    ix->bitmaps_dirty = true;
    return WV_OK;
}

static int upload_rows(wv_index* ix, const float* src, bool device_src, int ld, uint64_t n, uint64_t first_id) {
    if (first_id + n > ix->capacity) return fail(WV_EINVAL, "upload beyond capacity");
    if (n == 0) return WV_OK;
    HIP_TRY(hipSetDevice(ix->cfg.device));
    float* dst = ix->vecs.as<float>() + first_id * ix->ldx;
    const float* dsrc = src;
    if (!device_src) {
        HIP_TRY(ix->stage.ensure(n * (size_t)ix->dim * 4));
        HIP_TRY(hipMemcpyAsync(ix->stage.p, src, n * (size_t)ix->dim * 4, hipMemcpyHostToDevice, ix->stream));
        dsrc = ix->stage.as<float>();
        ld = ix->dim;
    }
    HIP_TRY(launch_pad_rows(dsrc, ld, n, ix->dim, dst, ix->ldx, ix->stream));
    if (ix->metric == WV_COSINE_DOT)  // normalize on write (insert.go:56-60, vector_cache.go:110-112)
        HIP_TRY(wv_launch_normalize(dst, dst, n, ix->dim, ix->ldx, ix->stream));
    HIP_TRY(wv_launch_rownorm(dst, n, ix->dim, ix->ldx, ix->xnorm.as<float>() + first_id,
                              ix->maxnorm.as<unsigned int>(), ix->stream));
    if (ix->use_split)
        HIP_TRY(wv_launch_split_rows(dst, ix->ldx, nullptr, n, n, ix->dim, 1.f, ix->xsplit.p, ix->ldx, first_id,
                                     ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    for (uint64_t i = first_id; i < first_id + n; ++i) ix->has_vec[i >> 6] |= 1ull << (i & 63);
    ix->n_rows = std::max(ix->n_rows, first_id + n);
    ix->bitmaps_dirty = true;
    int rc = rows_written(ix, nullptr, n, first_id);
    if (rc) return rc;
    return pq_rows_written(ix, nullptr, nullptr, n, first_id);
}

int wv_index_upload_vectors(wv_index* ix, const float* rows, uint64_t n, uint64_t first_id) {
    if (check(ix) || (!rows && n)) return fail(WV_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    return upload_rows(ix, rows, false, ix->dim, n, first_id);
}

int wv_index_upload_vectors_device(wv_index* ix, const float* d_rows, uint64_t n, uint64_t first_id, int ld) {
    if (check(ix) || (!d_rows && n) || ld < ix->dim) return fail(WV_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    return upload_rows(ix, d_rows, true, ld, n, first_id);
}

int wv_index_upload_graph(wv_index* ix, uint64_t n, const int8_t* levels, const uint32_t* layer0, int deg0,
                          const uint32_t* upper_row, const uint32_t* upper, uint64_t n_upper, int degU, int max_level,
                          uint64_t entrypoint) {
    if (check(ix)) return WV_EINVAL;
    if (n == 0 || n > ix->capacity || !levels || !layer0 || deg0 <= 0 || deg0 > 256 || max_level < 0 ||
        entrypoint >= n || (max_level > 0 && (!upper_row || !upper || degU <= 0 || degU > 256)))
        return fail(WV_EINVAL, "wv_index_upload_graph: bad argument");
    // A nil entrypoint is the reference's "entrypoint was deleted"
    // (search.go:473-476).  An entrypoint below max_level is legal: the
    // descent skips a node whose level is below the layer (search.go:226-233),
    // as after deleteEntrypoint wrote the lower level first (delete.go:405-414).
    // Checked before any loop reads `upper`, whose size is n_upper * max_level
    // * degU: the caller's array must have exactly that level stride.
    if (levels[entrypoint] < 0) return fail(WV_EDELETED, "wv_index_upload_graph: entrypoint is a nil node");
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    // validate neighbour ids on the host once (a bad id would fault the kernel)
    for (uint64_t i = 0; i < n * (uint64_t)deg0; ++i)
        if (layer0[i] != WV_NIL && layer0[i] >= n) return fail(WV_EINVAL, "layer0 neighbour out of range");
    if (max_level > 0) {
        for (uint64_t i = 0; i < n; ++i) {
            if (levels[i] >= 1 && (upper_row[i] == WV_NIL || upper_row[i] >= n_upper))
                return fail(WV_EINVAL, "upper_row out of range");
        }
        for (uint64_t i = 0; i < n_upper * (uint64_t)max_level * degU; ++i)
            if (upper[i] != WV_NIL && upper[i] >= n) return fail(WV_EINVAL, "upper neighbour out of range");
    }
    HIP_TRY(ix->levels.ensure(n));
    HIP_TRY(ix->layer0.ensure(n * (size_t)deg0 * 4));
    HIP_TRY(ix->upper_row.ensure(n * 4));
    HIP_TRY(ix->upper.ensure(std::max<uint64_t>(1, n_upper * (uint64_t)std::max(1, max_level) * std::max(1, degU)) * 4));
    HIP_TRY(hipMemcpyAsync(ix->levels.p, levels, n, hipMemcpyHostToDevice, ix->stream));
    HIP_TRY(hipMemcpyAsync(ix->layer0.p, layer0, n * (size_t)deg0 * 4, hipMemcpyHostToDevice, ix->stream));
    if (max_level > 0) {
        HIP_TRY(hipMemcpyAsync(ix->upper_row.p, upper_row, n * 4, hipMemcpyHostToDevice, ix->stream));
        HIP_TRY(hipMemcpyAsync(ix->upper.p, upper, n_upper * (size_t)max_level * degU * 4, hipMemcpyHostToDevice,
                               ix->stream));
    }
    HIP_TRY(hipStreamSynchronize(ix->stream));
    ix->nil_host.assign(ix->bm_words, ~0ull);
    for (uint64_t i = 0; i < n; ++i)
        if (levels[i] >= 0) ix->nil_host[i >> 6] &= ~(1ull << (i & 63));
    ix->any_nil = std::any_of(levels, levels + n, [](int8_t l) { return l < 0; });
    for (uint64_t i = 0; i < n; ++i)   // the new snapshot holds these added rows
        if (levels[i] >= 0) ix->pending_host[i >> 6] &= ~(1ull << (i & 63));
    ix->gn = n;
    ix->deg0 = deg0;
    ix->degU = max_level > 0 ? degU : 1;
    ix->max_level = max_level;
    ix->n_upper = n_upper;
    ix->entrypoint = entrypoint;
    ix->has_graph = true;
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_set_tombstones(wv_index* ix, const uint64_t* bits, uint64_t nbits) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    std::fill(ix->tomb_host.begin(), ix->tomb_host.end(), 0);
    const uint64_t w = std::min<uint64_t>((nbits + 63) / 64, ix->bm_words);
    for (uint64_t i = 0; i < w; ++i) ix->tomb_host[i] = bits ? bits[i] : 0;
    if (nbits & 63 && w == (nbits + 63) / 64 && w > 0) ix->tomb_host[w - 1] &= (1ull << (nbits & 63)) - 1;
    ix->n_tomb = 0;
    for (uint64_t i = 0; i < ix->bm_words; ++i) ix->n_tomb += (uint64_t)__builtin_popcountll(ix->tomb_host[i]);
    ix->any_tomb = ix->n_tomb > 0;
    ix->bitmaps_dirty = true;
    return WV_OK;
}

__global__ void scatter_rows_kernel(const float* src, int ld_src, const uint64_t* ids, uint64_t n, int ldx,
                                    float* X, const float* norms, float* xnorm) {
    const uint64_t r = blockIdx.x;
    if (r >= n) return;
    const uint64_t id = ids[r];
    for (int i = threadIdx.x; i < ldx; i += blockDim.x) X[id * ldx + i] = src[r * (uint64_t)ld_src + i];
    if (threadIdx.x == 0) xnorm[id] = norms[r];
}

int wv_index_add(wv_index* ix, const uint64_t* ids_in, const float* rows_in, uint64_t n_in) {
    if (check(ix) || (n_in && (!ids_in || !rows_in))) return fail(WV_EINVAL, "wv_index_add: bad argument");
    if (n_in == 0) return WV_OK;
    for (uint64_t i = 0; i < n_in; ++i)
        if (ids_in[i] >= ix->capacity) return fail(WV_EINVAL, "wv_index_add: id beyond capacity");
    // The reference applies Adds one after another, so the last write of a
    // repeated id wins (insert.go:43-65).  One scatter block per distinct id:
    // two blocks writing one row would leave a mix of both rows, and its |x|^2
    // (which the finalize certificate relies on) from either.
    std::vector<uint64_t> ids_v;
    std::vector<float> rows_v;
    const uint64_t* ids = ids_in;
    const float* rows = rows_in;
    uint64_t n = n_in;
    {
        std::vector<uint64_t> sorted(ids_in, ids_in + n_in);
        std::sort(sorted.begin(), sorted.end());
        if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) {
            std::vector<uint64_t> last_pos;   // positions of the last occurrence, in input order
            std::vector<uint8_t> seen(ix->bm_words * 64, 0);
            for (uint64_t i = n_in; i-- > 0;)
                if (!seen[ids_in[i]]) { seen[ids_in[i]] = 1; last_pos.push_back(i); }
            std::reverse(last_pos.begin(), last_pos.end());
            ids_v.resize(last_pos.size());
            rows_v.resize(last_pos.size() * (size_t)ix->dim);
            for (size_t j = 0; j < last_pos.size(); ++j) {
                ids_v[j] = ids_in[last_pos[j]];
                std::memcpy(rows_v.data() + j * ix->dim, rows_in + last_pos[j] * ix->dim, ix->dim * sizeof(float));
            }
            ids = ids_v.data();
            rows = rows_v.data();
            n = ids_v.size();
        }
    }
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    hipStream_t s = ix->stream;
    // rows -> [n][ldx] padded (normalized for cosine, insert.go:56-60), their
    // |x|^2, then scattered to their ids
    HIP_TRY(ix->stage.ensure(n * (size_t)ix->dim * 4));
    HIP_TRY(ix->dq_tmp.ensure(n * (size_t)ix->ldx * 4 + n * 4 + n * 8));
    float* tmp = ix->dq_tmp.as<float>();
    float* nrm = tmp + n * (size_t)ix->ldx;
    uint64_t* d_ids = reinterpret_cast<uint64_t*>(nrm + n + (n & 1));
    HIP_TRY(hipMemcpyAsync(ix->stage.p, rows, n * (size_t)ix->dim * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_ids, ids, n * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_pad_rows(ix->stage.as<float>(), ix->dim, n, ix->dim, tmp, ix->ldx, s));
    if (ix->metric == WV_COSINE_DOT) HIP_TRY(wv_launch_normalize(tmp, tmp, n, ix->dim, ix->ldx, s));
    HIP_TRY(wv_launch_rownorm(tmp, n, ix->dim, ix->ldx, nrm, ix->maxnorm.as<unsigned int>(), s));
    hipLaunchKernelGGL(scatter_rows_kernel, dim3((unsigned)n), dim3(128), 0, s, tmp, ix->ldx, d_ids, n, ix->ldx,
                       ix->vecs.as<float>(), nrm, ix->xnorm.as<float>());
    HIP_TRY(hipGetLastError());
    if (ix->use_split)
        HIP_TRY(wv_launch_split_rows(ix->vecs.as<float>(), ix->ldx, d_ids, n, n, ix->dim, 1.f, ix->xsplit.p, ix->ldx, 0,
                                     s));
    HIP_TRY(hipStreamSynchronize(s));
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t id = ids[i];
        ix->has_vec[id >> 6] |= 1ull << (id & 63);
        ix->pending_host[id >> 6] |= 1ull << (id & 63);
        ix->n_rows = std::max(ix->n_rows, id + 1);
    }
    ix->bitmaps_dirty = true;
    int rc = rows_written(ix, d_ids, n, 0);
    if (rc) return rc;
    return pq_rows_written(ix, d_ids, ids, n, 0);
}

static int edit_tombstones(wv_index* ix, const uint64_t* ids, uint64_t n, bool add) {
    if (check(ix) || (n && !ids)) return fail(WV_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    for (uint64_t i = 0; i < n; ++i) {
        if (ids[i] >= ix->capacity) return fail(WV_EINVAL, "tombstone id beyond capacity");
        const uint64_t bit = 1ull << (ids[i] & 63);
        uint64_t& w = ix->tomb_host[ids[i] >> 6];
        if (add && !(w & bit)) { w |= bit; ix->n_tomb++; }
        else if (!add && (w & bit)) { w &= ~bit; ix->n_tomb--; }
    }
    ix->any_tomb = ix->n_tomb > 0;
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_add_tombstones(wv_index* ix, const uint64_t* ids, uint64_t n) { return edit_tombstones(ix, ids, n, true); }
int wv_index_remove_tombstones(wv_index* ix, const uint64_t* ids, uint64_t n) {
    return edit_tombstones(ix, ids, n, false);
}

int wv_index_delta_size(wv_index* ix, uint64_t* n) {
    if (check(ix) || !n) return fail(WV_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    int rc = refresh_bitmaps(ix);
    if (rc) return rc;
    *n = ix->delta_count;
    return WV_OK;
}

// Re-home a capacity-sized device buffer at new_bytes: the first old_bytes
// copied, the rest zeroed (an unused buffer stays unallocated).
static hipError_t regrow(DevBuf& b, size_t old_bytes, size_t new_bytes, hipStream_t s) {
    if (!b.p || new_bytes <= b.cap) return hipSuccess;
    void* np = nullptr;
    hipError_t e = hipMalloc(&np, new_bytes);
    if (e != hipSuccess) return e;
    old_bytes = std::min(old_bytes, b.cap);
    if (old_bytes) e = hipMemcpyAsync(np, b.p, old_bytes, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(static_cast<char*>(np) + old_bytes, 0, new_bytes - old_bytes, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { (void)hipFree(np); return e; }
    (void)hipFree(b.p);
    b.p = np;
    b.cap = new_bytes;
    return hipSuccess;
}

// Capacity growth in place (the mirror of a shard that outgrew its
// allocation; hnsw grows its node array the same way,
// maintainance.go:31-100 growIndexToAccomodateNode): every row, image, norm, code, tombstone and the
// graph stay; the queued work is drained first.
int wv_index_reserve(wv_index* ix, uint64_t capacity) {
    if (check(ix) || capacity >= (1ull << 31)) return fail(WV_EINVAL, "wv_index_reserve: bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    if (capacity <= ix->capacity) return WV_OK;
    HIP_TRY(hipSetDevice(ix->cfg.device));
    hipStream_t s = ix->stream;
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t old_rows = align_rows(ix->capacity);
    const uint64_t cap_rows = align_rows(capacity);
    const size_t ld4 = (size_t)ix->ldx * 4, img = (size_t)ix->h16_ns * 16 * 2;
    const uint64_t words = (capacity + 63) / 64;
    HIP_TRY(regrow(ix->vecs, old_rows * ld4, cap_rows * ld4, s));
    HIP_TRY(regrow(ix->xsplit, old_rows * ld4, cap_rows * ld4, s));
    HIP_TRY(regrow(ix->xnorm, old_rows * 4, cap_rows * 4, s));
    HIP_TRY(regrow(ix->xns, old_rows * 4, cap_rows * 4, s));
    HIP_TRY(regrow(ix->ximg16, old_rows * img, cap_rows * img, s));
    HIP_TRY(regrow(ix->pq_codes, ix->capacity * ix->pq_stride, capacity * ix->pq_stride, s));
    // bitmaps are rewritten from the host copies by the next refresh
    HIP_TRY(ix->tomb.ensure(words * 8));
    HIP_TRY(ix->excl.ensure((words + 4) * 8));
    ix->has_vec.resize(words, 0);
    ix->tomb_host.resize(words, 0);
    ix->pending_host.resize(words, 0);
    if (!ix->has_code.empty()) ix->has_code.resize(words, 0);
    if (!ix->nil_host.empty()) ix->nil_host.resize(words, ~0ull);
    ix->capacity = capacity;
    ix->bm_words = words;
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_capacity(const wv_index* ix, uint64_t* capacity, uint64_t* n_rows) {
    if (!ix) return fail(WV_EINVAL, "null index");
    if (capacity) *capacity = ix->capacity;
    if (n_rows) *n_rows = ix->n_rows;
    return WV_OK;
}

// level draw of the restatement (oracle/wv_oracle.c insert_node): a
// counter-based U(0,1) per id, targetLevel = floor(-ln(U) * 1/ln(M))
// (insert.go:132, index.go:226) -- identical levels on the CPU and the GPU
static int draw_level(uint64_t seed, uint64_t id, double normalizer) {
    auto mix = [](uint64_t x) {
        x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 27; x *= 0x94D049BB133111EBull;
        x ^= x >> 31;
        return x;
    };
    const uint64_t r = mix(seed * 0xD1B54A32D192ED03ull + id * 0x9E3779B97F4A7C15ull + 1);
    const double u = ((double)(r >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    const int t = (int)std::floor(-std::log(u) * normalizer);
    return t > 126 ? 126 : t;
}

int wv_index_build_graph(wv_index* ix, int ef_construction, uint64_t seed, int batch_div) {
    if (check(ix) || ef_construction < 1 || ef_construction > wv::HNSW_EF_MAX || batch_div < 1)
        return fail(WV_EINVAL, "wv_index_build_graph: bad argument");
    std::lock_guard<std::mutex> guard(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    hipStream_t s = ix->stream;
    const uint64_t n = ix->n_rows;
    if (n == 0) return fail(WV_ESTATE, "wv_index_build_graph: no vectors");
    for (uint64_t i = 0; i < n; ++i)
        if (!(ix->has_vec[i >> 6] & (1ull << (i & 63)))) return fail(WV_ESTATE, "wv_index_build_graph: a row has no vector");
    const int M = ix->cfg.max_connections, M0 = 2 * M;
    if (M < 2 || M0 > 256) return fail(WV_EINVAL, "wv_index_build_graph: maxConnections out of range");
    // levels: the first node is insertInitialElement's level 0 (insert.go:67-101)
    std::vector<int8_t> lv(n);
    const double norm = 1.0 / std::log((double)M);
    int maxL = 0;
    uint64_t n_upper = 0;
    std::vector<uint32_t> urow(n, WV_NIL);
    for (uint64_t i = 0; i < n; ++i) {
        lv[i] = (int8_t)(i == 0 ? 0 : draw_level(seed, i, norm));
        maxL = std::max<int>(maxL, lv[i]);
        if (lv[i] >= 1) urow[i] = (uint32_t)n_upper++;
    }
    const int ul = std::max(1, maxL);
    HIP_TRY(ix->levels.ensure(n));
    HIP_TRY(ix->layer0.ensure(n * (size_t)M0 * 4));
    HIP_TRY(ix->upper_row.ensure(n * 4));
    HIP_TRY(ix->upper.ensure(std::max<uint64_t>(1, n_upper) * ul * (size_t)M * 4));
    HIP_TRY(ix->b_cnt0.ensure(n * 4));
    HIP_TRY(ix->b_cntu.ensure(std::max<uint64_t>(1, n_upper) * ul * 4));
    HIP_TRY(hipMemsetAsync(ix->levels.p, 0xFF, n, s));   // -1: not inserted yet
    HIP_TRY(hipMemsetAsync(ix->layer0.p, 0xFF, n * (size_t)M0 * 4, s));
    HIP_TRY(hipMemsetAsync(ix->upper.p, 0xFF, std::max<uint64_t>(1, n_upper) * ul * (size_t)M * 4, s));
    HIP_TRY(hipMemsetAsync(ix->b_cnt0.p, 0, n * 4, s));
    HIP_TRY(hipMemsetAsync(ix->b_cntu.p, 0, std::max<uint64_t>(1, n_upper) * ul * 4, s));
    HIP_TRY(hipMemcpyAsync(ix->upper_row.p, urow.data(), n * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ix->levels.p, lv.data(), 1, hipMemcpyHostToDevice, s));   // node 0
    uint64_t ep = 0;
    int top = 0;
    // per-wave search state as in run_hnsw (unfiltered layout)
    const int efc = std::max(64, (ef_construction + 63) / 64 * 64);
    const int fixed = wv_hnsw_per_wave_words(ix->dpad, efc, 0, 0, 0) - 1;
    int vc_tbits = 0;
    const int vc_log2 = choose_vc_log2(12 * 1024 / 4, fixed, n, &vc_tbits);
    int per_wave = (wv_hnsw_per_wave_words(ix->dpad, efc, 0, vc_log2, 0) + 3) & ~3;
    int wpb = 4;
    while (wpb > 1 && (size_t)wpb * per_wave * 4 > 160 * 1024) --wpb;
    const int bmax = 16384;
    uint64_t done = 1;
    // WV_BUILD_TRACE=1 (diagnostic): per-phase device times (events) summed
    // over intervals of 64 batches, printed to stderr with the host time
    const bool trace = std::getenv("WV_BUILD_TRACE") != nullptr;
    hipEvent_t tev[5] = {};
    double tph[4] = {0, 0, 0, 0};
    uint64_t tbatches = 0, treq = 0, truns = 0;
    auto thost = std::chrono::steady_clock::now();
    if (trace)
        for (auto& e : tev) HIP_TRY(hipEventCreate(&e));
    while (done < n) {
        const int nb = (int)std::min<uint64_t>(n - done, std::max<uint64_t>(1, std::min<uint64_t>(bmax, done / batch_div)));
        int lb = 1;
        for (int i = 0; i < nb; ++i) lb = std::max(lb, lv[done + i] + 1);
        HIP_TRY(ix->b_tgt.ensure(nb));
        HIP_TRY(ix->b_ci.ensure((size_t)nb * lb * ef_construction * 4));
        HIP_TRY(ix->b_cd.ensure((size_t)nb * lb * ef_construction * 4));
        HIP_TRY(ix->b_cn.ensure((size_t)nb * lb * 4));
        const size_t nreq = (size_t)nb * lb * M;
        HIP_TRY(ix->b_rk.ensure(nreq * 8));
        HIP_TRY(ix->b_rn.ensure(nreq * 4));
        HIP_TRY(ix->b_rk2.ensure(nreq * 8));
        HIP_TRY(ix->b_rn2.ensure(nreq * 4));
        HIP_TRY(ix->b_uk.ensure(nreq * 8));
        HIP_TRY(ix->b_ul.ensure(nreq * 4));
        HIP_TRY(ix->b_uo.ensure(nreq * 4));
        HIP_TRY(ix->b_nr.ensure(8));
        HIP_TRY(hipMemcpyAsync(ix->b_tgt.p, lv.data() + done, nb, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemsetAsync(ix->b_cn.p, 0, (size_t)nb * lb * 4, s));
        wv::BuildParams b{};
        wv::HnswParams& h = b.h;
        h.X = ix->vecs.as<float>();
        h.levels = ix->levels.as<int8_t>();
        h.layer0 = ix->layer0.as<uint32_t>();
        h.upper_row = ix->upper_row.as<uint32_t>();
        h.upper = ix->upper.as<uint32_t>();
        h.N = done;
        h.entrypoint = (uint32_t)ep;
        h.D = ix->dim;
        h.ldx = ix->ldx;
        h.ldq = ix->dpad;
        h.metric = ix->metric;
        h.deg0 = M0;
        h.degU = M;
        h.max_level = top;
        h.upper_levels = ul;
        h.nq = nb;
        h.ef = ef_construction;
        h.efc = efc;
        h.sc = 0;
        h.vc_log2 = vc_log2;
        h.vc_tbits = vc_tbits;
        h.xs_log2 = 0;
        h.dpad = ix->dpad;
        h.per_wave_words = per_wave;
        b.first = done;
        b.nb = nb;
        b.lb = lb;
        b.M = M;
        b.M0 = M0;
        b.target = ix->b_tgt.as<int8_t>();
        b.cand_i = ix->b_ci.as<uint32_t>();
        b.cand_d = ix->b_cd.as<float>();
        b.cand_n = ix->b_cn.as<int32_t>();
        b.counts0 = ix->b_cnt0.as<uint32_t>();
        b.countsU = ix->b_cntu.as<uint32_t>();
        b.req_key = ix->b_rk.as<uint64_t>();
        b.req_node = ix->b_rn.as<uint32_t>();
        if (trace) HIP_TRY(hipEventRecord(tev[0], s));
        HIP_TRY(wv_launch_build_search(&b, wpb, s));
        if (trace) HIP_TRY(hipEventRecord(tev[1], s));
        HIP_TRY(wv_launch_build_select(&b, s));
        if (trace) HIP_TRY(hipEventRecord(tev[2], s));
        // reverse links grouped by (level, neighbour), batch order kept (stable)
        size_t tb = 0, tb2 = 0, tb3 = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ix->b_rk.as<uint64_t>(), ix->b_rk2.as<uint64_t>(),
                                                   ix->b_rn.as<uint32_t>(), ix->b_rn2.as<uint32_t>(), (int)nreq, 0, 64,
                                                   s));
        HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, tb2, ix->b_rk2.as<uint64_t>(), ix->b_uk.as<uint64_t>(),
                                                      ix->b_ul.as<uint32_t>(), ix->b_nr.as<uint32_t>(), (int)nreq, s));
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, ix->b_ul.as<uint32_t>(), ix->b_uo.as<uint32_t>(),
                                                 (int)nreq, s));
        HIP_TRY(ix->b_tmp.ensure(std::max(tb, std::max(tb2, tb3))));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(ix->b_tmp.p, tb, ix->b_rk.as<uint64_t>(), ix->b_rk2.as<uint64_t>(),
                                                   ix->b_rn.as<uint32_t>(), ix->b_rn2.as<uint32_t>(), (int)nreq, 0, 64,
                                                   s));
        HIP_TRY(hipMemsetAsync(ix->b_ul.p, 0, nreq * 4, s));
        HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(ix->b_tmp.p, tb2, ix->b_rk2.as<uint64_t>(),
                                                      ix->b_uk.as<uint64_t>(), ix->b_ul.as<uint32_t>(),
                                                      ix->b_nr.as<uint32_t>(), (int)nreq, s));
        HIP_TRY(hipcub::DeviceScan::ExclusiveSum(ix->b_tmp.p, tb3, ix->b_ul.as<uint32_t>(), ix->b_uo.as<uint32_t>(),
                                                 (int)nreq, s));
        uint32_t n_runs = 0;
        if (trace) HIP_TRY(hipEventRecord(tev[3], s));
        HIP_TRY(hipMemcpyAsync(&n_runs, ix->b_nr.p, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        b.run_key = ix->b_uk.as<uint64_t>();
        b.run_off = ix->b_uo.as<uint32_t>();
        b.run_len = ix->b_ul.as<uint32_t>();
        b.sorted_node = ix->b_rn2.as<uint32_t>();
        b.n_runs = (int)n_runs;
        HIP_TRY(wv_launch_build_link(&b, s));
        if (trace) {
            HIP_TRY(hipEventRecord(tev[4], s));
            HIP_TRY(hipEventSynchronize(tev[4]));
            for (int i = 0; i < 4; ++i) {
                float ms = 0.f;
                HIP_TRY(hipEventElapsedTime(&ms, tev[i], tev[i + 1]));
                tph[i] += ms;
            }
            ++tbatches;
            treq += nreq;
            truns += n_runs;
            if (tbatches % 64 == 0 || done + nb >= n) {
                const auto now = std::chrono::steady_clock::now();
                std::fprintf(stderr,
                             "[build] done %llu nb %d lb %d | %llu batches: host %.1f ms, search %.1f select %.1f "
                             "sort %.1f link %.1f ms, req %.2fM runs %.2fM\n",
                             (unsigned long long)(done + nb), nb, lb, (unsigned long long)tbatches,
                             std::chrono::duration<double, std::milli>(now - thost).count(), tph[0], tph[1], tph[2],
                             tph[3], treq / 1e6, truns / 1e6);
                thost = now;
                tph[0] = tph[1] = tph[2] = tph[3] = 0;
                tbatches = treq = truns = 0;
            }
        }
        // the batch is in the graph: its levels make it reachable for the next one
        HIP_TRY(hipMemcpyAsync(ix->levels.as<int8_t>() + done, lv.data() + done, nb, hipMemcpyHostToDevice, s));
        for (int i = 0; i < nb; ++i)   // insert.go:202-213: a higher node becomes the entrypoint
            if (lv[done + i] > top) { top = lv[done + i]; ep = done + i; }
        done += nb;
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (trace)
        for (auto& e : tev) HIP_TRY(hipEventDestroy(e));
    ix->nil_host.assign(ix->bm_words, ~0ull);
    for (uint64_t i = 0; i < lv.size(); ++i)
        if (lv[i] >= 0) ix->nil_host[i >> 6] &= ~(1ull << (i & 63));
    ix->gn = n;
    ix->deg0 = M0;
    ix->degU = M;
    ix->max_level = top;
    ix->n_upper = n_upper;
    ix->entrypoint = ep;
    ix->has_graph = true;
    ix->any_nil = false;
    for (uint64_t i = 0; i < n; ++i) ix->pending_host[i >> 6] &= ~(1ull << (i & 63));
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_download_graph(wv_index* ix, int8_t* levels, uint32_t* layer0, uint32_t* upper_row, uint32_t* upper) {
    if (check(ix) || !ix->has_graph) return fail(WV_ESTATE, "wv_index_download_graph: no graph");
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    hipStream_t s = ix->stream;
    const uint64_t n = ix->gn;
    if (levels) HIP_TRY(hipMemcpyAsync(levels, ix->levels.p, n, hipMemcpyDeviceToHost, s));
    if (layer0) HIP_TRY(hipMemcpyAsync(layer0, ix->layer0.p, n * (size_t)ix->deg0 * 4, hipMemcpyDeviceToHost, s));
    if (upper_row) HIP_TRY(hipMemcpyAsync(upper_row, ix->upper_row.p, n * 4, hipMemcpyDeviceToHost, s));
    if (upper && ix->max_level > 0)
        HIP_TRY(hipMemcpyAsync(upper, ix->upper.p, ix->n_upper * (size_t)ix->max_level * ix->degU * 4,
                               hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return WV_OK;
}

int wv_index_graph_info(wv_index* ix, uint64_t* n, int* deg0, int* degU, int* max_level, uint64_t* n_upper,
                        uint64_t* entrypoint) {
    if (check(ix) || !ix->has_graph) return fail(WV_ESTATE, "wv_index_graph_info: no graph");
    if (n) *n = ix->gn;
    if (deg0) *deg0 = ix->deg0;
    if (degU) *degU = ix->degU;
    if (max_level) *max_level = ix->max_level;
    if (n_upper) *n_upper = ix->n_upper;
    if (entrypoint) *entrypoint = ix->entrypoint;
    return WV_OK;
}

// ---- product quantization ---------------------------------
namespace {
// NewProductQuantizer (ssdhelpers/product_quantization.go:116-179) and
// ExtractCode (:191-237), read on the host: bits = int(log2 ks), bytes =
// int(log2(ks-1))/8 + 1; whole-byte codes are big-endian `bytes`-wide fields,
// bit-packed ones (useBitsEncoding, bits < 8*bytes) are cut from the
// (bytes+1)-byte big-endian word at index*bits/8.
struct CodeLayout {
    int bits = 0, bytes = 0;
    bool packed = false;
    bool init(int ks, bool use_bits) {
        if (ks < 2 || ks > 65536) return false;
        bits = (int)std::floor(std::log2((double)ks));
        bytes = (int)std::floor(std::log2((double)(ks - 1))) / 8 + 1;
        packed = use_bits && bits != 8 * bytes;
        return true;
    }
    static uint64_t be(const uint8_t* p, int nb) {
        uint64_t v = 0;
        for (int i = 0; i < nb; ++i) v = (v << 8) | p[i];
        return v;
    }
    uint64_t get(const uint8_t* enc, int index) const {
        if (!packed) return be(enc + (size_t)index * bytes, bytes);
        uint64_t code = be(enc + (size_t)index * bits / 8, bytes + 1);
        const int rest = (index + 1) * bits % 8, from_start = index * bits % 8;
        code >>= from_start < rest ? 16 - rest : 8 - rest;
        return code & ((1ull << bits) - 1);
    }
};
}  // namespace

int wv_pq_code_len(int segments, int centroids, int use_bits_encoding) {
    CodeLayout L;
    if (segments <= 0 || !L.init(centroids, use_bits_encoding != 0)) return -1;
    return segments * L.bytes;   // ProductQuantizer.Encode allocates m * bytes (:348-354)
}

int wv_index_set_pq(wv_index* ix, int segments, int centroids, int use_bits_encoding, int encoder,
                    const float* centroid_table) {
    CodeLayout L;
    if (check(ix) || !centroid_table || segments <= 0 || ix->dim % segments || !L.init(centroids, use_bits_encoding) ||
        (encoder != WV_PQ_TILE && encoder != WV_PQ_KMEANS))
        return fail(WV_EINVAL, "wv_index_set_pq: bad argument (segments must divide dims, 2 <= centroids <= 65536)");
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    ix->pq_m = segments;
    ix->pq_ks = centroids;
    ix->pq_ds = ix->dim / segments;
    ix->pq_encoder = encoder;
    ix->pq_use_bits = use_bits_encoding != 0;
    ix->pq_stride = centroids > 256 ? ((2 * (uint64_t)segments + 7) & ~7ull) : (((uint64_t)segments + 3) & ~3ull);
    const size_t tbytes = (size_t)segments * centroids * ix->pq_ds * 4;
    HIP_TRY(ix->pq_cent.ensure(tbytes));
    HIP_TRY(ix->pq_codes.ensure(ix->capacity * ix->pq_stride));
    HIP_TRY(hipMemcpyAsync(ix->pq_cent.p, centroid_table, tbytes, hipMemcpyHostToDevice, ix->stream));
    HIP_TRY(hipMemsetAsync(ix->pq_codes.p, 0, ix->capacity * ix->pq_stride, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    ix->has_code.assign(ix->bm_words, 0);
    ix->pq_set = true;
    ix->pq_on = false;
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_upload_pq_codes(wv_index* ix, const uint8_t* encoded, uint64_t n, uint64_t first_id) {
    if (check(ix) || (n && !encoded)) return fail(WV_EINVAL, "wv_index_upload_pq_codes: bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    if (!ix->pq_set) return fail(WV_ESTATE, "wv_index_upload_pq_codes: no quantizer (wv_index_set_pq)");
    if (first_id + n > ix->capacity) return fail(WV_EINVAL, "wv_index_upload_pq_codes: beyond capacity");
    if (n == 0) return WV_OK;
    HIP_TRY(hipSetDevice(ix->cfg.device));
    CodeLayout L;
    L.init(ix->pq_ks, ix->pq_use_bits);
    const size_t len = (size_t)ix->pq_m * L.bytes;
    std::vector<uint8_t> row(len + 8, 0), out(n * ix->pq_stride, 0);
    for (uint64_t r = 0; r < n; ++r) {
        std::memcpy(row.data(), encoded + r * len, len);   // zero tail: the packed reader looks one byte ahead
        uint8_t* dst = out.data() + r * ix->pq_stride;
        for (int i = 0; i < ix->pq_m; ++i) {
            const uint64_t c = L.get(row.data(), i);
            if (c >= (uint64_t)ix->pq_ks) return fail(WV_EINVAL, "wv_index_upload_pq_codes: code out of range");
            if (ix->pq_ks > 256) reinterpret_cast<uint16_t*>(dst)[i] = (uint16_t)c;
            else dst[i] = (uint8_t)c;
        }
    }
    HIP_TRY(hipMemcpyAsync(ix->pq_codes.as<uint8_t>() + first_id * ix->pq_stride, out.data(), out.size(),
                           hipMemcpyHostToDevice, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    for (uint64_t i = first_id; i < first_id + n; ++i) ix->has_code[i >> 6] |= 1ull << (i & 63);
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_pq_encode(wv_index* ix) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    if (!ix->pq_set || ix->pq_encoder != WV_PQ_KMEANS)
        return fail(WV_ESTATE, "wv_index_pq_encode: needs a KMeans quantizer (wv_index_set_pq)");
    HIP_TRY(hipSetDevice(ix->cfg.device));
    wv::PqParams pq = pq_params(ix);
    HIP_TRY(wv_launch_pq_encode(ix->vecs.as<float>(), ix->ldx, nullptr, ix->n_rows, &pq, ix->pq_codes.as<uint8_t>(),
                                ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    for (uint64_t w = 0; w < ix->bm_words; ++w) ix->has_code[w] |= ix->has_vec[w];
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_index_download_pq_codes(wv_index* ix, uint16_t* out, uint64_t first_id, uint64_t n) {
    if (check(ix) || (n && !out)) return fail(WV_EINVAL, "wv_index_download_pq_codes: bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    if (!ix->pq_set) return fail(WV_ESTATE, "wv_index_download_pq_codes: no quantizer");
    if (first_id + n > ix->capacity) return fail(WV_EINVAL, "wv_index_download_pq_codes: beyond capacity");
    HIP_TRY(hipSetDevice(ix->cfg.device));
    std::vector<uint8_t> raw(n * ix->pq_stride);
    HIP_TRY(hipMemcpyAsync(raw.data(), ix->pq_codes.as<uint8_t>() + first_id * ix->pq_stride, raw.size(),
                           hipMemcpyDeviceToHost, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    for (uint64_t r = 0; r < n; ++r)
        for (int i = 0; i < ix->pq_m; ++i) {
            const uint8_t* src = raw.data() + r * ix->pq_stride;
            out[r * ix->pq_m + i] = ix->pq_ks > 256 ? reinterpret_cast<const uint16_t*>(src)[i] : src[i];
        }
    return WV_OK;
}

int wv_index_set_compressed(wv_index* ix, int on) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    if (on) {
        if (!ix->pq_set) return fail(WV_ESTATE, "wv_index_set_compressed: no quantizer (wv_index_set_pq)");
        for (uint64_t w = 0; w < ix->bm_words; ++w)
            if (ix->has_vec[w] & ~ix->has_code[w])
                return fail(WV_ESTATE, "wv_index_set_compressed: a row with a vector has no code");
    }
    ix->pq_on = on != 0;
    ix->bitmaps_dirty = true;
    return WV_OK;
}

int wv_search_time_ef(const wv_index* ix, int k) { return ix ? search_time_ef(ix->cfg, k) : -1; }
int wv_config_search_time_ef(const wv_config* cfg, int k) { return cfg ? search_time_ef(*cfg, k) : -1; }

namespace {
// one pinned staging slot of wv_search_batch, returned when the call ends
struct SlotLease {
    wv_index* ix;
    wv_index::HostSlot* sl = nullptr;
    explicit SlotLease(wv_index* x) : ix(x) {
        std::unique_lock<std::mutex> l(ix->slot_mu);
        ix->slot_cv.wait(l, [&] {
            for (auto& c : ix->slots)
                if (!c.busy) return true;
            return false;
        });
        for (auto& c : ix->slots)
            if (!c.busy) { sl = &c; break; }
        sl->busy = true;
    }
    ~SlotLease() {
        std::lock_guard<std::mutex> l(ix->slot_mu);
        sl->busy = false;
        ix->slot_cv.notify_one();
    }
};
}  // namespace

int wv_search_batch(wv_index* ix, const float* queries, int nq, int k, int ef, const uint64_t* allow_bits,
                    uint64_t allow_nbits, uint64_t allow_stride_words, int mode, uint64_t* out_ids, float* out_dists,
                    int32_t* out_n) {
    if (check(ix) || nq < 0 || k <= 0 || (nq && (!queries || !out_ids || !out_dists || !out_n)))
        return fail(WV_EINVAL, "wv_search_batch: bad argument");
    if (nq == 0) return WV_OK;
    const uint64_t words = (allow_nbits + 63) / 64;
    const uint64_t arows = allow_bits ? (allow_stride_words ? (uint64_t)nq : 1) : 0;
    const uint64_t astride = allow_stride_words ? allow_stride_words : words;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t qb = (size_t)nq * ix->dim * 4, ab = arows * astride * 8, ib = (size_t)nq * k * 8,
                 db = (size_t)nq * k * 4, nb = (size_t)nq * 4;
    const size_t o_a = al(qb), o_i = o_a + al(ab), o_d = o_i + al(ib), o_n = o_d + al(db), need = o_n + al(nb);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    SlotLease lease(ix);
    wv_index::HostSlot& sl = *lease.sl;
    if (sl.cap < need) {
        if (sl.pin) HIP_TRY(hipHostFree(sl.pin));
        sl.pin = nullptr;
        sl.cap = 0;
        const size_t want = std::max<size_t>(need + need / 4, 1 << 20);
        HIP_TRY(hipHostMalloc(&sl.pin, want, hipHostMallocDefault));
        sl.cap = want;
    }
    if (!sl.done) HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    char* pin = static_cast<char*>(sl.pin);
    std::memcpy(pin, queries, qb);
    if (ab) std::memcpy(pin + o_a, allow_bits, ab);
    {
        std::lock_guard<std::mutex> g(ix->mu);
        HIP_TRY(hipSetDevice(ix->cfg.device));
        hipStream_t s = ix->stream;
        const float* dq = nullptr;
        int rc = stage_queries(ix, reinterpret_cast<const float*>(pin), nq, &dq, s);
        if (rc) return rc;
        const uint64_t* dallow = nullptr;
        if (ab) {
            // an AUTO batch with per-query allow lists gathers into g_allow:
            // keep the caller's bitmaps in their own buffer then
            DevBuf& dst = allow_stride_words && mode == WV_MODE_AUTO ? ix->allow_keep : ix->g_allow;
            HIP_TRY(dst.ensure(ab));
            HIP_TRY(hipMemcpyAsync(dst.p, pin + o_a, ab, hipMemcpyHostToDevice, s));
            dallow = dst.as<uint64_t>();
        }
        HIP_TRY(ix->out_ids.ensure(ib));
        HIP_TRY(ix->out_d.ensure(db));
        HIP_TRY(ix->out_n.ensure(nb));
        rc = search_core(ix, dq, nq, k, ef, dallow, allow_nbits, allow_stride_words, mode, ix->out_ids.as<uint64_t>(),
                         ix->out_d.as<float>(), ix->out_n.as<int32_t>(), s);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(pin + o_i, ix->out_ids.p, ib, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(pin + o_d, ix->out_d.p, db, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(pin + o_n, ix->out_n.p, nb, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(sl.done, s));
    }
    // the index is free for the next batch while this one finishes
    HIP_TRY(hipEventSynchronize(sl.done));
    std::memcpy(out_ids, pin + o_i, ib);
    std::memcpy(out_dists, pin + o_d, db);
    std::memcpy(out_n, pin + o_n, nb);
    return WV_OK;
}

int wv_search_batch_device(wv_index* ix, const float* d_queries, int nq, int k, int ef, const uint64_t* d_allow_bits,
                           uint64_t allow_nbits, uint64_t allow_stride_words, int mode, uint64_t* d_out_ids,
                           float* d_out_dists, int32_t* d_out_n, void* stream) {
    if (check(ix) || nq < 0 || k <= 0 || (nq && (!d_queries || !d_out_ids || !d_out_dists || !d_out_n)))
        return fail(WV_EINVAL, "wv_search_batch_device: bad argument");
    if (nq == 0) return WV_OK;
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    hipStream_t s = stream ? (hipStream_t)stream : ix->stream;
    const bool foreign = s != ix->stream;
    if (foreign) {
        if (!ix->ev_in) {
            HIP_TRY(hipEventCreateWithFlags(&ix->ev_in, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&ix->ev_out, hipEventDisableTiming));
        }
        HIP_TRY(hipEventRecord(ix->ev_in, ix->stream));
        HIP_TRY(hipStreamWaitEvent(s, ix->ev_in, 0));
    } else {
        // NULL: the index's own (non-blocking) stream, which would not wait
        // for work the caller queued on the legacy default stream -- e.g. a
        // torch kernel that just wrote d_queries: order after it explicitly
        if (!ix->ev_null) HIP_TRY(hipEventCreateWithFlags(&ix->ev_null, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ix->ev_null, nullptr));
        HIP_TRY(hipStreamWaitEvent(s, ix->ev_null, 0));
    }
    const float* dq = d_queries;
    int rc = WV_OK;
    if (ix->metric == WV_COSINE_DOT) {
        // the caller's rows are [nq][dpad]; normalize a padded copy
        HIP_TRY(ix->q_norm.ensure((size_t)nq * ix->dpad * 4));
        HIP_TRY(launch_pad_rows(d_queries, ix->dpad, nq, ix->dim, ix->q_norm.as<float>(), ix->dpad, s));
        HIP_TRY(wv_launch_normalize(ix->q_norm.as<float>(), ix->q_norm.as<float>(), nq, ix->dim, ix->dpad, s));
        dq = ix->q_norm.as<float>();
    }
    rc = search_core(ix, dq, nq, k, ef, d_allow_bits, allow_nbits, allow_stride_words, mode, d_out_ids, d_out_dists,
                     d_out_n, s);
    if (foreign) {
        HIP_TRY(hipEventRecord(ix->ev_out, s));
        HIP_TRY(hipStreamWaitEvent(ix->stream, ix->ev_out, 0));
    }
    return rc;
}

int wv_index_query_ld(const wv_index* ix) { return ix ? ix->dpad : -1; }

int wv_index_synchronize(wv_index* ix) {
    if (check(ix)) return fail(WV_EINVAL, "wv_index_synchronize: bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    return WV_OK;
}

int wv_search_by_vector(wv_index* ix, const float* vector, int k, const uint64_t* allow_bits, uint64_t allow_nbits,
                        uint64_t* out_ids, float* out_dists, int32_t* out_n) {
    return wv_search_batch(ix, vector, 1, k, 0, allow_bits, allow_nbits, 0, WV_MODE_AUTO, out_ids, out_dists, out_n);
}

// SearchByVectorDistance (search.go:90-158) for a batch of queries, on the
// device: round 1 (limit 100) is the batch's SearchByVector where it would
// run HNSW; every exact round -- round 1 of a flat search, and all rounds
// past the first (limit 1100, 11100, ...: their ef exceeds the beam) -- is
// answered by one threshold pass + segmented sort (wv_sbd.hip), launched
// beside round 1 so the batch syncs once.  The rounds' arithmetic
// (searchByDistParams, :552-619) then runs on the host over the counts.  A
// query whose within-target set outgrows its list (WV_SBD_CAP, 16384) or a
// compressed index takes the per-query path.
namespace {
// the search.go:90-158 loop over an exact sorted list (from round r0: 1 when
// round 1 is exact too, 2 after an HNSW round 1): the end of the kept prefix
int64_t sbd_exact_rounds(int r0, int64_t Qn, int64_t A, int64_t n, int64_t max_limit) {
    int64_t prev = 0, total = 100, limit = 100, kept = r0 == 1 ? 0 : 100;
    for (int r = 1;; ++r) {
        if (r > 1) {
            prev = total;
            limit *= 10;
            total = prev + limit;
            if (max_limit >= 0 && total > max_limit) break;   // maxLimitReached
        }
        if (total > (int64_t)1 << 40) break;
        if (r < r0) continue;
        const int64_t lo = std::min(prev, n), hi = std::min(total, n);
        if (hi - lo <= 0) break;
        kept = std::max(lo, std::min(hi, Qn));   // (appending stops at the first entry past the target)
        if (!(hi <= A)) break;                   // lastFound <= target
    }
    return kept;
}
}  // namespace

int wv_search_by_vector_distance_batch(wv_index* ix, const float* queries, int nq, const float* targets,
                                       int64_t max_limit, const uint64_t* allow_bits, uint64_t allow_nbits,
                                       uint64_t allow_stride_words, uint64_t* out_ids, float* out_dists,
                                       int64_t out_cap, int64_t* out_n) {
    if (check(ix) || nq < 0 || out_cap < 0 || (nq && (!queries || !targets || !out_n)) ||
        (out_cap && nq && (!out_ids || !out_dists)))
        return fail(WV_EINVAL, "wv_search_by_vector_distance_batch: bad argument");
    if (nq == 0) return WV_OK;
    HIP_TRY(hipSetDevice(ix->cfg.device));
    const uint64_t words = (allow_nbits + 63) / 64;
    const uint64_t astride = allow_stride_words ? allow_stride_words : words;
    auto allow_of = [&](int q) -> const uint64_t* {
        return allow_bits ? allow_bits + (allow_stride_words ? (uint64_t)q * allow_stride_words : 0) : nullptr;
    };
    std::vector<int> legacy;   // queries for the per-query path
    std::vector<int> hnsw_q;   // queries whose round 1 is an HNSW search
    {
        std::lock_guard<std::mutex> g(ix->mu);
        if (ix->pq_on) {
            for (int q = 0; q < nq; ++q) legacy.push_back(q);
        } else {
            const int ef = search_time_ef(ix->cfg, 100);
            const bool can_hnsw = ix->has_graph && ef <= wv::HNSW_EF_MAX;
            for (int q = 0; q < nq; ++q) {
                bool flat = !can_hnsw;
                if (!flat && allow_bits && !ix->cfg.forbid_flat) {
                    // allowList.Len() < flatSearchCutoff (search.go:74-78)
                    const uint64_t* a = allow_of(q);
                    uint64_t c = 0;
                    for (uint64_t w = 0; w < words; ++w) c += (uint64_t)__builtin_popcountll(a[w]);
                    flat = (int64_t)c < ix->cfg.flat_search_cutoff;
                }
                if (!flat) hnsw_q.push_back(q);
            }
        }
    }
    if ((int)legacy.size() < nq) {
        int cap = 16384;
        if (const char* e = std::getenv("WV_SBD_CAP")) cap = std::max(128, std::atoi(e));
        const int nh = (int)hnsw_q.size();
        std::vector<float> hq((size_t)std::max(nh, 1) * ix->dim);
        std::vector<uint64_t> hallow;
        for (int i = 0; i < nh; ++i)
            std::memcpy(hq.data() + (size_t)i * ix->dim, queries + (size_t)hnsw_q[i] * ix->dim, 4 * (size_t)ix->dim);
        if (allow_bits && allow_stride_words && nh) {
            hallow.resize((size_t)nh * astride);
            for (int i = 0; i < nh; ++i)
                std::memcpy(hallow.data() + (size_t)i * astride, allow_of(hnsw_q[i]), 8 * astride);
        }
        std::vector<uint64_t> r1_ids((size_t)std::max(nh, 1) * 100);
        std::vector<float> r1_d((size_t)std::max(nh, 1) * 100);
        std::vector<int32_t> r1_n(std::max(nh, 1));
        std::vector<unsigned int> cnt(3 * (size_t)nq);
        std::vector<std::vector<unsigned long long>> lists(nq);
        {
            std::lock_guard<std::mutex> g(ix->mu);
            hipStream_t s = ix->stream;
            int rc = refresh_bitmaps(ix);
            if (rc) return rc;
            const uint64_t* dallow = nullptr;
            if (allow_bits) {
                const size_t ab = (allow_stride_words ? (size_t)nq : 1) * astride * 8;
                HIP_TRY(ix->allow_keep.ensure(ab));
                HIP_TRY(hipMemcpyAsync(ix->allow_keep.p, allow_bits, ab, hipMemcpyHostToDevice, s));
                dallow = ix->allow_keep.as<uint64_t>();
            }
            // every query's threshold pass (its queries staged first: round
            // 1's search restages q_in)
            const float* dq = nullptr;
            rc = stage_queries(ix, queries, nq, &dq, s);
            if (rc) return rc;
            HIP_TRY(ix->sbd_q.ensure((size_t)nq * ix->dpad * 4));
            HIP_TRY(hipMemcpyAsync(ix->sbd_q.p, dq, (size_t)nq * ix->dpad * 4, hipMemcpyDeviceToDevice, s));
            HIP_TRY(ix->sbd_t.ensure((size_t)nq * 4));
            HIP_TRY(hipMemcpyAsync(ix->sbd_t.p, targets, (size_t)nq * 4, hipMemcpyHostToDevice, s));
            HIP_TRY(ix->sbd_keys.ensure((size_t)nq * cap * 8));
            HIP_TRY(ix->sbd_tmp.ensure((size_t)nq * cap * 8));
            HIP_TRY(ix->sbd_cnt.ensure((size_t)nq * 12));
            HIP_TRY(ix->sbd_off.ensure((size_t)nq * 8));
            HIP_TRY(hipMemsetAsync(ix->sbd_cnt.p, 0, (size_t)nq * 12, s));
            wv::SbdParams sp{};
            sp.X = ix->vecs.as<float>();
            sp.Q = ix->sbd_q.as<float>();
            sp.target = ix->sbd_t.as<float>();
            sp.excl = ix->excl.as<uint64_t>();
            sp.excl_nbits = ix->capacity;
            sp.allow = dallow;
            sp.allow_nbits = allow_nbits;
            sp.allow_stride = allow_stride_words;
            sp.N = ix->n_rows;
            sp.D = ix->dim;
            sp.ldx = ix->ldx;
            sp.dpad = ix->dpad;
            sp.metric = ix->metric;
            sp.nq = nq;
            // ~4 blocks per CU over the batch, whole 4-wave steps of 256 rows
            const uint64_t target_blocks = std::max<uint64_t>(1, (uint64_t)ix->n_cus * 4 / (uint64_t)nq);
            sp.rows_per_block = std::max<uint64_t>(4096, (sp.N + target_blocks - 1) / target_blocks);
            sp.rows_per_block = (sp.rows_per_block + 255) / 256 * 256;
            while ((sp.N + sp.rows_per_block - 1) / sp.rows_per_block > 65535) sp.rows_per_block *= 2;
            sp.cap = cap;
            sp.keys = ix->sbd_keys.as<unsigned long long>();
            sp.cnt = ix->sbd_cnt.as<unsigned int>();
            HIP_TRY(wv_launch_sbd_scan(&sp, s));
            HIP_TRY(wv_sbd_sort(ix->sbd_keys.as<unsigned long long>(), ix->sbd_tmp.as<unsigned long long>(),
                                ix->sbd_cnt.as<unsigned int>(), nq, cap, ix->sbd_off.as<int>(), &ix->sbd_scr,
                                &ix->sbd_scr_cap, s));
            // round 1 of the HNSW queries: their SearchByVector(limit 100)
            if (nh) {
                rc = stage_queries(ix, hq.data(), nh, &dq, s);
                if (rc) return rc;
                const uint64_t* dal = dallow;
                if (allow_bits && allow_stride_words) {
                    HIP_TRY(ix->g_allow.ensure(hallow.size() * 8));
                    HIP_TRY(hipMemcpyAsync(ix->g_allow.p, hallow.data(), hallow.size() * 8, hipMemcpyHostToDevice, s));
                    dal = ix->g_allow.as<uint64_t>();
                }
                HIP_TRY(ix->out_ids.ensure((size_t)nh * 100 * 8));
                HIP_TRY(ix->out_d.ensure((size_t)nh * 100 * 4));
                HIP_TRY(ix->out_n.ensure((size_t)nh * 4));
                rc = search_core(ix, dq, nh, 100, 0, dal, allow_nbits, allow_stride_words, WV_MODE_AUTO,
                                 ix->out_ids.as<uint64_t>(), ix->out_d.as<float>(), ix->out_n.as<int32_t>(), s);
                if (rc) return rc;
                HIP_TRY(hipMemcpyAsync(r1_ids.data(), ix->out_ids.p, (size_t)nh * 100 * 8, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipMemcpyAsync(r1_d.data(), ix->out_d.p, (size_t)nh * 100 * 4, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipMemcpyAsync(r1_n.data(), ix->out_n.p, (size_t)nh * 4, hipMemcpyDeviceToHost, s));
            }
            HIP_TRY(hipMemcpyAsync(cnt.data(), ix->sbd_cnt.p, (size_t)nq * 12, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            // the sorted lists, as far as the rounds keep them (and the caller
            // takes them)
            std::vector<int64_t> need(nq, 0);
            std::vector<char> is_h(nq, 0);
            for (int q : hnsw_q) is_h[q] = 1;
            std::vector<int> hs(nq, -1);
            for (int i = 0; i < nh; ++i) hs[hnsw_q[i]] = i;
            for (int q = 0; q < nq; ++q) {
                const int64_t Qn = cnt[3 * q], A = cnt[3 * q + 1], n = cnt[3 * q + 2];
                if (is_h[q]) {   // (an HNSW round 1 that ends the deepening needs no list)
                    const int i = hs[q];
                    const int64_t hi = std::min<int64_t>(100, r1_n[i]);
                    if (!(hi > 0 && r1_d[(size_t)i * 100 + hi - 1] <= targets[q] && (max_limit < 0 || 1100 <= max_limit)))
                        continue;
                }
                const int64_t kept = sbd_exact_rounds(is_h[q] ? 2 : 1, Qn, A, n, max_limit);
                need[q] = std::min<int64_t>(kept, Qn);
                if (Qn > cap && need[q] > 0) { legacy.push_back(q); need[q] = 0; continue; }
                if (need[q] > 0) {
                    lists[q].resize(need[q]);
                    HIP_TRY(hipMemcpyAsync(lists[q].data(), ix->sbd_tmp.as<unsigned long long>() + (size_t)q * cap,
                                           8 * need[q], hipMemcpyDeviceToHost, s));
                }
            }
            HIP_TRY(hipStreamSynchronize(s));
        }
        std::vector<int> hslot(nq, -1);
        for (int i = 0; i < nh; ++i) hslot[hnsw_q[i]] = i;
        const uint64_t id_base = ix->cfg.id_base;
        for (int q = 0; q < nq; ++q) {
            if (std::find(legacy.begin(), legacy.end(), q) != legacy.end()) continue;
            const float t = targets[q];
            int64_t m = 0;
            auto put = [&](uint64_t id, float d) {
                if (m < out_cap) { out_ids[(size_t)q * out_cap + m] = id; out_dists[(size_t)q * out_cap + m] = d; }
                m++;
            };
            auto qual = [&](float d) { return d <= t || std::fabs((double)d - (double)t) <= 1e-6; };
            bool exact_more = true;
            if (hslot[q] >= 0) {
                // round 1 from the HNSW search: its qualifying prefix, and
                // whether the deepening continues
                const int i = hslot[q];
                const int64_t hi = std::min<int64_t>(100, r1_n[i]);
                for (int64_t j = 0; j < hi; ++j) {
                    const float d = r1_d[(size_t)i * 100 + j];
                    if (!qual(d)) break;
                    put(r1_ids[(size_t)i * 100 + j], d);
                }
                exact_more = hi > 0 && r1_d[(size_t)i * 100 + hi - 1] <= t && (max_limit < 0 || 1100 <= max_limit);
            }
            if (exact_more) {
                const int64_t from = hslot[q] >= 0 ? 100 : 0;
                for (int64_t j = from; j < (int64_t)lists[q].size(); ++j) {
                    const unsigned long long key = lists[q][j];
                    uint32_t u = (uint32_t)(key >> 32);
                    u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
                    float d;
                    std::memcpy(&d, &u, 4);
                    put(id_base + (uint32_t)key, d);
                }
            }
            out_n[q] = m;
        }
    }
    for (int q : legacy) {
        int rc = wv_search_by_vector_distance(ix, queries + (size_t)q * ix->dim, targets[q], max_limit, allow_of(q),
                                              allow_nbits, out_cap ? out_ids + (size_t)q * out_cap : nullptr,
                                              out_cap ? out_dists + (size_t)q * out_cap : nullptr, out_cap, out_n + q);
        if (rc) return rc;
    }
    return WV_OK;
}

int wv_search_by_vector_distance(wv_index* ix, const float* vector, float target, int64_t max_limit,
                                 const uint64_t* allow_bits, uint64_t allow_nbits, uint64_t* out_ids,
                                 float* out_dists, int64_t out_cap, int64_t* out_n) {
    if (check(ix) || !vector || !out_n) return fail(WV_EINVAL, "bad argument");
    // search.go:90-158 with searchByDistParams (:552-619)
    int64_t offset = 0, limit = 100, total = 100, n_out = 0;
    std::vector<uint64_t> ids;
    std::vector<float> ds;
    std::vector<int32_t> nn(1);
    for (bool first = true;; first = false) {
        if (!first) {
            offset = total;
            limit *= 10;
            total = offset + limit;
            if (max_limit >= 0 && total > max_limit) break;
        }
        if (total > (int64_t)0x7FFFFFFF) break;
        ids.assign(total, 0);
        ds.assign(total, 0.f);
        int rc = wv_search_by_vector(ix, vector, (int)total, allow_bits, allow_nbits, ids.data(), ds.data(), nn.data());
        if (rc) return rc;
        const int64_t n = nn[0];
        const int64_t lo = std::min(offset, n), hi = std::min(total, n);
        if (hi - lo <= 0) break;
        const bool cont = ds[hi - 1] <= target;
        for (int64_t i = lo; i < hi; ++i) {
            if (ds[i] <= target || std::fabs((double)ds[i] - (double)target) <= 1e-6) {
                if (n_out < out_cap) { out_ids[n_out] = ids[i]; out_dists[n_out] = ds[i]; }
                n_out++;
            } else {
                break;
            }
        }
        if (!cont) break;
    }
    *out_n = n_out;
    return WV_OK;
}

int wv_merge_shards_device(const float* d_in_dists, const uint64_t* d_in_ids, const int32_t* d_in_n, int n_shards,
                           int nq, int k, float* d_out_dists, uint64_t* d_out_ids, int32_t* d_out_n, void* stream) {
    if (n_shards <= 0 || n_shards > 16 || nq < 0 || k <= 0) return fail(WV_EINVAL, "wv_merge_shards_device: bad argument");
    if (nq == 0) return WV_OK;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(merge_shards_kernel, dim3((nq + 127) / 128), dim3(128), 0, s, d_in_dists, d_in_ids, d_in_n,
                       n_shards, nq, k, d_out_dists, d_out_ids, d_out_n);
    HIP_TRY(hipGetLastError());
    return WV_OK;
}

int wv_index_set_timing(wv_index* ix, int enable) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    ix->timing = enable != 0;
    ix->ev_used = 0;
    return WV_OK;
}

// the recorded event sets -> per-batch averages (one sync, on request)
static int read_timing(wv_index* ix) {
    if (ix->ev_used == 0) return WV_OK;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    for (size_t b = 0; b < ix->ev_used; ++b) {
        const auto& e = ix->ev_pool[b];
        const uint8_t m = ix->ev_mask[b];
        for (int pr = 0; pr < 4; ++pr) {
            if ((m & (3u << (2 * pr))) != (3u << (2 * pr))) continue;
            HIP_TRY(hipEventSynchronize(e[2 * pr + 1]));
            float t = 0.f;
            HIP_TRY(hipEventElapsedTime(&t, e[2 * pr], e[2 * pr + 1]));
            a[pr] += t;
        }
    }
    const float inv = 1.0f / (float)ix->ev_used;
    ix->t_mfma = a[0] * inv;
    ix->t_fin = a[1] * inv;
    ix->t_hnsw = a[2] * inv;
    ix->t_pre = a[3] * inv;
    ix->ev_used = 0;
    return WV_OK;
}

int wv_last_kernel_times(wv_index* ix, float* bf_mfma_ms, float* bf_finalize_ms, float* hnsw_ms) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    int rc = read_timing(ix);
    if (rc) return rc;
    if (bf_mfma_ms) *bf_mfma_ms = ix->t_mfma;
    if (bf_finalize_ms) *bf_finalize_ms = ix->t_fin;
    if (hnsw_ms) *hnsw_ms = ix->t_hnsw;
    return WV_OK;
}

int wv_last_seed_time(wv_index* ix, float* seed_ms) {
    if (check(ix) || !seed_ms) return fail(WV_EINVAL, "bad argument");
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    int rc = read_timing(ix);
    if (rc) return rc;
    *seed_ms = ix->t_pre;
    return WV_OK;
}

int wv_last_batch_stats(wv_index* ix, uint64_t* dist_evals, uint64_t* expansions, uint64_t* fallbacks) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    unsigned long long acc[3] = {0, 0, 0};
    if (ix->stat_acc.p) {
        HIP_TRY(hipMemcpyAsync(acc, ix->stat_acc.p, 24, hipMemcpyDeviceToHost, ix->stat_stream));
        HIP_TRY(hipStreamSynchronize(ix->stat_stream));
    }
    if (dist_evals) *dist_evals = ix->last_dist + acc[0];
    if (expansions) *expansions = ix->last_exp + acc[1];
    if (fallbacks) *fallbacks = ix->last_fallbacks + acc[2];
    return WV_OK;
}

int wv_last_side_stats(wv_index* ix, uint64_t* overflowed, uint64_t* redone, uint64_t* claims, int* side_rows,
                       int* spill_cap) {
    if (check(ix)) return WV_EINVAL;
    std::lock_guard<std::mutex> g(ix->mu);
    HIP_TRY(hipSetDevice(ix->cfg.device));
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
    if (ix->stat_acc.p) {
        HIP_TRY(hipMemcpyAsync(acc, ix->stat_acc.p, 48, hipMemcpyDeviceToHost, ix->stat_stream));
        HIP_TRY(hipStreamSynchronize(ix->stat_stream));
    }
    if (overflowed) *overflowed = acc[3];
    if (redone) *redone = acc[4];
    if (claims) *claims = acc[5];
    if (side_rows) *side_rows = ix->last_side_rows;
    if (spill_cap) *spill_cap = ix->last_side_xs;
    return WV_OK;
}

}  // extern "C"
