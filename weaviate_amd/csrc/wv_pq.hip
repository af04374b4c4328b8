// wv_pq.hip -- product quantization on the device.
//
// adapters/repos/db/vector/ssdhelpers/product_quantization.go and kmeans.go:
//   * wv_pq_encode_kernel: ProductQuantizer.Encode (:348-354) with KMeans
//     encoders -- per (row, segment) the nearest centroid by asm.L2
//     (KMeans.Nearest, kmeans.go:78-110; among equal distances the LAST
//     centroid wins, as nNearest's `minD[j] < distance` scan replaces on ties).
//   * wv_pq_scan_kernel: flatSearch (hnsw/flat_search.go:19-74) on a
//     compressed index, where distBetweenNodeAndVec is the PQ distance
//     (hnsw/index.go:493-511): a chunk of queries x a row list -> (dist, j)
//     keys for a stable segmented radix sort, i.e. (dist, id) order.
//   * wv_pq_topk_kernel: the first k of every sorted segment.
// The HNSW kernel computes the same PQ distance per gathered row
// (wv_hnsw.hip, pq_dist_row in wv_device.h).
#include "wv_device.h"
#include "wv_params.h"

namespace wv {

// one thread per (row, segment); codes written in the device layout
// (u8 or u16 per segment, rows padded to pq.stride bytes)
__global__ __launch_bounds__(256) void wv_pq_encode_kernel(const float* __restrict__ X, int ldx,
                                                           const uint64_t* __restrict__ ids, uint64_t n_rows,
                                                           PqParams pq, uint8_t* __restrict__ codes) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t r = t / pq.m;
    const int seg = (int)(t % pq.m);
    if (r >= n_rows) return;
    const uint64_t row = ids ? ids[r] : r;   // a row list (hnsw.Add) or rows 0..n_rows-1
    const float* x = X + row * ldx + (uint64_t)seg * pq.ds;
    const float* cs = pq.cent + (uint64_t)seg * pq.ks * pq.ds;
    uint32_t best = 0;
    float bd = 3.40282346638528859812e+38f;   // math.MaxFloat32
    for (int c = 0; c < pq.ks; ++c) {
        const float d = asm_l2_serial(x, cs + (uint64_t)c * pq.ds, pq.ds);
        if (!(bd < d)) { bd = d; best = (uint32_t)c; }
    }
    uint8_t* dst = codes + row * pq.stride;
    if (pq.wide) reinterpret_cast<uint16_t*>(dst)[seg] = (uint16_t)best;
    else dst[seg] = (uint8_t)best;
}

template <int METRIC>
__device__ __forceinline__ void pq_scan_one(const PqScanParams& p, int qi, uint64_t j) {
    const int q = p.q0 + qi;
    const uint64_t o = (uint64_t)qi * p.nr + j;
    const uint32_t row = p.rows ? p.rows[j] : (uint32_t)j;
    bool ok = !bit_test(p.excl, p.excl_nbits, row);
    if (ok && p.allow) ok = bit_test(p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0), p.allow_nbits, row);
    float d = __builtin_inff(), key = __builtin_inff();
    if (ok) {
        d = pq_dist_row<METRIC>(p.Q + (uint64_t)q * p.ldq, p.pq, row);
        key = d == 0.f ? 0.f : d;   // -0 sorts with +0 (equal distances, id order)
    }
    p.key[o] = key;
    p.dist[o] = d;
    p.val[o] = (uint32_t)j;
}

// grid: x over rows, y over the queries of the chunk
__global__ __launch_bounds__(256) void wv_pq_scan_kernel(PqScanParams p) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int qi = blockIdx.y;
    if (j >= p.nr || qi >= p.nqc) return;
    if (p.metric == WV_METRIC_L2) pq_scan_one<WV_METRIC_L2>(p, qi, j);
    else if (p.metric == WV_METRIC_DOT) pq_scan_one<WV_METRIC_DOT>(p, qi, j);
    else pq_scan_one<WV_METRIC_COSINE>(p, qi, j);
}

// one block per query of the chunk: the first k sorted entries that are not
// excluded (+inf keys sort last)
__global__ __launch_bounds__(64) void wv_pq_topk_kernel(const float* __restrict__ skey, const uint32_t* __restrict__ sval,
                                                        const float* __restrict__ dist, const uint32_t* __restrict__ rows,
                                                        uint64_t nr, int q0, int k, uint64_t id_base,
                                                        uint64_t* __restrict__ out_ids, float* __restrict__ out_d,
                                                        int32_t* __restrict__ out_n) {
    const int qi = blockIdx.x;
    const int q = q0 + qi;
    const float* kk = skey + (uint64_t)qi * nr;
    const uint32_t* vv = sval + (uint64_t)qi * nr;
    const uint64_t lim = nr < (uint64_t)k ? nr : (uint64_t)k;
    int n = 0;
    for (uint64_t i = threadIdx.x; i < lim; i += blockDim.x) {
        if (kk[i] == __builtin_inff()) continue;
        const uint32_t j = vv[i];
        out_ids[(uint64_t)q * k + i] = id_base + (rows ? rows[j] : j);
        out_d[(uint64_t)q * k + i] = dist[(uint64_t)qi * nr + j];
        n = (int)i + 1;
    }
    // the count is the last valid position + 1 (entries are contiguous)
    for (int off = 32; off > 0; off >>= 1) n = max(n, __shfl_xor(n, off, 64));
    if (threadIdx.x == 0) out_n[q] = n;
}

}  // namespace wv

extern "C" {

hipError_t wv_launch_pq_encode(const float* X, int ldx, const uint64_t* ids, uint64_t n_rows, const wv::PqParams* pq,
                               uint8_t* codes, hipStream_t s) {
    const uint64_t total = n_rows * (uint64_t)pq->m;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_pq_encode_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, X, ldx, ids,
                       n_rows, *pq, codes);
    return hipGetLastError();
}

hipError_t wv_launch_pq_scan(const wv::PqScanParams* p, hipStream_t s) {
    if (p->nr == 0 || p->nqc == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_pq_scan_kernel, dim3((unsigned)((p->nr + 255) / 256), (unsigned)p->nqc), dim3(256), 0, s,
                       *p);
    return hipGetLastError();
}

hipError_t wv_launch_pq_topk(const float* skey, const uint32_t* sval, const float* dist, const uint32_t* rows,
                             uint64_t nr, int q0, int nqc, int k, uint64_t id_base, uint64_t* out_ids, float* out_d,
                             int32_t* out_n, hipStream_t s) {
    if (nqc == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::wv_pq_topk_kernel, dim3((unsigned)nqc), dim3(64), 0, s, skey, sval, dist, rows, nr, q0, k,
                       id_base, out_ids, out_d, out_n);
    return hipGetLastError();
}

}  // extern "C"
