// wv_sbd.hip -- SearchByVectorDistance on the device, batched
// (adapters/repos/db/vector/hnsw/search.go:90-158 with searchByDistParams,
// :552-619).
//
// The reference deepens: SearchByVector(limit 100), then 1100, 11100, ...,
// each round appending the entries [offset, total) that are within the target
// distance (or InDelta 1e-6 of it) and continuing while the round's last entry
// is <= target.  Every round past the first asks a limit whose ef exceeds the
// beam (1100 > HNSW_EF_MAX): on the GPU those rounds are exact, and an exact
// search's ranks [offset, total) are the ranks of the sorted set of rows within
// the target.  So one threshold pass answers every round past the first at
// once: per query, the allowed rows with d - target <= 1e-6 (float64, as
// floatcomp.InDelta) are appended to a per-query list with their sort keys,
// counted (|Q|, and A = those with d <= target), and the rows the search
// could return are counted too (n); a segmented sort orders the lists by
// (d, id).  The host then applies the rounds' arithmetic to |Q|, A and n.
// Distances are the reference-order exact ones (exact_dist_rows, bit-identical
// to the asm distancer).
#include "wv_device.h"
#include "wv_params.h"

#include <hipcub/hipcub.hpp>

namespace wv {

// SbdParams: wv_params.h


__device__ __forceinline__ unsigned long long sbd_key(float d, uint32_t row) {
    uint32_t u = d == 0.f ? 0u : __float_as_uint(d);   // (-0 and +0: one key)
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | row;
}

// grid (nq, row blocks), 256 threads: each wave takes 64 candidate rows a
// step, keeps the allowed ones, computes their distances 32 at a time and
// appends the ones within the target
template <int METRIC>
__global__ __launch_bounds__(256) void sbd_scan_kernel(SbdParams p) {
    __shared__ float qv[1024];
    __shared__ uint32_t ids[4][64];
    __shared__ float ds[4][64];
    const int q = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (q >= p.nq || p.dpad > 1024) return;
    for (int i = threadIdx.x; i < p.dpad; i += 256) qv[i] = p.Q[(uint64_t)q * p.dpad + i];
    __syncthreads();
    const double t = (double)p.target[q];
    const uint64_t* allow = p.allow ? p.allow + (p.allow_stride ? (uint64_t)q * p.allow_stride : 0) : nullptr;
    const uint64_t r_begin = (uint64_t)blockIdx.y * p.rows_per_block;
    uint64_t r_end = r_begin + p.rows_per_block;
    if (r_end > p.N) r_end = p.N;
    unsigned int n_a = 0, n_ok = 0;   // (lane 0's running counts)
    for (uint64_t r0 = r_begin + 64 * (uint64_t)wave; r0 < r_end; r0 += 256) {
        const uint64_t r = r0 + lane;
        bool ok = r < r_end && !bit_test(p.excl, p.excl_nbits, r);
        if (ok && allow) ok = bit_test(allow, p.allow_nbits, r);
        const uint64_t m = __ballot(ok);
        const int n = __popcll(m);
        if (ok) ids[wave][mbcnt64(m)] = (uint32_t)r;
        __builtin_amdgcn_wave_barrier();
        if (n == 0) continue;
        exact_dist_rows<METRIC, 4, true>(qv, p.X, p.ldx, p.D, ids[wave], n, ds[wave], lane);
        if (n > 32) exact_dist_rows<METRIC, 4, true>(qv, p.X, p.ldx, p.D, ids[wave] + 32, n - 32, ds[wave] + 32, lane);
        __builtin_amdgcn_wave_barrier();
        const float d = lane < n ? ds[wave][lane] : 0.f;
        const uint32_t id = lane < n ? ids[wave][lane] : 0u;
        const bool in = lane < n && (double)d - t <= 1e-6;
        const bool below = lane < n && d <= p.target[q];
        const uint64_t im = __ballot(in);
        const int ni = __popcll(im);
        unsigned int base = 0;
        if (ni) {
            if (lane == 0) base = atomicAdd(p.cnt + 3 * q, (unsigned int)ni);
            base = (unsigned int)__builtin_amdgcn_readfirstlane((int)base);
            const unsigned int pos = base + (unsigned int)mbcnt64(im);
            if (in && pos < (unsigned int)p.cap) p.keys[(uint64_t)q * p.cap + pos] = sbd_key(d, id);
        }
        n_a += (unsigned int)__popcll(__ballot(below));
        n_ok += (unsigned int)n;
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0 && n_a) atomicAdd(p.cnt + 3 * q + 1, n_a);
    if (lane == 0 && n_ok) atomicAdd(p.cnt + 3 * q + 2, n_ok);
}

// segment bounds of the sort: [q cap, q cap + min(|Q|, cap))
__global__ void sbd_offsets_kernel(const unsigned int* cnt, int nq, int cap, int* beg, int* end) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    beg[q] = q * cap;
    end[q] = q * cap + (int)min(cnt[3 * q], (unsigned int)cap);
}

}  // namespace wv

extern "C" {

hipError_t wv_launch_sbd_scan(const wv::SbdParams* p, hipStream_t s) {
    if (p->nq == 0 || p->N == 0) return hipSuccess;
    if (p->dpad > 1024) return hipErrorInvalidValue;
    const uint64_t blocks_y = (p->N + p->rows_per_block - 1) / p->rows_per_block;
    if (blocks_y > 65535) return hipErrorInvalidValue;
    const dim3 grid((unsigned)p->nq, (unsigned)blocks_y);
    if (p->metric == WV_METRIC_L2) hipLaunchKernelGGL(wv::sbd_scan_kernel<WV_METRIC_L2>, grid, dim3(256), 0, s, *p);
    else if (p->metric == WV_METRIC_DOT) hipLaunchKernelGGL(wv::sbd_scan_kernel<WV_METRIC_DOT>, grid, dim3(256), 0, s, *p);
    else hipLaunchKernelGGL(wv::sbd_scan_kernel<WV_METRIC_COSINE>, grid, dim3(256), 0, s, *p);
    return hipGetLastError();
}

// sort every query's list by (d, id): keys in place via tmp (same size)
hipError_t wv_sbd_sort(unsigned long long* keys, unsigned long long* tmp, const unsigned int* cnt, int nq, int cap,
                       int* offsets, void** scratch, size_t* scratch_cap, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(wv::sbd_offsets_kernel, dim3((nq + 255) / 256), dim3(256), 0, s, cnt, nq, cap, offsets,
                       offsets + nq);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t need = 0;
    e = hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, need, keys, tmp, nq * cap, nq, offsets, offsets + nq, 0,
                                                   64, s);
    if (e != hipSuccess) return e;
    if (need > *scratch_cap) {
        if (*scratch) (void)hipFree(*scratch);
        *scratch = nullptr;
        *scratch_cap = 0;
        e = hipMalloc(scratch, need);
        if (e != hipSuccess) return e;
        *scratch_cap = need;
    }
    return hipcub::DeviceSegmentedRadixSort::SortKeys(*scratch, need, keys, tmp, nq * cap, nq, offsets, offsets + nq,
                                                      0, 64, s);
}

}  // extern "C"
