// wv_h16_dev.h -- device helpers of the f16 key passes (wv_h16.hip): LDS-DMA
// as inline asm with counted waits, the tile eligibility words, the LDS stage
// layout.
#pragma once
#include "wv_device.h"
#include "wv_params.h"
#include "wv_topk.h"

#include <float.h>

namespace wv {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// LDS-DMA (global_load_lds_dword{,x4}) as inline asm: the destination is the
// wave-uniform LDS byte address in M0 (+ lane * size).  Written as asm so the
// compiler's waitcnt pass does not see them: for a builtin LDS-DMA it waits
// vmcnt(0) before every LDS read it cannot prove disjoint -- the prefetch of
// the next tiles would be drained before the current one is read.  The
// kernel places the (counted) vmcnt waits itself.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_wave_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_wave_base) : "memory");
}
// the same from a wave-uniform base (SGPR pair) + a per-lane 32-bit byte
// offset: a tile's address update is scalar work, no per-lane 64-bit adds
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_wave_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_wave_base) : "memory");
}
// a wave-uniform pointer the compiler cannot prove uniform, moved to SGPRs
template <class T>
__device__ __forceinline__ const T* uniform_ptr(const T* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const T*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void glds4(const void* src, uint32_t lds_wave_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_wave_base) : "memory");
}
// the same at device scope (sc1: past the CU's L1, so a word other CUs
// update with atomics is read from L2)
__device__ __forceinline__ void glds4_dev(const void* src, uint32_t lds_wave_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_wave_base) : "memory");
}
// the same from a wave-uniform base (SGPR pair) + a per-lane byte offset +
// an immediate (a loop of them keeps no per-iteration address registers)
template <int OFF>
__device__ __forceinline__ void glds4s_dev(const void* sbase, uint32_t voff, uint32_t lds_wave_base) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2 offset:%4 sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_wave_base), "i"(OFF) : "memory");
}
// wait until at most n of this wave's vector-memory ops are outstanding
__device__ __forceinline__ void vm_wait(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}
__device__ __forceinline__ void block_barrier() {
#ifdef WV_H16_ABLATE_NO_BARRIER
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
}

// Eligibility of a tile's 64 rows (bit r: row r is not excluded, is allowed,
// and is < N), read with scalar loads: the tile index is wave-uniform, so
// the words come through the constant address space (s_load), which neither
// waits behind the LDS operand reads (a word staged in LDS cost 0.31 ms per
// 1M x 10k pass: its read stalled the wave at every tile) nor counts against
// the LDS-DMA's vmcnt.
__device__ __forceinline__ uint64_t tile_okw(const H16Params& p, uint64_t tile, bool has_allow) {
    typedef const __attribute__((address_space(4))) uint64_t cu64;
    const uint32_t tl = __builtin_amdgcn_readfirstlane((uint32_t)tile);
    uint64_t okw = ~((cu64*)p.excl)[tl];
    if (has_allow) okw &= ((cu64*)p.allow)[tl];
    const uint64_t row0 = (uint64_t)tl * H_BN;
    if (row0 + H_BN > p.N) okw &= p.N > row0 ? ((1ull << (p.N - row0)) - 1) : 0ull;
    return okw;
}

// LDS stage: [2 row blocks][ns k-steps][64 lanes] uint4 image, then 64 floats
// of s|x|^2, then the exclusion and allow words of the tile.
template <int NS>
struct H16Stage {
    static constexpr int IMG_U4 = 2 * NS * 64;
    static constexpr int U4 = IMG_U4 + 16 + 1;
};
#ifndef WV_H16_TPS
#define WV_H16_TPS 3   // (round 4: 3 tiles per stage, 2.66 -> 2.60 ms per 1M x 10k pass; 3 stages of 3 = 150 KiB at D = 128)
#endif
constexpr int H_TPS8 = WV_H16_TPS;   // tiles per LDS stage (8-wave kernel): one barrier per H_TPS8 tiles
constexpr int H_STAGES = 3;   // a stage holds H_TPS tiles; stage p % 3 computes while p + 1, p + 2 land

}  // namespace wv
