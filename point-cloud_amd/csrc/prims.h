// prims.h — device primitives for gfx950: wave64 helpers, exclusive scan of
// u32 arrays (reduce-then-scan, 4096-element tiles, dwordx4 loads) and a
// stable LSD radix sort of (u32 key, u32 value) pairs with ballot-based
// in-wave ranking (64-lane match masks) and LDS-staged coalesced scatter.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcc {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Peers of this lane: the lanes with `act` whose value v (NB low bits) equals
// this lane's.  One v_cmp per bit (its lane mask is the ballot) and the per-lane
// select as a 32-bit xor on both halves; every lane of the wave must be active.
template <int NB>
__device__ __forceinline__ uint64_t wave_peers(uint32_t v, bool act) {
    const uint64_t a = __builtin_amdgcn_ballot_w64(act);
    uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const int32_t sx = ((int32_t)(v << (31 - b))) >> 31;   // ~0 if the bit is set, 0 otherwise (v_bfe_i32)
        const uint64_t bb = __builtin_amdgcn_ballot_w64(sx != 0);
        lo &= ~((uint32_t)bb ^ (uint32_t)sx);   // lanes whose bit equals this lane's (one v_bitop3 per half)
        hi &= ~((uint32_t)(bb >> 32) ^ (uint32_t)sx);
    }
    return ((uint64_t)hi << 32) | lo;
}
// number of set bits of m below this lane
__device__ __forceinline__ uint32_t mask_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Workgroup barrier that orders LDS only: waits lgkmcnt(0) but leaves global
// loads in flight (a plain __syncthreads() drains vmcnt and kills prefetch).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---------------------------------------------------------------- block scan
// Exclusive scan of one u32 per thread across a BS-thread block; returns the
// exclusive prefix and writes the block total to *total (all threads).
template <int BS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds /* BS/64 + 1 */, uint32_t* total) {
    const uint32_t lane = lane_id(), w = threadIdx.x / kWave;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t y = __shfl_up(x, d, kWave);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == kWave - 1) lds[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < BS / kWave; i++) { uint32_t t = lds[i]; lds[i] = acc; acc += t; }
        lds[BS / kWave] = acc;
    }
    __syncthreads();
    uint32_t r = lds[w] + x - v;
    *total = lds[BS / kWave];
    __syncthreads();
    return r;
}

// Same with LDS-only barriers (global loads issued before stay in flight).
template <int BS>
__device__ __forceinline__ uint32_t block_excl_scan_lds(uint32_t v, uint32_t* lds /* BS/64 + 1 */, uint32_t* total) {
    const uint32_t lane = lane_id(), w = threadIdx.x / kWave;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t y = __shfl_up(x, d, kWave);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == kWave - 1) lds[w] = x;
    lds_barrier();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < BS / kWave; i++) { uint32_t t = lds[i]; lds[i] = acc; acc += t; }
        lds[BS / kWave] = acc;
    }
    lds_barrier();
    uint32_t r = lds[w] + x - v;
    *total = lds[BS / kWave];
    lds_barrier();
    return r;
}

template <int BS>
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* lds) {
    uint32_t t;
    block_excl_scan<BS>(v, lds, &t);
    return t;
}

// ---------------------------------------------------------------- scan
struct ScanTemp { uint32_t* bsums = nullptr; uint32_t cap = 0; };
// out[i] = sum(in[0..i)), optional *d_total = sum(in).  in may alias out.
void scan_excl_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* d_total, ScanTemp& tmp, hipStream_t st);

// ---------------------------------------------------------------- radix sort
struct SortTemp { uint32_t* counts = nullptr; uint64_t cap = 0; ScanTemp scan; };
// Stable sort of (keys, vals) by the low `bits` bits of keys.  Ping-pongs
// between (k0,v0) and (k1,v1); returns 0 if the result is in (k0,v0), 1 if in (k1,v1).
int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, int bits, SortTemp& tmp,
                     hipStream_t st);

}  // namespace pcc
