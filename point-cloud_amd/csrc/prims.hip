// prims.hip — exclusive scan + stable LSD radix sort for gfx950 (see prims.h).
#include "prims.h"
#include "hip_check.h"

namespace pcc {

constexpr int kScanBS = 256, kScanIPT = 16, kScanTile = kScanBS * kScanIPT;

__global__ __launch_bounds__(kScanBS) void k_scan_reduce(const uint32_t* __restrict__ in, uint32_t n,
                                                         uint32_t* __restrict__ bsums) {
    __shared__ uint32_t lds[kScanBS / kWave + 1];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanIPT;
    uint32_t s = 0;
    if (base + kScanIPT <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int i = 0; i < kScanIPT / 4; i++) { uint4 v = p[i]; s += v.x + v.y + v.z + v.w; }
    } else {
        for (uint64_t i = base; i < n; i++) s += in[i];
    }
    uint32_t t = block_sum<kScanBS>(s, lds);
    if (threadIdx.x == 0) bsums[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void k_scan_sums(uint32_t* __restrict__ bsums, uint32_t nb, uint32_t* d_total) {
    __shared__ uint32_t lds[1024 / kWave + 1];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        uint32_t i = b0 + threadIdx.x;
        uint32_t v = i < nb ? bsums[i] : 0, tot;
        uint32_t e = block_excl_scan<1024>(v, lds, &tot);
        if (i < nb) bsums[i] = carry + e;
        __syncthreads();
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && d_total) *d_total = carry;
}

__global__ __launch_bounds__(kScanBS) void k_scan_down(const uint32_t* in, uint32_t* out, uint32_t n,
                                                       const uint32_t* __restrict__ bsums) {
    __shared__ uint32_t lds[kScanBS / kWave + 1];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanIPT;
    uint32_t v[kScanIPT];
    const bool full = base + kScanIPT <= n;
    if (full) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int i = 0; i < kScanIPT / 4; i++) { uint4 q = p[i]; v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w; }
    } else {
#pragma unroll
        for (int i = 0; i < kScanIPT; i++) v[i] = (base + i < n) ? in[base + i] : 0;
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanIPT; i++) s += v[i];
    uint32_t tot;
    uint32_t e = block_excl_scan<kScanBS>(s, lds, &tot) + bsums[blockIdx.x];
    if (full) {
        uint4* p = reinterpret_cast<uint4*>(out + base);
#pragma unroll
        for (int i = 0; i < kScanIPT / 4; i++) {
            uint4 q;
            q.x = e; e += v[4 * i];
            q.y = e; e += v[4 * i + 1];
            q.z = e; e += v[4 * i + 2];
            q.w = e; e += v[4 * i + 3];
            p[i] = q;
        }
    } else {
        for (int i = 0; i < kScanIPT; i++)
            if (base + i < n) { out[base + i] = e; e += v[i]; }
    }
}

// Small arrays (the per-level tables of deep levels, config 3's levels): one
// block walks tiles of 16 384 words with a running carry, one launch instead of
// three (each launch of a few microseconds costs as much again in dispatch gaps).
constexpr uint32_t kScanSingleMax = 32768;
__global__ __launch_bounds__(1024) void k_scan_single(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* d_total) {
    constexpr uint32_t T = 1024 * kScanIPT;
    __shared__ uint32_t lds[1024 / kWave + 1];
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < n; t0 += T) {
        const uint32_t base = t0 + threadIdx.x * kScanIPT;
        uint32_t v[kScanIPT], s = 0;
#pragma unroll
        for (int i = 0; i < kScanIPT; i++) {
            v[i] = base + i < n ? in[base + i] : 0u;
            s += v[i];
        }
        uint32_t tot;
        uint32_t e = block_excl_scan<1024>(s, lds, &tot) + carry;   // (ends with a barrier: in-place safe)
#pragma unroll
        for (int i = 0; i < kScanIPT; i++)
            if (base + i < n) { out[base + i] = e; e += v[i]; }
        carry += tot;
    }
    if (threadIdx.x == 0 && d_total) *d_total = carry;
}

void scan_excl_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* d_total, ScanTemp& tmp, hipStream_t st) {
    if (n == 0) {
        if (d_total) HIP_CHECK(hipMemsetAsync(d_total, 0, 4, st));
        return;
    }
    if (n <= kScanSingleMax) {
        k_scan_single<<<1, 1024, 0, st>>>(in, out, n, d_total);
        HIP_CHECK(hipGetLastError());
        return;
    }
    uint32_t nb = (n + kScanTile - 1) / kScanTile;
    if (tmp.cap < nb) {
        if (tmp.bsums) HIP_CHECK(hipFree(tmp.bsums));
        tmp.cap = nb + 1024;
        HIP_CHECK(hipMalloc(&tmp.bsums, tmp.cap * sizeof(uint32_t)));
    }
    // dwordx4 loads need 16-B alignment of `in`/`out`: all callers pass hipMalloc bases.
    k_scan_reduce<<<nb, kScanBS, 0, st>>>(in, n, tmp.bsums);
    k_scan_sums<<<1, 1024, 0, st>>>(tmp.bsums, nb, d_total);
    k_scan_down<<<nb, kScanBS, 0, st>>>(in, out, n, tmp.bsums);
    HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------- radix sort
constexpr int kRsBS = 256, kRsIPT = 16, kRsTile = kRsBS * kRsIPT, kRsWaves = kRsBS / kWave;

template <int BITS>
__global__ __launch_bounds__(kRsBS) void k_rs_upsweep(const uint32_t* __restrict__ keys, uint32_t n, int shift,
                                                      uint32_t* __restrict__ counts, uint32_t nblocks) {
    constexpr int R = 1 << BITS;
    __shared__ uint32_t hist[R];
    for (int i = threadIdx.x; i < R; i += kRsBS) hist[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kRsTile;
#pragma unroll
    for (int r = 0; r < kRsIPT; r++) {
        uint64_t i = base + (uint64_t)r * kRsBS + threadIdx.x;
        if (i < n) atomicAdd(&hist[(keys[i] >> shift) & (R - 1)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < R; d += kRsBS) counts[(uint64_t)d * nblocks + blockIdx.x] = hist[d];
}

template <int BITS>
__global__ __launch_bounds__(kRsBS) void k_rs_downsweep(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                        uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                        uint32_t n, int shift, const uint32_t* __restrict__ offs,
                                                        uint32_t nblocks) {
    constexpr int R = 1 << BITS;
    __shared__ uint32_t skey[kRsTile], sval[kRsTile];
    __shared__ uint32_t wcnt[kRsWaves][R], wpre[kRsWaves][R];
    __shared__ uint32_t run[R], dbase[R], goff[R];
    __shared__ uint32_t lds[kRsWaves + 1];
    const uint32_t w = threadIdx.x / kWave;
    for (int i = threadIdx.x; i < R; i += kRsBS) {
        run[i] = 0;
        goff[i] = offs[(uint64_t)i * nblocks + blockIdx.x];
        for (int q = 0; q < kRsWaves; q++) wcnt[q][i] = 0;
    }
    const uint64_t base = (uint64_t)blockIdx.x * kRsTile;
    uint32_t k[kRsIPT], v[kRsIPT], rank[kRsIPT];
#pragma unroll
    for (int r = 0; r < kRsIPT; r++) {
        uint64_t i = base + (uint64_t)r * kRsBS + threadIdx.x;
        if (i < n) { k[r] = kin[i]; v[r] = vin[i]; }
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int r = 0; r < kRsIPT; r++) {
        uint64_t i = base + (uint64_t)r * kRsBS + threadIdx.x;
        const bool valid = i < n;
        const uint32_t d = (k[r] >> shift) & (R - 1);
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; b++) {
            uint64_t bb = __ballot(valid && ((d >> b) & 1));
            same &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rw = __popcll(same & lt);
        if (valid && rw == 0) wcnt[w][d] = (uint32_t)__popcll(same);
        __syncthreads();
        for (int t = threadIdx.x; t < R; t += kRsBS) {
            uint32_t acc = run[t];
#pragma unroll
            for (int q = 0; q < kRsWaves; q++) { uint32_t c = wcnt[q][t]; wpre[q][t] = acc; acc += c; wcnt[q][t] = 0; }
            run[t] = acc;
        }
        __syncthreads();
        rank[r] = valid ? wpre[w][d] + rw : 0;
    }
    // tile-local digit bases
    {
        uint32_t tot;
        if (R <= kRsBS) {
            uint32_t c = threadIdx.x < (uint32_t)R ? run[threadIdx.x] : 0;
            uint32_t e = block_excl_scan<kRsBS>(c, lds, &tot);
            if (threadIdx.x < (uint32_t)R) dbase[threadIdx.x] = e;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRsIPT; r++) {
        uint64_t i = base + (uint64_t)r * kRsBS + threadIdx.x;
        if (i < n) {
            const uint32_t d = (k[r] >> shift) & (R - 1);
            const uint32_t p = dbase[d] + rank[r];
            skey[p] = k[r];
            sval[p] = v[r];
        }
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)((n - base) < (uint64_t)kRsTile ? (n - base) : (uint64_t)kRsTile);
    for (uint32_t j = threadIdx.x; j < tn; j += kRsBS) {
        const uint32_t key = skey[j];
        const uint32_t d = (key >> shift) & (R - 1);
        const uint32_t dst = goff[d] + (j - dbase[d]);
        kout[dst] = key;
        vout[dst] = sval[j];
    }
}

template <int BITS>
static void rs_pass(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout, uint32_t n, int shift,
                    SortTemp& tmp, hipStream_t st) {
    const uint32_t nb = (n + kRsTile - 1) / kRsTile;
    const uint64_t need = (uint64_t)nb << BITS;
    if (tmp.cap < need) {
        if (tmp.counts) HIP_CHECK(hipFree(tmp.counts));
        tmp.cap = need + 4096;
        HIP_CHECK(hipMalloc(&tmp.counts, tmp.cap * sizeof(uint32_t)));
    }
    k_rs_upsweep<BITS><<<nb, kRsBS, 0, st>>>(kin, n, shift, tmp.counts, nb);
    scan_excl_u32(tmp.counts, tmp.counts, (uint32_t)need, nullptr, tmp.scan, st);
    k_rs_downsweep<BITS><<<nb, kRsBS, 0, st>>>(kin, vin, kout, vout, n, shift, tmp.counts, nb);
    HIP_CHECK(hipGetLastError());
}

int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, uint32_t n, int bits, SortTemp& tmp,
                     hipStream_t st) {
    if (n <= 1 || bits <= 0) return 0;
    const int passes = (bits + 7) / 8;
    const int per = (bits + passes - 1) / passes;
    int cur = 0, shift = 0;
    for (int p = 0; p < passes; p++) {
        const uint32_t* ki = cur ? k1 : k0;
        const uint32_t* vi = cur ? v1 : v0;
        uint32_t* ko = cur ? k0 : k1;
        uint32_t* vo = cur ? v0 : v1;
        switch (per) {
            case 1: rs_pass<1>(ki, vi, ko, vo, n, shift, tmp, st); break;
            case 2: rs_pass<2>(ki, vi, ko, vo, n, shift, tmp, st); break;
            case 3: rs_pass<3>(ki, vi, ko, vo, n, shift, tmp, st); break;
            case 4: rs_pass<4>(ki, vi, ko, vo, n, shift, tmp, st); break;
            case 5: rs_pass<5>(ki, vi, ko, vo, n, shift, tmp, st); break;
            case 6: rs_pass<6>(ki, vi, ko, vo, n, shift, tmp, st); break;
            case 7: rs_pass<7>(ki, vi, ko, vo, n, shift, tmp, st); break;
            default: rs_pass<8>(ki, vi, ko, vo, n, shift, tmp, st); break;
        }
        shift += per;
        cur ^= 1;
    }
    return cur;
}

}  // namespace pcc
