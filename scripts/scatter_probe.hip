// scatter_probe.hip — DIAGNOSTIC ONLY (not part of the product): does a
// block-segmented scatter of 16-B records into ~1.5k contiguous per-(slab,
// block) streams reach streaming bandwidth on MI355X (partial lines merged in
// L2 / Infinity Cache), compared with a plain 16-B copy?  Decides the level-0
// binning design.
//   hipcc --offload-arch=gfx950 -O3 -o scatter_probe scatter_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hsh(uint64_t x) {
    x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void k_fill(float4* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = make_float4((float)i, 1.f, 2.f, __uint_as_float(hsh(i)));
}

// bins from the payload (as the real kernel recomputes the slab from the position)
__device__ __forceinline__ uint32_t bin_of(const float4& v, uint32_t nb) { return __float_as_uint(v.w) % nb; }

__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, uint32_t* __restrict__ k, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        b[i] = a[i];
        k[i] = (uint32_t)i;
    }
}

// per-block histogram (block b owns a contiguous range)
__global__ __launch_bounds__(1024) void k_count(const float4* __restrict__ a, uint64_t n, uint32_t nb, uint32_t B,
                                                uint32_t* cnt) {
    __shared__ uint32_t h[4096];
    for (uint32_t i = threadIdx.x; i < nb; i += 1024) h[i] = 0;
    __syncthreads();
    const uint64_t lo = n * blockIdx.x / B, hi = n * (blockIdx.x + 1) / B;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 1024) atomicAdd(&h[bin_of(a[i], nb)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += 1024) cnt[(uint64_t)i * B + blockIdx.x] = h[i];
}

// block-segmented scatter: tile of 1024, rank by LDS atomics (order inside a tile
// is not stable here; only bandwidth is probed), running per-bin counters in LDS
__global__ __launch_bounds__(1024) void k_scatter(const float4* __restrict__ a, uint64_t n, uint32_t nb, uint32_t B,
                                                  const uint32_t* __restrict__ off, float4* __restrict__ o,
                                                  uint32_t* __restrict__ ok) {
    __shared__ uint32_t run[4096];
    __shared__ uint32_t base[4096];
    for (uint32_t i = threadIdx.x; i < nb; i += 1024) { run[i] = 0; base[i] = off[(uint64_t)i * B + blockIdx.x]; }
    __syncthreads();
    const uint64_t lo = n * blockIdx.x / B, hi = n * (blockIdx.x + 1) / B;
    for (uint64_t t = lo; t < hi; t += 1024) {
        const uint64_t i = t + threadIdx.x;
        if (i < hi) {
            const float4 v = a[i];
            const uint32_t d = bin_of(v, nb);
            const uint32_t r = atomicAdd(&run[d], 1u);
            const uint64_t dst = (uint64_t)base[d] + r;
            o[dst] = v;
            ok[dst] = (uint32_t)i;
        }
    }
}

// same, but each thread handles 4 consecutive tiles' points before the next
// step (more bytes in flight per CU)
int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000000ull;
    float4 *a, *o;
    uint32_t *k, *cnt;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&o, n * 16));
    CK(hipMalloc(&k, n * 4));
    k_fill<<<8192, 256>>>(a, n);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(e0));
        k_copy<<<8192, 256>>>(a, o, k, n);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy 16B+4B: %.3f ms  %.2f TB/s\n", ms, n * 36.0 / ms / 1e9);
    }
    for (uint32_t nb : {64u, 256u, 1552u, 4096u}) {
        for (uint32_t B : {256u, 512u, 1024u, 2048u}) {
            CK(hipMalloc(&cnt, (uint64_t)nb * B * 4));
            k_count<<<B, 1024>>>(a, n, nb, B, cnt);
            CK(hipDeviceSynchronize());
            std::vector<uint32_t> h((uint64_t)nb * B);
            CK(hipMemcpy(h.data(), cnt, h.size() * 4, hipMemcpyDeviceToHost));
            uint64_t acc = 0;
            for (auto& v : h) { uint32_t c = v; v = (uint32_t)acc; acc += c; }
            CK(hipMemcpy(cnt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
            for (int rep = 0; rep < 2; rep++) {
                CK(hipEventRecord(e0));
                k_scatter<<<B, 1024>>>(a, n, nb, B, cnt, o, k);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) printf("scatter bins %u blocks %u: %.3f ms  %.2f TB/s\n", nb, B, ms, n * 36.0 / ms / 1e9);
            }
            CK(hipEventRecord(e0));
            k_count<<<B, 1024>>>(a, n, nb, B, cnt);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("   count pass: %.3f ms\n", ms);
            CK(hipFree(cnt));
        }
    }
    return 0;
}
