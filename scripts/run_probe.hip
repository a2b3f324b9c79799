// run_probe.hip — DIAGNOSTIC ONLY (not part of the product): read bandwidth of
// the second level-0 binning pass if the first one wrote its tiles in place
// (tile-major, DESIGN.md §4 "pass 0 folded into pass 1"): pass 2 then reads, for
// one low digit b, the run of b of every tile (L points each, consecutive runs a
// tile apart) instead of one contiguous segment.  Prints TB/s of 16-B records +
// 4-B (or 2-B) keys read and written, for several run lengths, against a plain
// contiguous copy of the same bytes.
//   hipcc --offload-arch=gfx950 -O3 -o run_probe run_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int T = 3072;   // points per tile

// v = virtual index in (digit-major, tile-minor) order; runs of L points, T / L digits
template <int KB>
__global__ __launch_bounds__(256) void k_runs(const float4* __restrict__ a, const void* __restrict__ ka, float4* __restrict__ o,
                                              uint32_t* __restrict__ ko, uint64_t n, uint32_t L, uint64_t ntiles) {
    const uint32_t nd = T / L;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < n; v += (uint64_t)gridDim.x * 256) {
        const uint64_t r = v / L, i = v % L;
        const uint64_t b = r / ntiles, t = r % ntiles;
        const uint64_t p = t * T + b * L + i;
        (void)nd;
        o[v] = a[p];
        if (KB == 4) ko[v] = reinterpret_cast<const uint32_t*>(ka)[p];
        else ko[v] = (uint32_t)(t * T) + reinterpret_cast<const uint16_t*>(ka)[p];
    }
}

int main(int argc, char** argv) {
    const uint64_t ntiles = argc > 1 ? strtoull(argv[1], 0, 10) : 300000ull;
    const uint64_t n = ntiles * T;
    float4 *a, *o;
    uint32_t *k, *ko;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&o, n * 16));
    CK(hipMalloc(&k, n * 4));
    CK(hipMalloc(&ko, n * 4));
    CK(hipMemset(a, 1, n * 16));
    CK(hipMemset(k, 0, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    for (int kb : {4, 2}) {
        for (uint32_t L : {3072u, 192u, 96u, 48u, 24u}) {
            for (int rep = 0; rep < 3; rep++) {
                CK(hipEventRecord(e0));
                if (kb == 4) k_runs<4><<<16384, 256>>>(a, k, o, ko, n, L, ntiles);
                else k_runs<2><<<16384, 256>>>(a, k, o, ko, n, L, ntiles);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep == 2)
                    printf("keys %dB run %4u points: %.3f ms  %.2f TB/s (read %d + write 20 B per point)\n", kb, L, ms,
                           n * (16.0 + kb + 20.0) / ms / 1e9, 16 + kb);
            }
        }
    }
    return 0;
}
