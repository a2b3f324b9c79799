// Diagnostic: does v_cvt_i32_f32 saturate like Rust `f32 as i32` (NaN -> 0)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <cstdint>
#include "../point-cloud_amd/csrc/pcc_math.h"
__global__ void k(const float* in, int32_t* out, int n) {
    int i = threadIdx.x;
    if (i < n) {
        int32_t r;
        asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(in[i]));
        out[i] = r;
    }
}
int main() {
    float v[] = {NAN, -NAN, INFINITY, -INFINITY, 2147483648.0f, 2147483520.0f, 4294967296.0f, -2147483648.0f,
                 -2147483904.0f, 1e30f, -1e30f, 3.7f, -3.7f, -0.0f, 0.5f, -0.5f, 16777217.0f, -1.0f};
    const int n = sizeof(v) / sizeof(v[0]);
    float* d; int32_t* o;
    hipMalloc(&d, sizeof v); hipMalloc(&o, n * 4);
    hipMemcpy(d, v, sizeof v, hipMemcpyHostToDevice);
    k<<<1, 64>>>(d, o, n);
    int32_t h[64];
    hipMemcpy(h, o, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; i++) {
        const int32_t ref = pcc::sat_i32(v[i]);
        printf("%14g hw=%d ref=%d %s\n", (double)v[i], h[i], ref, h[i] == ref ? "" : "MISMATCH");
        bad += h[i] != ref;
    }
    printf("mismatches %d\n", bad);
    return bad ? 1 : 0;
}
