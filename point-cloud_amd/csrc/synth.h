// synth.h — deterministic synthetic point clouds, generated
// identically on host and on gfx950 (counter-based hash, exact f32 ops, no
// transcendentals) so GPU-generated inputs need no host copy for parity.
//   kind 0: uniform in [lo, lo+ext)^3
//   kind 1: clustered: 32 blobs, centres in the middle 90 % of the domain,
//           sigma 10..80, Irwin-Hall(4) offsets (a Gaussian-like bump built
//           from 4 uniforms so host and device agree bit for bit)
//   kind 2: config 3 of SURVEY.md §8d: Gaussian mixture (Box-Muller), see below
#pragma once
#include <math.h>
#include <stdint.h>
#include "pcc_math.h"

namespace pcc {

PCC_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
PCC_HD uint64_t synth_hash(uint64_t seed, uint64_t i, uint32_t a) {
    return splitmix64(splitmix64(seed) ^ (i * 4u + a));
}
PCC_HD float synth_unit(uint64_t h) { return (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f); }

// ---- kind 2 (config 3): Gaussian mixture, K = 32 equally
// weighted clusters, centres uniform in the middle 90 % of the domain
// ([-900, 900)^3 for [-1000, 1000)), sigma_k = 10 * 2^U[0,3), Box-Muller
// normals.  Transcendentals are fixed polynomials in plain f32 ops (no FMA
// contraction on either side) and the square root is the correctly rounded one,
// so host and device produce the same bits.
PCC_HD float synth_bits_f(uint32_t b) {
    union { uint32_t u; float f; } c;
    c.u = b;
    return c.f;
}
// ln(u), u normal and > 0: u = m 2^e, ln m = 2 atanh(s), s = (m-1)/(m+1) < 1/3
PCC_HD float synth_log(float u) {
    union { float f; uint32_t u; } c;
    c.f = u;
    const int e = (int)((c.u >> 23) & 255u) - 127;
    const float m = synth_bits_f((c.u & 0x7FFFFFu) | 0x3F800000u);
    const float s = (m - 1.0f) / (m + 1.0f);
    const float s2 = s * s;
    float p = 0.0909090909f;               // 1/11
    p = (p * s2) + 0.111111111f;           // 1/9
    p = (p * s2) + 0.142857143f;           // 1/7
    p = (p * s2) + 0.2f;                   // 1/5
    p = (p * s2) + 0.333333333f;           // 1/3
    p = (p * s2) + 1.0f;
    return ((float)e * 0.693147181f) + ((2.0f * s) * p);
}
// cos and sin of 2 pi u, u in [0, 1): quadrant from 4u, Taylor on [0, pi/2)
PCC_HD void synth_cossin(float u, float& co, float& si) {
    const float a = 4.0f * u;
    const float qf = floorf(a);
    const int q = (int)qf;
    const float x = (a - qf) * 1.57079633f;
    const float x2 = x * x;
    float s = -2.50521084e-8f;             // -1/11!
    s = (s * x2) + 2.75573192e-6f;
    s = (s * x2) - 1.98412698e-4f;
    s = (s * x2) + 8.33333333e-3f;
    s = (s * x2) - 0.166666667f;
    s = ((s * x2) + 1.0f) * x;
    float c = 2.08767570e-9f;              // 1/12!
    c = (c * x2) - 2.75573192e-7f;
    c = (c * x2) + 2.48015873e-5f;
    c = (c * x2) - 1.38888889e-3f;
    c = (c * x2) + 4.16666667e-2f;
    c = (c * x2) - 0.5f;
    c = (c * x2) + 1.0f;
    co = q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
    si = q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
}
// 2^f, f in [0, 1): Taylor of e^(f ln 2)
PCC_HD float synth_exp2_frac(float f) {
    const float x = f * 0.693147181f;
    float p = 1.98412698e-4f;              // 1/7!
    p = (p * x) + 1.38888889e-3f;
    p = (p * x) + 8.33333333e-3f;
    p = (p * x) + 4.16666667e-2f;
    p = (p * x) + 0.166666667f;
    p = (p * x) + 0.5f;
    p = (p * x) + 1.0f;
    return (p * x) + 1.0f;
}
// (0, 1]: (24 hash bits + 1) / 2^24, so the logarithm is finite
PCC_HD float synth_unit_open0(uint64_t h24) { return (float)((uint32_t)(h24 & 0xFFFFFFu) + 1u) * (1.0f / 16777216.0f); }
// correctly rounded f32 square root (the double root is within an ulp of the
// true root, so rounding it to f32 cannot cross an f32 rounding boundary)
PCC_HD float synth_sqrt(float v) { return (float)sqrt((double)v); }

PCC_HD void synth_gauss_mix(uint64_t seed, uint64_t i, uint64_t hc, float lo, float ext, float& x, float& y,
                            float& z) {
    const uint32_t k = (uint32_t)(hc >> 59);   // cluster 0..31, equal weights
    const float e3 = 3.0f * synth_unit(synth_hash(seed ^ 0xC2u, k, 0));
    const float ef = floorf(e3);
    const float sig = 10.0f * (synth_exp2_frac(e3 - ef) * (ef == 0.0f ? 1.0f : (ef == 1.0f ? 2.0f : 4.0f)));
    float n[4];
    for (int pr = 0; pr < 2; pr++) {           // two Box-Muller pairs -> 3 normals used
        const uint64_t h = synth_hash(seed, i, (uint32_t)pr);
        const float r = synth_sqrt(-2.0f * synth_log(synth_unit_open0(h >> 40)));
        float co, si;
        synth_cossin(synth_unit(h << 24), co, si);
        n[2 * pr] = r * co;
        n[2 * pr + 1] = r * si;
    }
    float v[3];
    for (int a = 0; a < 3; a++) {
        const float c = (lo + 0.05f * ext) + (0.9f * ext) * synth_unit(synth_hash(seed ^ 0xC1u, k, (uint32_t)a));
        v[a] = c + sig * n[a];
    }
    x = v[0]; y = v[1]; z = v[2];
}

PCC_HD void synth_point(uint64_t seed, int kind, uint64_t i, float lo, float ext,
                        float& x, float& y, float& z, uint32_t& rgba) {
    uint64_t hc = synth_hash(seed, i, 3);
    if (kind == 0) {
        x = lo + ext * synth_unit(synth_hash(seed, i, 0));
        y = lo + ext * synth_unit(synth_hash(seed, i, 1));
        z = lo + ext * synth_unit(synth_hash(seed, i, 2));
    } else if (kind == 2) {
        synth_gauss_mix(seed, i, hc, lo, ext, x, y, z);
    } else {
        uint32_t k = (uint32_t)(hc >> 59);
        float v[3];
        float sig = 10.0f * (1.0f + 7.0f * synth_unit(synth_hash(seed ^ 0xC2u, k, 0)));
        for (int a = 0; a < 3; a++) {
            float c = (lo + 0.05f * ext) + (0.9f * ext) * synth_unit(synth_hash(seed ^ 0xC1u, k, (uint32_t)a));
            uint64_t h = synth_hash(seed, i, (uint32_t)a);
            uint64_t h2 = splitmix64(h);
            float s = synth_unit(h) + synth_unit(h << 24) + synth_unit(h2) + synth_unit(h2 << 24);
            v[a] = c + sig * (s - 2.0f);
        }
        x = v[0]; y = v[1]; z = v[2];
    }
    rgba = (uint32_t)hc;   // little-endian bytes r,g,b,a = low 4 bytes of hc
}

}  // namespace pcc
