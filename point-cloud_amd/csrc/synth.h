// synth.h — deterministic synthetic point clouds, generated
// identically on host and on gfx950 (counter-based hash, exact f32 ops, no
// transcendentals) so GPU-generated inputs need no host copy for parity.
//   kind 0: uniform in [lo, lo+ext)^3
//   kind 1: clustered: 32 blobs, centres in the middle 90 % of the domain,
//           sigma 10..80, Irwin-Hall(4) offsets (a Gaussian-like bump built
//           from 4 uniforms so host and device agree bit for bit)
#pragma once
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

PCC_HD void synth_point(uint64_t seed, int kind, uint64_t i, float lo, float ext,
                        float& x, float& y, float& z, uint32_t& rgba) {
    uint64_t hc = synth_hash(seed, i, 3);
    if (kind == 0) {
        x = lo + ext * synth_unit(synth_hash(seed, i, 0));
        y = lo + ext * synth_unit(synth_hash(seed, i, 1));
        z = lo + ext * synth_unit(synth_hash(seed, i, 2));
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
