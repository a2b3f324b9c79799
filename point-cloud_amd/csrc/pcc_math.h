// pcc_math.h — exact f32 cell / hex-slot arithmetic shared by host C++ and
// gfx950 device code.  Every function reproduces the reference's operation
// order so that GPU results are bit-identical:
//   hex.rs:3-85, metadata.rs:91-112, cell.rs:276-278, glam Vec3::distance_squared.
// Compile host and device with -ffp-contract=off (no FMA contraction): rustc
// never contracts a*b+c, and hipcc would otherwise emit v_fma_f32.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define PCC_HD __host__ __device__ __forceinline__
#else
#define PCC_HD inline
#endif

namespace pcc {

constexpr float kSqrt3 = 1.73205080757f;  // hex.rs:3

struct I3 { int32_t x, y, z; };

// Rust `f32 as i32`: saturating, NaN -> 0.  On gfx950 this is exactly what
// v_cvt_i32_f32 does in hardware (verified for NaN, +-inf, +-2^31 boundaries
// and rounding toward zero: scripts/cvt_test.hip), so the device path is one
// instruction; the host path is branch-free selects.
PCC_HD int32_t sat_i32(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return r;
#else
    const float c = fminf(fmaxf(v, -2147483648.0f), 2147483520.0f);  // 2147483520 = largest f32 < 2^31
    int32_t r = (int32_t)c;
    r = (v >= 2147483648.0f) ? INT32_MAX : r;
    return (v != v) ? 0 : r;
#endif
}

// metadata.rs:91-93  max_cell_size / 2u32.pow(h) as f32
PCC_HD float cell_size(float max_cell_size, uint32_t h) {
    return max_cell_size / (float)(h >= 32 ? 0u : (1u << h));
}
// metadata.rs:95-97
PCC_HD float sub_cell_size(float cs, uint32_t dim) { return cs / (float)dim; }
// cell.rs:276-278 sub_grid_index_for_point uses sub_cell_size / 2.0
PCC_HD float hex_radius(float sub) { return sub / 2.0f; }
// metadata.rs:100-102 (per axis)
PCC_HD int32_t cell_index1(float p, float cs) { return sat_i32(floorf(p / cs)); }
// metadata.rs:104-106 (per axis)
PCC_HD float cell_pos1(int32_t i, float cs) { return ((float)i * cs) + (cs / 2.0f); }

// hex.rs:67-85 AxialIndex::from_world, then hex.rs:45-51 to_offset
PCC_HD I3 hex_from_world(float px, float py, float pz, float cr) {
    float x = px / (cr * kSqrt3);
    float y = py / ((-cr) * kSqrt3);
    float t = (kSqrt3 * y) + 1.0f;
    float t1 = floorf(t + x);
    float t2 = t - x;
    float t3 = (2.0f * x) + 1.0f;
    float qf = (t1 + t3) / 3.0f;
    float rf = (t1 + t2) / 3.0f;
    int32_t q = sat_i32(floorf(qf));
    int32_t r = (int32_t)(0u - (uint32_t)sat_i32(floorf(rf)));
    int32_t h = sat_i32(pz / cr);
    // i32 `+` wraps in the reference's release build; only saturated indices
    // (infinite coordinates) get near the ends of the range
    I3 o = { (int32_t)((uint32_t)q + (uint32_t)((r - (r & 1)) / 2)), r, h };
    return o;
}

// hex.rs:18-24 to_axial, then hex.rs:55-65 AxialIndex::to_world
PCC_HD void hex_to_world(I3 o, float cr, float& X, float& Y, float& Z) {
    int32_t q = (int32_t)((uint32_t)o.x - (uint32_t)((o.y - (o.y & 1)) / 2));   // wrapping, as hex.rs:18-24 in release
    float qf = (float)q, rf = (float)o.y, hf = (float)o.z;
    X = cr * ((kSqrt3 * qf) + ((kSqrt3 / 2.0f) * rf));
    Y = ((cr * 3.0f) / 2.0f) * rf;
    Z = hf * cr;
}

// glam 0.27 Vec3::distance_squared: (a-b).dot(a-b) = ((dx*dx)+(dy*dy))+(dz*dz)
PCC_HD float dist2(float cx, float cy, float cz, float px, float py, float pz) {
    float dx = cx - px, dy = cy - py, dz = cz - pz;
    return ((dx * dx) + (dy * dy)) + (dz * dz);
}

// Slot-table geometry of one z-layer of a cell (see DESIGN.md "slab"): offset
// indices relative to the slot holding the cell centre fall inside
// [-TX/2, TX/2) x [-TY/2, TY/2).  Width of a cell in hex columns is
// 2*dim/sqrt3, in hex rows 4*dim/3 (cell side = 2*dim hex radii).
struct SlabGeom {
    int32_t tx, ty;      // table extents
    int32_t nl;          // z-layers a cell can touch (local layer index range)
};
PCC_HD SlabGeom slab_geom(uint32_t dim) {
    SlabGeom g;
    g.tx = 2 * ((int32_t)(dim * 577u / 1000u) + 3);   // dim/sqrt3 + margin (dim 96: 116, observed |dx| <= 56)
    g.ty = 2 * ((int32_t)(dim * 2u / 3u) + 2);        // 2*dim/3 + margin  (dim 96: 132, observed |dy| <= 64)
    g.nl = 2 * (int32_t)dim + 5;                      // layers [2*dim*iz - 2, 2*dim*(iz+1) + 2]
    return g;
}

}  // namespace pcc
