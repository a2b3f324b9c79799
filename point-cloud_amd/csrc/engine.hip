// engine.hip — MI355X-native hierarchy/LOD build (gfx950).
//
// Replaces the per-batch, per-point loop of point-converter/src/converter.rs:96-139
// and cell.rs:70-153 with the level-synchronous restatement of SURVEY.md
// Appendix C (validated in oracle/pyref.py::convert_keyed):
//
//   level 0 binning  : input points -> slabs (cell, hex z-layer), stable in key
//                      order (LSD radix sort on the slab id + gather)
//   per level h      : one workgroup per slab, slot table in LDS
//      sweep 1       : winners = argmin(dist2, key) per slot (ds_min_u64)
//      sweep 2       : key-ordered replay -> one emission per non-first arrival,
//                      written straight into the child slab it belongs to
//   bucket resolve   : per (cell, octant) bucket: keep (Some) or spill (None),
//                      spill batch via counting over key-ordered child slabs
//   next level       : spilled buckets become the next level's cells; their
//                      child slabs are already laid out contiguously.
//
// Key facts this relies on:
//   * child hex z-layer u comes from parent layer t = u/2 (truncating) because
//     r_{h+1} = r_h / 2 exactly, so each child slab has exactly ONE parent slab
//     and inherits its key order;
//   * keys (input indices) are unique at every level; event batches are
//     monotone in key inside every cell.
#include "engine.h"

#include <algorithm>
#include <chrono>
#include <cstring>

#include "hip_check.h"
#include "pcc_math.h"
#include "prims.h"
#include "synth.h"

namespace pcc {

// ------------------------------------------------------------------ constants
constexpr uint64_t kEmpty64 = ~0ull;
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
constexpr int kDenseBS = 1024;
constexpr int kDenseTab = 16560;     // 120 x 138 slots: one z-layer of a dim-96 cell
constexpr int kDenseClaim = 2048;
constexpr int kSmallBS = 256;
constexpr uint32_t kSmallMax = 1024; // slabs with fewer arrivals use the hashed kernel
constexpr int kSmallTab = 2048;
constexpr int kSmallClaim = 512;
constexpr int kKeptMax = 8192;       // LDS sort capacity for kept (Some) buckets
constexpr int kDests = 24;           // 8 octants x 3 child layers per slab
constexpr uint32_t kMaxDepth = 31;   // 2u32.pow(h) overflows at h = 32 (metadata.rs:92)

enum ErrBits : uint32_t {
    ERR_SLOT_RANGE = 1u << 0,
    ERR_LAYER = 1u << 1,
    ERR_OCTANT = 1u << 2,
    ERR_SEL = 1u << 3,
    ERR_KEPT_CAP = 1u << 4,
    ERR_L0_RANGE = 1u << 5,
    ERR_NONFINITE = 1u << 6,
};

struct Counters {
    uint32_t arena_cur;   // next-level arena allocation cursor
    uint32_t out_cur;     // grid + kept output arena cursor
    uint32_t err;
    uint32_t nbig, nsmall;
    uint32_t ncells_next, nslabs_next;
    uint32_t pad;
    unsigned long long arrivals_next;  // sum of next-level slab sizes
    unsigned long long grid_total;     // grid winners written so far
    unsigned long long dense_arrivals, small_arrivals;
};

struct Arena {
    float *x, *y, *z;
    uint32_t *c, *k, *e;
};

struct Engine::Dev {
    Arena ar[2] = {};
    Point* out = nullptr;           // grid winners + kept bucket lists (== N points total)
    Counters* ctr = nullptr;
    float* bbox_part = nullptr;     // per-block min/max partials
    uint32_t* bbox_flag = nullptr;
    uint32_t* files = nullptr;      // per file: start_lo, start_hi, eb0, batch
    ScanTemp scan;
    SortTemp sort;
    uint64_t cap = 0;
    // chunked bump allocator for per-build tables (reset at every build, chunks kept)
    std::vector<std::pair<uint8_t*, uint64_t>> chunks;
    size_t chunk_i = 0;
    uint64_t chunk_used = 0;
    void* get(uint64_t bytes) {
        bytes = (std::max<uint64_t>(bytes, 1) + 255) & ~255ull;
        while (chunk_i < chunks.size() && chunk_used + bytes > chunks[chunk_i].second) { chunk_i++; chunk_used = 0; }
        if (chunk_i == chunks.size()) {
            uint64_t sz = std::max<uint64_t>(bytes, 256ull << 20);
            uint8_t* p = nullptr;
            HIP_CHECK(hipMalloc(&p, sz));
            chunks.push_back({p, sz});
            chunk_used = 0;
        }
        void* r = chunks[chunk_i].first + chunk_used;
        chunk_used += bytes;
        return r;
    }
    void reset_pool() { chunk_i = 0; chunk_used = 0; }
};

struct Engine::Level {
    uint32_t h = 0, ncells = 0, nslabs = 0, nbig = 0, nsmall = 0;
    int arena = 0;
    int32_t* cell_idx = nullptr;     // 3 * ncells
    uint32_t* cell_sb = nullptr;     // spill batch of the parent bucket (eb' = max(eb, sb))
    uint32_t* cell_slab0 = nullptr;  // ncells + 1
    uint32_t* slab_cell = nullptr;
    int32_t* slab_layer = nullptr;
    uint32_t* slab_off = nullptr;
    uint32_t* slab_n = nullptr;
    uint32_t* big_list = nullptr;
    uint32_t* small_list = nullptr;
    uint32_t* slab_grid_off = nullptr;
    uint32_t* slab_grid_n = nullptr;
    uint32_t* dest_off = nullptr;    // 24 * nslabs
    uint32_t* dest_n = nullptr;
    uint32_t* bkt_state = nullptr;   // 8 * ncells
    uint32_t* bkt_off = nullptr;
    uint32_t* bkt_n = nullptr;
    uint32_t* bkt_sb = nullptr;
    uint32_t* bkt_nd = nullptr;
    Dev* dev = nullptr;
    template <class T>
    void alloc(T*& p, uint64_t n) { p = static_cast<T*>(dev->get(n * sizeof(T))); }
};

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ void set_err(Counters* c, uint32_t bit) { atomicOr(&c->err, bit); }

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }

// event batch of input index i (lib.rs:31-52: batches restart at every file)
__device__ __forceinline__ uint32_t event_batch(const uint32_t* files, uint32_t nfiles, uint64_t i) {
    uint32_t lo = 0, hi = nfiles - 1;
    while (lo < hi) {   // last file with start <= i
        uint32_t mid = (lo + hi + 1) >> 1;
        uint64_t s = (uint64_t)files[4 * mid] | ((uint64_t)files[4 * mid + 1] << 32);
        if (s <= i) lo = mid; else hi = mid - 1;
    }
    uint64_t s = (uint64_t)files[4 * lo] | ((uint64_t)files[4 * lo + 1] << 32);
    return files[4 * lo + 2] + (uint32_t)((i - s) / files[4 * lo + 3]);
}

// ------------------------------------------------------------------ input kernels
__global__ void k_synth(Point* out, uint64_t first, uint64_t n, uint64_t seed, int kind, float lo, float ext) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        float x, y, z;
        uint32_t c;
        synth_point(seed, kind, j, lo, ext, x, y, z, c);
        Point p;
        p.x = x; p.y = y; p.z = z;
        memcpy(p.rgba, &c, 4);
        out[first + j] = p;
    }
}

// bounding-volume/src/lib.rs:23-52 + converter.rs:96-104: the final AABB is the
// componentwise min/max over all points (f32::min/max are exact).
constexpr int kBBoxBS = 256, kBBoxBlocks = 2048;
__global__ __launch_bounds__(kBBoxBS) void k_bbox(const Point* __restrict__ in, uint64_t n, float* part,
                                                  uint32_t* flag) {
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool bad = false;
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (uint64_t i = blockIdx.x * (uint64_t)kBBoxBS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBBoxBS) {
        float4 v = p4[i];
        bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z));
        mn[0] = fminf(mn[0], v.x); mn[1] = fminf(mn[1], v.y); mn[2] = fminf(mn[2], v.z);
        mx[0] = fmaxf(mx[0], v.x); mx[1] = fmaxf(mx[1], v.y); mx[2] = fmaxf(mx[2], v.z);
    }
    for (int d = 32; d > 0; d >>= 1)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
        }
    __shared__ float s[kBBoxBS / 64][6];
    const int w = threadIdx.x / 64;
    if (bad) atomicOr(flag, 1u);
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; a++) { s[w][a] = mn[a]; s[w][3 + a] = mx[a]; }
    __syncthreads();
    if (threadIdx.x < 6) {
        float r = s[0][threadIdx.x];
        for (int q = 1; q < kBBoxBS / 64; q++) r = threadIdx.x < 3 ? fminf(r, s[q][threadIdx.x]) : fmaxf(r, s[q][threadIdx.x]);
        part[blockIdx.x * 6 + threadIdx.x] = r;
    }
}

__global__ void k_bbox_final(float* part, uint32_t nb) {
    if (threadIdx.x < 6) {
        float r = part[threadIdx.x];
        for (uint32_t b = 1; b < nb; b++) r = threadIdx.x < 3 ? fminf(r, part[b * 6 + threadIdx.x]) : fmaxf(r, part[b * 6 + threadIdx.x]);
        part[threadIdx.x] = r;
    }
}

// ------------------------------------------------------------------ level-0 binning
struct L0Params {
    float cs, cr;
    int32_t lo[3];
    int32_t g[3];
    int32_t nl;
    int32_t dim2;   // 2 * sub_grid_dimension
};

// dense slab id of a point: ((cell - lo) linearised) * nl + (layer - (dim2*iz - 2))
__device__ __forceinline__ int64_t l0_dense(const L0Params& P, float x, float y, float z) {
    int32_t ix = cell_index1(x, P.cs), iy = cell_index1(y, P.cs), iz = cell_index1(z, P.cs);
    int32_t gx = ix - P.lo[0], gy = iy - P.lo[1], gz = iz - P.lo[2];
    int32_t t = sat_i32(z / P.cr);   // hex.rs:83 z slot (truncation)
    int64_t ll = (int64_t)t - ((int64_t)P.dim2 * iz - 2);
    if (gx < 0 || gy < 0 || gz < 0 || gx >= P.g[0] || gy >= P.g[1] || gz >= P.g[2] || ll < 0 || ll >= P.nl) return -1;
    return (((int64_t)gz * P.g[1] + gy) * P.g[0] + gx) * P.nl + ll;
}

constexpr int kHistLds = 12288;
__global__ __launch_bounds__(256) void k_l0_hist(const Point* __restrict__ in, uint64_t n, L0Params P, uint32_t* hist,
                                                 uint32_t D, Counters* ctr) {
    __shared__ uint32_t h[kHistLds];
    const bool lds = D <= (uint32_t)kHistLds;
    if (lds) {
        for (uint32_t i = threadIdx.x; i < D; i += 256) h[i] = 0;
        __syncthreads();
    }
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        float4 v = p4[i];
        int64_t d = l0_dense(P, v.x, v.y, v.z);
        if (d < 0) { set_err(ctr, ERR_L0_RANGE); continue; }
        if (lds) atomicAdd(&h[d], 1u); else atomicAdd(&hist[d], 1u);
    }
    if (lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < D; i += 256)
            if (h[i]) atomicAdd(&hist[i], h[i]);
    }
}

// per dense slab: non-empty flag; per grid cell: non-empty flag
__global__ void k_l0_flags(const uint32_t* hist, uint32_t D, int32_t nl, uint32_t* sflag, uint32_t* cflag, uint32_t G) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < D) sflag[d] = hist[d] ? 1u : 0u;
    if (d < G) {
        uint32_t any = 0;
        for (int32_t l = 0; l < nl; l++) any |= hist[(uint64_t)d * nl + l];
        cflag[d] = any ? 1u : 0u;
    }
}

__global__ void k_l0_tables(const uint32_t* hist, const uint32_t* cnt_scan, const uint32_t* sflag_scan,
                            const uint32_t* cflag, const uint32_t* cflag_scan, uint32_t D, uint32_t G, L0Params P,
                            int32_t* cell_idx, uint32_t* cell_sb, uint32_t* cell_slab0, uint32_t* slab_cell,
                            int32_t* slab_layer, uint32_t* slab_off, uint32_t* slab_n, uint32_t* big_list,
                            uint32_t* small_list, Counters* ctr) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < G && cflag[d]) {
        const uint32_t r = cflag_scan[d];
        const int32_t gx = (int32_t)(d % (uint32_t)P.g[0]);
        const int32_t gy = (int32_t)((d / (uint32_t)P.g[0]) % (uint32_t)P.g[1]);
        const int32_t gz = (int32_t)(d / ((uint32_t)P.g[0] * (uint32_t)P.g[1]));
        cell_idx[3 * r] = P.lo[0] + gx;
        cell_idx[3 * r + 1] = P.lo[1] + gy;
        cell_idx[3 * r + 2] = P.lo[2] + gz;
        cell_sb[r] = 0;
        cell_slab0[r] = sflag_scan[(uint64_t)d * P.nl];
    }
    if (d < D && hist[d]) {
        const uint32_t sid = sflag_scan[d];
        const uint32_t g = d / (uint32_t)P.nl;
        const int32_t ll = (int32_t)(d % (uint32_t)P.nl);
        const int32_t gz = (int32_t)(g / ((uint32_t)P.g[0] * (uint32_t)P.g[1]));
        const int32_t iz = P.lo[2] + gz;
        slab_cell[sid] = cflag_scan[g];
        slab_layer[sid] = ll + (P.dim2 * iz - 2);
        slab_off[sid] = cnt_scan[d];
        slab_n[sid] = hist[d];
        if (hist[d] >= kSmallMax) big_list[atomicAdd(&ctr->nbig, 1u)] = sid;
        else small_list[atomicAdd(&ctr->nsmall, 1u)] = sid;
    }
}

__global__ void k_l0_keys(const Point* __restrict__ in, uint64_t n, L0Params P, const uint32_t* sflag_scan,
                          uint32_t* keys, uint32_t* vals) {
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        float4 v = p4[i];
        int64_t d = l0_dense(P, v.x, v.y, v.z);
        keys[i] = d < 0 ? 0 : sflag_scan[d];
        vals[i] = (uint32_t)i;
    }
}

__global__ void k_l0_gather(const Point* __restrict__ in, const uint32_t* __restrict__ perm, uint64_t n, Arena A,
                            const uint32_t* files, uint32_t nfiles) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t src = perm[i];
        float4 v = reinterpret_cast<const float4*>(in)[src];
        A.x[i] = v.x; A.y[i] = v.y; A.z[i] = v.z;
        A.c[i] = __float_as_uint(v.w);
        A.k[i] = src;
        A.e[i] = event_batch(files, nfiles, src);
    }
}

// ------------------------------------------------------------------ slab kernels
struct SlabParams {
    Arena in, nx;
    Point* out;
    const int32_t* cell_idx;
    const uint32_t* cell_sb;
    const uint32_t* slab_cell;
    const int32_t* slab_layer;
    const uint32_t* slab_off;
    const uint32_t* slab_n;
    const uint32_t* list;
    uint32_t* slab_grid_off;
    uint32_t* slab_grid_n;
    uint32_t* dest_off;
    uint32_t* dest_n;
    Counters* ctr;
    float cs, cr, cs_child, cr_child;
    int32_t tx, ty;
};

// Routing of a point from slab (cell c, layer t) to its child slab:
// octant from cell_index at h+1 (metadata.rs:100-102; child = 2*parent + bit),
// child layer u = trunc(z / r_{h+1}) in {2t-1, 2t, 2t+1} -> sel = u - 2t + 1.
__device__ __forceinline__ int dest_of(const SlabParams& P, int32_t cx, int32_t cy, int32_t cz, int32_t t, float x,
                                       float y, float z, uint32_t& err) {
    int32_t bx = cell_index1(x, P.cs_child) - 2 * cx;
    int32_t by = cell_index1(y, P.cs_child) - 2 * cy;
    int32_t bz = cell_index1(z, P.cs_child) - 2 * cz;
    int32_t u = sat_i32(z / P.cr_child);
    int32_t sel = u - 2 * t + 1;
    if ((bx | by | bz) & ~1) { err |= ERR_OCTANT; return -1; }
    if (sel < 0 || sel > 2) { err |= ERR_SEL; return -1; }
    return (bx | (by << 1) | (bz << 2)) * 3 + sel;
}

__device__ __forceinline__ uint32_t hash_slot(uint32_t k) { return (k * 2654435761u) >> 16; }

template <bool DENSE>
struct SlabLds;

template <>
struct SlabLds<true> {
    static constexpr int BS = kDenseBS, TAB = kDenseTab, CLAIM = kDenseClaim, NW = BS / 64;
    unsigned long long tab[TAB];
    uint32_t claim[CLAIM];
    uint32_t tkey[1];
    uint32_t dcnt[kDests], doff[kDests], dcur[kDests];
    uint32_t wcnt[NW][kDests], wpre[NW][kDests];
    uint32_t nwin, wbase, wctr, err;
};
template <>
struct SlabLds<false> {
    static constexpr int BS = kSmallBS, TAB = kSmallTab, CLAIM = kSmallClaim, NW = BS / 64;
    unsigned long long tab[TAB];
    uint32_t claim[CLAIM];
    uint32_t tkey[TAB];
    uint32_t dcnt[kDests], doff[kDests], dcur[kDests];
    uint32_t wcnt[NW][kDests], wpre[NW][kDests];
    uint32_t nwin, wbase, wctr, err;
};

// slot -> table entry (DENSE: direct; otherwise LDS open addressing on the local slot id)
template <bool DENSE>
__device__ __forceinline__ int slot_entry(SlabLds<DENSE>& S, uint32_t local, bool insert) {
    if constexpr (DENSE) {
        return (int)local;
    } else {
        uint32_t h = hash_slot(local) & (SlabLds<false>::TAB - 1);
        for (int probe = 0; probe < SlabLds<false>::TAB; probe++) {
            uint32_t k = S.tkey[h];
            if (k == local) return (int)h;
            if (k == kEmpty32) {
                if (!insert) return -1;
                uint32_t old = atomicCAS(&S.tkey[h], kEmpty32, local);
                if (old == kEmpty32 || old == local) return (int)h;
            }
            h = (h + 1) & (SlabLds<false>::TAB - 1);
        }
        return -1;
    }
}

template <bool DENSE>
__global__ __launch_bounds__(SlabLds<DENSE>::BS) void k_slab(SlabParams P) {
    using L = SlabLds<DENSE>;
    constexpr int BS = L::BS, TAB = L::TAB, CLAIM = L::CLAIM, NW = L::NW;
    __shared__ L S;
    const uint32_t tid = threadIdx.x, wv = tid / 64;
    const uint32_t s = P.list[blockIdx.x];
    const uint32_t cr_ = P.slab_cell[s];
    const int32_t t = P.slab_layer[s];
    const uint32_t off = P.slab_off[s], n = P.slab_n[s];
    const int32_t cx = P.cell_idx[3 * cr_], cy = P.cell_idx[3 * cr_ + 1], cz = P.cell_idx[3 * cr_ + 2];
    const uint32_t sb = P.cell_sb[cr_];
    // reference slot: the one holding the cell centre (metadata.rs:104-106)
    const I3 c0 = hex_from_world(cell_pos1(cx, P.cs), cell_pos1(cy, P.cs), cell_pos1(cz, P.cs), P.cr);
    const int32_t rx = c0.x - P.tx / 2, ry = c0.y - P.ty / 2;
    uint32_t err = 0;
    if (tid == 0) atomicAdd(DENSE ? &P.ctr->dense_arrivals : &P.ctr->small_arrivals, (unsigned long long)n);

    for (int i = tid; i < TAB; i += BS) {
        S.tab[i] = kEmpty64;
        if constexpr (!DENSE) S.tkey[i] = kEmpty32;
    }
    for (int i = tid; i < CLAIM; i += BS) S.claim[i] = kEmpty32;
    if (tid < kDests) { S.dcnt[tid] = 0; S.dcur[tid] = 0; }
    if (tid < NW * kDests) { (&S.wcnt[0][0])[tid] = 0; }
    if (tid == 0) { S.nwin = 0; S.wctr = 0; S.err = 0; }
    __syncthreads();

    // ---------------------------------------------------------------- sweep 1
    for (uint32_t base = 0; base < n; base += BS) {
        const uint32_t j = base + tid;
        if (j < n) {
            const float x = P.in.x[off + j], y = P.in.y[off + j], z = P.in.z[off + j];
            const I3 sl = hex_from_world(x, y, z, P.cr);
            const int32_t lx = sl.x - rx, ly = sl.y - ry;
            if (sl.z != t) err |= ERR_LAYER;
            else if (lx < 0 || ly < 0 || lx >= P.tx || ly >= P.ty) err |= ERR_SLOT_RANGE;
            else {
                const int e = slot_entry<DENSE>(S, (uint32_t)(ly * P.tx + lx), true);
                float X, Y, Z;
                hex_to_world(sl, P.cr, X, Y, Z);
                const float d2 = dist2(X, Y, Z, x, y, z);
                const unsigned long long pk = ((unsigned long long)f2u(d2) << 32) | j;
                const unsigned long long old = atomicMin(&S.tab[e], pk);
                if (old == kEmpty64) atomicAdd(&S.nwin, 1u);
                const int d = dest_of(P, cx, cy, cz, t, x, y, z, err);
                if (d >= 0) atomicAdd(&S.dcnt[d], 1u);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        const uint32_t wb = atomicAdd(&P.ctr->out_cur, S.nwin);
        S.wbase = wb;
        P.slab_grid_off[s] = wb;
        P.slab_grid_n[s] = S.nwin;
        atomicAdd(&P.ctr->grid_total, (unsigned long long)S.nwin);
    }
    __syncthreads();
    // winners -> output arena (grid points; order inside a cell is free: cell.rs:158-160 HashMap order)
    for (int i = tid; i < TAB; i += BS) {
        const unsigned long long e = S.tab[i];
        if (e != kEmpty64) {
            const uint32_t j = (uint32_t)e;
            const float x = P.in.x[off + j], y = P.in.y[off + j], z = P.in.z[off + j];
            const uint32_t c = P.in.c[off + j];
            const int d = dest_of(P, cx, cy, cz, t, x, y, z, err);
            if (d >= 0) atomicSub(&S.dcnt[d], 1u);
            const uint32_t r = atomicAdd(&S.wctr, 1u);
            Point p;
            p.x = x; p.y = y; p.z = z;
            memcpy(p.rgba, &c, 4);
            P.out[S.wbase + r] = p;
            S.tab[i] = kEmpty64;
        }
    }
    __syncthreads();
    if (tid < kDests) {
        const uint32_t c = S.dcnt[tid];
        const uint32_t o = c ? atomicAdd(&P.ctr->arena_cur, c) : 0u;
        S.doff[tid] = o;
        P.dest_off[s * kDests + tid] = o;
        P.dest_n[s * kDests + tid] = c;
    }
    __syncthreads();

    // ---------------------------------------------------------------- sweep 2
    const uint64_t lt = lanemask_lt();
    for (uint32_t base = 0; base < n; base += BS) {
        const uint32_t j = base + tid;
        bool pending = false;
        float x = 0, y = 0, z = 0, d2 = 0;
        uint32_t c = 0, k = 0, eb = 0, ch = 0;
        int e = 0;
        if (j < n) {
            x = P.in.x[off + j]; y = P.in.y[off + j]; z = P.in.z[off + j];
            c = P.in.c[off + j]; k = P.in.k[off + j]; eb = max(P.in.e[off + j], sb);
            const I3 sl = hex_from_world(x, y, z, P.cr);
            const int32_t lx = sl.x - rx, ly = sl.y - ry;
            if (sl.z == t && lx >= 0 && ly >= 0 && lx < P.tx && ly < P.ty) {
                e = slot_entry<DENSE>(S, (uint32_t)(ly * P.tx + lx), false);
                if (e >= 0) {
                    float X, Y, Z;
                    hex_to_world(sl, P.cr, X, Y, Z);
                    d2 = dist2(X, Y, Z, x, y, z);
                    pending = true;
                    ch = (uint32_t)e & (CLAIM - 1);
                }
            }
        }
        // cell.rs:70-94 replayed in key order: per round, the earliest pending
        // arrival of every slot (claim = min thread index) is applied.
        int32_t em = -1;
        for (;;) {
            if (pending) atomicMin(&S.claim[ch], tid);
            __syncthreads();
            bool won = false;
            if (pending && S.claim[ch] == tid) {
                const unsigned long long occ = S.tab[e];
                const unsigned long long mine = ((unsigned long long)f2u(d2) << 32) | j;
                if (occ == kEmpty64) {
                    S.tab[e] = mine;
                } else if (d2 < __uint_as_float((uint32_t)(occ >> 32))) {  // strict: ties keep the old point
                    S.tab[e] = mine;
                    em = (int32_t)(uint32_t)occ;   // displaced occupant, emitted at this arrival's key
                } else {
                    em = (int32_t)j;               // the arrival itself overflows
                }
                pending = false;
                won = true;
            }
            __syncthreads();
            if (won) S.claim[ch] = kEmpty32;
            if (!__syncthreads_or(pending)) break;
        }
        // emission: point (self or displaced), key/eb of this arrival
        int d = -1;
        float ex = x, ey = y, ez = z;
        uint32_t ec = c;
        if (em >= 0) {
            if ((uint32_t)em != j) {
                ex = P.in.x[off + em]; ey = P.in.y[off + em]; ez = P.in.z[off + em]; ec = P.in.c[off + em];
            }
            d = dest_of(P, cx, cy, cz, t, ex, ey, ez, err);
        }
        const bool v = d >= 0;
        uint64_t same = __ballot(v);
#pragma unroll
        for (int b = 0; b < 5; b++) {
            const uint64_t bb = __ballot(v && ((d >> b) & 1));
            same &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rw = __popcll(same & lt);
        if (v && rw == 0) S.wcnt[wv][d] = (uint32_t)__popcll(same);
        __syncthreads();
        if (tid < kDests) {
            uint32_t acc = S.dcur[tid];
#pragma unroll
            for (int q = 0; q < NW; q++) { const uint32_t cc = S.wcnt[q][tid]; S.wpre[q][tid] = acc; acc += cc; S.wcnt[q][tid] = 0; }
            S.dcur[tid] = acc;
        }
        __syncthreads();
        if (v) {
            const uint32_t pos = S.doff[d] + S.wpre[wv][d] + rw;
            P.nx.x[pos] = ex; P.nx.y[pos] = ey; P.nx.z[pos] = ez;
            P.nx.c[pos] = ec; P.nx.k[pos] = k; P.nx.e[pos] = eb;
        }
    }
    if (err) atomicOr(&S.err, err);
    __syncthreads();
    if (tid == 0 && S.err) set_err(P.ctr, S.err);
}

// ------------------------------------------------------------------ bucket resolution
struct BucketParams {
    Arena nx;          // arrivals of level h+1 (== emissions of level h)
    Point* out;
    const uint32_t* cell_slab0;
    const int32_t* slab_layer;
    const uint32_t* dest_off;
    const uint32_t* dest_n;
    uint32_t* bkt_state;
    uint32_t* bkt_off;
    uint32_t* bkt_n;
    uint32_t* bkt_sb;
    uint32_t* bkt_nd;
    Counters* ctr;
    uint32_t L;
};

constexpr int kBktBS = 256;

// number of elements with eb <= e among the first min(n, cap) of a key-ordered dest list
__device__ __forceinline__ uint32_t count_le(const uint32_t* E, uint32_t off, uint32_t n, uint32_t cap, uint32_t e) {
    uint32_t lo = 0, hi = n < cap ? n : cap;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (E[off + mid] <= e) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// cell.rs:108-153 add_points_in_overflow, resolved for all batches at once
// (SURVEY.md Appendix C.3): bucket = (cell, child octant), emissions key-ordered
// inside each of its child slabs.
__global__ __launch_bounds__(kBktBS) void k_bucket(BucketParams B) {
    __shared__ uint32_t lds[kBktBS / 64 + 1];
    __shared__ uint32_t skey[kKeptMax], spos[kKeptMax];
    __shared__ uint32_t s_cnt, s_off;
    __shared__ uint32_t s_min, s_max;
    const uint32_t b = blockIdx.x, cell = b >> 3, oct = b & 7;
    const uint32_t s0 = B.cell_slab0[cell], s1 = B.cell_slab0[cell + 1];
    const uint32_t nd = (s1 - s0) * 3;
    const uint32_t L = B.L;
    uint32_t tot = 0, nne = 0, emin = 0xFFFFFFFFu, emax = 0;
    for (uint32_t i = threadIdx.x; i < nd; i += kBktBS) {
        const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
        const uint32_t n = B.dest_n[di];
        if (n) {
            const uint32_t o = B.dest_off[di];
            tot += n;
            nne++;
            emin = min(emin, B.nx.e[o]);
            emax = max(emax, B.nx.e[o + n - 1]);
        }
    }
    if (threadIdx.x == 0) { s_min = 0xFFFFFFFFu; s_max = 0; }
    __syncthreads();
    atomicMin(&s_min, emin);
    atomicMax(&s_max, emax);
    tot = block_sum<kBktBS>(tot, lds);
    nne = block_sum<kBktBS>(nne, lds);
    emin = s_min;
    emax = s_max;
    if (tot == 0) {
        if (threadIdx.x == 0) { B.bkt_state[b] = 0; B.bkt_n[b] = 0; B.bkt_nd[b] = 0; B.bkt_off[b] = 0; B.bkt_sb[b] = 0; }
        return;
    }
    const bool spilled = tot > L || (tot == L && emin != emax);
    if (!spilled) {
        // Some(list): the bucket's points in key order, kept in this cell's file
        if (tot > (uint32_t)kKeptMax) {
            if (threadIdx.x == 0) { set_err(B.ctr, ERR_KEPT_CAP); B.bkt_state[b] = 0; }
            return;
        }
        if (threadIdx.x == 0) { s_cnt = 0; s_off = atomicAdd(&B.ctr->out_cur, tot); }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nd; i += kBktBS) {
            const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
            const uint32_t n = B.dest_n[di];
            if (n) {
                const uint32_t o = B.dest_off[di];
                const uint32_t p = atomicAdd(&s_cnt, n);
                for (uint32_t q = 0; q < n; q++) { skey[p + q] = B.nx.k[o + q]; spos[p + q] = o + q; }
            }
        }
        uint32_t np2 = 1;
        while (np2 < tot) np2 <<= 1;
        __syncthreads();
        for (uint32_t i = tot + threadIdx.x; i < np2; i += kBktBS) { skey[i] = 0xFFFFFFFFu; spos[i] = 0; }
        __syncthreads();
        // bitonic sort by key (keys are unique)
        for (uint32_t kk = 2; kk <= np2; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                for (uint32_t i = threadIdx.x; i < np2; i += kBktBS) {
                    const uint32_t ix = i ^ jj;
                    if (ix > i) {
                        const bool up = (i & kk) == 0;
                        const uint32_t a = skey[i], c = skey[ix];
                        if ((a > c) == up) {
                            skey[i] = c; skey[ix] = a;
                            const uint32_t t2 = spos[i]; spos[i] = spos[ix]; spos[ix] = t2;
                        }
                    }
                }
                __syncthreads();
            }
        for (uint32_t i = threadIdx.x; i < tot; i += kBktBS) {
            const uint32_t o = spos[i];
            Point p;
            p.x = B.nx.x[o]; p.y = B.nx.y[o]; p.z = B.nx.z[o];
            const uint32_t c = B.nx.c[o];
            memcpy(p.rgba, &c, 4);
            B.out[s_off + i] = p;
        }
        if (threadIdx.x == 0) { B.bkt_state[b] = 1; B.bkt_off[b] = s_off; B.bkt_n[b] = tot; B.bkt_nd[b] = 0; B.bkt_sb[b] = 0; }
        return;
    }
    // None: spilled.  Spill batch sb = smallest e with c(e) >= L + [c(e0) == L],
    // c(e) = #bucket emissions with eb <= e (== Appendix C.3's rank rule).
    auto count = [&](uint32_t e) -> uint32_t {
        uint32_t c = 0;
        for (uint32_t i = threadIdx.x; i < nd; i += kBktBS) {
            const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
            const uint32_t n = B.dest_n[di];
            if (n) c += count_le(B.nx.e, B.dest_off[di], n, L + 1, e);
        }
        return block_sum<kBktBS>(c, lds);
    };
    const uint32_t c0 = count(emin);
    const uint32_t target = L + (c0 == L ? 1u : 0u);
    uint32_t lo = emin, hi = emax;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (count(mid) >= target) hi = mid; else lo = mid + 1;
    }
    if (threadIdx.x == 0) { B.bkt_state[b] = 2; B.bkt_n[b] = tot; B.bkt_nd[b] = nne; B.bkt_sb[b] = lo; B.bkt_off[b] = 0; }
}

// ------------------------------------------------------------------ next level tables
__global__ void k_next_flags(const uint32_t* bkt_state, const uint32_t* bkt_nd, uint32_t nb, uint32_t* f, uint32_t* ndv) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) {
        const bool sp = bkt_state[b] == 2;
        f[b] = sp ? 1u : 0u;
        ndv[b] = sp ? bkt_nd[b] : 0u;
    }
}

struct NextParams {
    const uint32_t* bkt_state;
    const uint32_t* bkt_sb;
    const uint32_t* rank;      // exclusive scan of spilled flags
    const uint32_t* sbase;     // exclusive scan of non-empty dest counts
    const int32_t* cell_idx;
    const uint32_t* cell_slab0;
    const int32_t* slab_layer;
    const uint32_t* dest_off;
    const uint32_t* dest_n;
    int32_t* ncell_idx;
    uint32_t* ncell_sb;
    uint32_t* ncell_slab0;
    uint32_t* nslab_cell;
    int32_t* nslab_layer;
    uint32_t* nslab_off;
    uint32_t* nslab_n;
    uint32_t* nbig_list;
    uint32_t* nsmall_list;
    Counters* ctr;
};

__global__ __launch_bounds__(256) void k_next_emit(NextParams Q) {
    __shared__ uint32_t lds[256 / 64 + 1];
    __shared__ uint32_t carry;
    const uint32_t b = blockIdx.x;
    if (Q.bkt_state[b] != 2) return;
    const uint32_t cell = b >> 3, oct = b & 7;
    const uint32_t r = Q.rank[b], base = Q.sbase[b];
    if (threadIdx.x == 0) {
        // child index = 2 * parent + octant bit (floor(2q) = 2 floor(q) + {0,1})
        Q.ncell_idx[3 * r] = 2 * Q.cell_idx[3 * cell] + (int32_t)(oct & 1);
        Q.ncell_idx[3 * r + 1] = 2 * Q.cell_idx[3 * cell + 1] + (int32_t)((oct >> 1) & 1);
        Q.ncell_idx[3 * r + 2] = 2 * Q.cell_idx[3 * cell + 2] + (int32_t)((oct >> 2) & 1);
        Q.ncell_sb[r] = Q.bkt_sb[b];
        Q.ncell_slab0[r] = base;
        carry = 0;
    }
    __syncthreads();
    const uint32_t s0 = Q.cell_slab0[cell], s1 = Q.cell_slab0[cell + 1];
    const uint32_t nd = (s1 - s0) * 3;
    for (uint32_t i0 = 0; i0 < nd; i0 += 256) {
        const uint32_t i = i0 + threadIdx.x;
        uint32_t n = 0, di = 0;
        if (i < nd) {
            di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
            n = Q.dest_n[di];
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<256>(n ? 1u : 0u, lds, &tot);
        if (n) {
            const uint32_t sid = base + carry + ex;
            const int32_t t = Q.slab_layer[s0 + i / 3];
            Q.nslab_cell[sid] = r;
            Q.nslab_layer[sid] = 2 * t + (int32_t)(i % 3) - 1;
            Q.nslab_off[sid] = Q.dest_off[di];
            Q.nslab_n[sid] = n;
            atomicAdd(&Q.ctr->arrivals_next, (unsigned long long)n);
            if (n >= kSmallMax) Q.nbig_list[atomicAdd(&Q.ctr->nbig, 1u)] = sid;
            else Q.nsmall_list[atomicAdd(&Q.ctr->nsmall, 1u)] = sid;
        }
        __syncthreads();
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
}

__global__ void k_set_u32(uint32_t* p, uint32_t v) { *p = v; }

// ------------------------------------------------------------------ host side
static unsigned grid_for(uint64_t n, unsigned bs, unsigned cap = 65536) {
    uint64_t g = (n + bs - 1) / bs;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

Engine::Engine(const Config& cfg, int device, hipStream_t stream) : cfg_(cfg), device_(device), stream_(stream) {
    HIP_CHECK(hipSetDevice(device_));
    if (!stream_) {
        HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        own_stream_ = true;
    }
    dev_ = new Dev();
    HIP_CHECK(hipMalloc(&dev_->ctr, sizeof(Counters)));
    HIP_CHECK(hipMalloc(&dev_->bbox_part, kBBoxBlocks * 6 * sizeof(float)));
    HIP_CHECK(hipMalloc(&dev_->bbox_flag, sizeof(uint32_t)));
}

Engine::~Engine() {
    try {
        free_all();
    } catch (...) {
    }
    if (own_stream_) (void)hipStreamDestroy(stream_);
}

void Engine::free_all() {
    for (auto& u : ev_used_) { ev_pool_.push_back(u.second.first); ev_pool_.push_back(u.second.second); }
    ev_used_.clear();
    for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
    ev_pool_.clear();
    for (Level* l : levels_) delete l;
    levels_.clear();
    if (dev_) {
        for (int a = 0; a < 2; a++) {
            (void)hipFree(dev_->ar[a].x); (void)hipFree(dev_->ar[a].y); (void)hipFree(dev_->ar[a].z);
            (void)hipFree(dev_->ar[a].c); (void)hipFree(dev_->ar[a].k); (void)hipFree(dev_->ar[a].e);
        }
        (void)hipFree(dev_->out);
        (void)hipFree(dev_->ctr);
        (void)hipFree(dev_->bbox_part);
        (void)hipFree(dev_->bbox_flag);
        (void)hipFree(dev_->scan.bsums);
        (void)hipFree(dev_->sort.counts);
        (void)hipFree(dev_->sort.scan.bsums);
        for (auto& c : dev_->chunks) (void)hipFree(c.first);
        delete dev_;
        dev_ = nullptr;
    }
    (void)hipFree(d_in_);
    d_in_ = nullptr;
}

enum Stage { ST_L0 = 0, ST_DENSE, ST_SMALL, ST_BUCKET, ST_NEXT };

void Engine::ev_begin(int stage) {
    if (!profiling_) return;
    auto take = [&]() {
        hipEvent_t e;
        if (!ev_pool_.empty()) { e = ev_pool_.back(); ev_pool_.pop_back(); }
        else HIP_CHECK(hipEventCreate(&e));
        return e;
    };
    hipEvent_t a = take(), b = take();
    HIP_CHECK(hipEventRecord(a, stream_));
    ev_used_.push_back({stage, {a, b}});
}

void Engine::ev_end(int stage) {
    if (!profiling_) return;
    for (auto it = ev_used_.rbegin(); it != ev_used_.rend(); ++it)
        if (it->first == stage) { HIP_CHECK(hipEventRecord(it->second.second, stream_)); return; }
}

void Engine::ev_collect() {
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (auto& u : ev_used_) {
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, u.second.first, u.second.second));
        switch (u.first) {
            case ST_L0: prof_.level0_ms += ms; break;
            case ST_DENSE: prof_.dense_ms += ms; prof_.dense_launches++; break;
            case ST_SMALL: prof_.small_ms += ms; prof_.small_launches++; break;
            case ST_BUCKET: prof_.bucket_ms += ms; break;
            default: prof_.next_ms += ms; break;
        }
        ev_pool_.push_back(u.second.first);
        ev_pool_.push_back(u.second.second);
    }
    ev_used_.clear();
}

int Engine::fail(int code, const std::string& msg) {
    err_ = msg;
    return code;
}

void Engine::reserve(uint64_t n) {
    if (n <= cap_) return;
    if (n >= 0xFFFFFFFFull) throw std::runtime_error("more than 2^32-1 points per build are not supported");
    Point* p = nullptr;
    HIP_CHECK(hipMalloc(&p, std::max<uint64_t>(n, 1) * sizeof(Point)));
    if (n_) HIP_CHECK(hipMemcpyAsync(p, d_in_, n_ * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    (void)hipFree(d_in_);
    d_in_ = p;
    cap_ = n;
}

void Engine::add_file_host(const Point* pts, uint64_t n, uint32_t batch) {
    if (built_) throw std::runtime_error("engine already built");
    reserve(n_ + n);
    if (n) HIP_CHECK(hipMemcpyAsync(d_in_ + n_, pts, n * sizeof(Point), hipMemcpyHostToDevice, stream_));
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += n;
    nbatches_ += (uint32_t)std::max<uint64_t>(1, (n + std::max<uint32_t>(batch, 1) - 1) / std::max<uint32_t>(batch, 1));
    HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::add_file_device(const Point* dpts, uint64_t n, uint32_t batch) {
    if (built_) throw std::runtime_error("engine already built");
    reserve(n_ + n);
    if (n) HIP_CHECK(hipMemcpyAsync(d_in_ + n_, dpts, n * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += n;
    nbatches_ += (uint32_t)std::max<uint64_t>(1, (n + std::max<uint32_t>(batch, 1) - 1) / std::max<uint32_t>(batch, 1));
}

void Engine::add_file_synth(uint64_t seed, int kind, uint64_t n, uint32_t batch, float lo, float ext) {
    if (built_) throw std::runtime_error("engine already built");
    reserve(n_ + n);
    if (n) k_synth<<<grid_for(n, 256, 1 << 20), 256, 0, stream_>>>(d_in_, n_, n, seed, kind, lo, ext);
    HIP_CHECK(hipGetLastError());
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += n;
    nbatches_ += (uint32_t)std::max<uint64_t>(1, (n + std::max<uint32_t>(batch, 1) - 1) / std::max<uint32_t>(batch, 1));
}

int Engine::build() {
    // a repeated build() re-runs everything from the resident input (bench steps)
    for (Level* l : levels_) delete l;
    levels_.clear();
    dev_->reset_pool();
    built_ = true;
    prof_ = StageProfile();
    const auto t0 = std::chrono::steady_clock::now();
    if (cfg_.sub_grid_dimension == 0) return fail(-22, "sub_grid_dimension must be > 0");
    if (cfg_.cell_point_overflow_limit > (uint32_t)kKeptMax)
        return fail(-22, "cell_point_overflow_limit > 8192 is not supported by the GPU build");
    const SlabGeom g = slab_geom(cfg_.sub_grid_dimension);
    if (g.tx * g.ty > kDenseTab)
        return fail(-22, "sub_grid_dimension too large for the LDS slot table (max 96)");
    hierarchies_ = nbatches_ > 0 ? 1u : 0u;   // converter.rs:141-158 runs for every batch, even empty
    stats_ = BuildStats();
    if (n_ == 0) return 0;

    // allocate arenas (SoA, N entries each) + output arena (N points: grid + kept == N)
    if (dev_->cap < n_) {
        for (int a = 0; a < 2; a++) {
            Arena& A = dev_->ar[a];
            (void)hipFree(A.x); (void)hipFree(A.y); (void)hipFree(A.z); (void)hipFree(A.c); (void)hipFree(A.k); (void)hipFree(A.e);
            HIP_CHECK(hipMalloc(&A.x, n_ * 4)); HIP_CHECK(hipMalloc(&A.y, n_ * 4)); HIP_CHECK(hipMalloc(&A.z, n_ * 4));
            HIP_CHECK(hipMalloc(&A.c, n_ * 4)); HIP_CHECK(hipMalloc(&A.k, n_ * 4)); HIP_CHECK(hipMalloc(&A.e, n_ * 4));
        }
        (void)hipFree(dev_->out);
        HIP_CHECK(hipMalloc(&dev_->out, n_ * sizeof(Point)));
        dev_->cap = n_;
    }
    // file table for event batches
    {
        std::vector<uint32_t> ft;
        for (size_t f = 0; f < file_start_.size(); f++) {
            ft.push_back((uint32_t)file_start_[f]);
            ft.push_back((uint32_t)(file_start_[f] >> 32));
            ft.push_back(file_eb0_[f]);
            ft.push_back(file_batch_[f]);
        }
        dev_->files = static_cast<uint32_t*>(dev_->get(ft.size() * 4));
        HIP_CHECK(hipMemcpyAsync(dev_->files, ft.data(), ft.size() * 4, hipMemcpyHostToDevice, stream_));
    }
    HIP_CHECK(hipMemsetAsync(dev_->ctr, 0, sizeof(Counters), stream_));

    // bbox (K0)
    ev_begin(ST_L0);
    HIP_CHECK(hipMemsetAsync(dev_->bbox_flag, 0, 4, stream_));
    const unsigned nbb = grid_for(n_, kBBoxBS, kBBoxBlocks);
    k_bbox<<<nbb, kBBoxBS, 0, stream_>>>(d_in_, n_, dev_->bbox_part, dev_->bbox_flag);
    k_bbox_final<<<1, 64, 0, stream_>>>(dev_->bbox_part, nbb);
    HIP_CHECK(hipGetLastError());
    float bb[6];
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(bb, dev_->bbox_part, sizeof bb, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(&bad, dev_->bbox_flag, 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    if (bad) return fail(-22, "input contains NaN or infinite coordinates (unsupported)");
    for (int a = 0; a < 3; a++) { bmin_[a] = bb[a]; bmax_[a] = bb[3 + a]; }

    int rc = level0_bin();
    if (rc) return rc;
    stats_.ms_level0_bin = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t h = 0;; h++) {
        if (h >= kMaxDepth) return fail(-75, "hierarchy depth limit (31) reached: more than cell_point_overflow_limit duplicate points?");
        const auto tl = std::chrono::steady_clock::now();
        rc = run_level(h);
        if (rc) return rc;
        stats_.ms_level.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count());
        if (levels_.size() == h + 1) break;   // no next level
    }
    hierarchies_ = std::max<uint32_t>(hierarchies_, (uint32_t)levels_.size());
    stats_.levels = (uint32_t)levels_.size();
    if (profiling_) {
        ev_collect();
        Counters hc;
        HIP_CHECK(hipMemcpy(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost));
        prof_.dense_arrivals = hc.dense_arrivals;
        prof_.small_arrivals = hc.small_arrivals;
    }
    stats_.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

int Engine::level0_bin() {
    const uint32_t dim = cfg_.sub_grid_dimension;
    const float cs = cell_size(cfg_.max_cell_size, 0);
    const float cr = hex_radius(sub_cell_size(cs, dim));
    L0Params P;
    P.cs = cs;
    P.cr = cr;
    const SlabGeom g = slab_geom(dim);
    P.nl = g.nl;
    P.dim2 = 2 * (int32_t)dim;
    uint64_t G = 1;
    for (int a = 0; a < 3; a++) {
        P.lo[a] = cell_index1(bmin_[a], cs);
        const int32_t hi = cell_index1(bmax_[a], cs);
        P.g[a] = hi - P.lo[a] + 1;
        G *= (uint64_t)P.g[a];
    }
    const uint64_t D = G * (uint64_t)P.nl;
    if (G > (1u << 20))
        return fail(-27, "level-0 cell grid too large (bounding box spans > 2^20 cells of max_cell_size)");
    // scratch: hist, flags and scans over D and G (reuse arena B's arrays)
    uint32_t* hist = static_cast<uint32_t*>(dev_->get(D * 4));
    uint32_t* cnt_scan = static_cast<uint32_t*>(dev_->get(D * 4));
    uint32_t* sflag = static_cast<uint32_t*>(dev_->get(D * 4));
    uint32_t* cflag = static_cast<uint32_t*>(dev_->get(G * 4));
    uint32_t* cscan = static_cast<uint32_t*>(dev_->get(G * 4));
    uint32_t* d_tot = static_cast<uint32_t*>(dev_->get(16));
    HIP_CHECK(hipMemsetAsync(hist, 0, D * 4, stream_));
    k_l0_hist<<<grid_for(n_, 256, 4096), 256, 0, stream_>>>(d_in_, n_, P, hist, (uint32_t)D, dev_->ctr);
    k_l0_flags<<<grid_for(std::max<uint64_t>(D, G), 256), 256, 0, stream_>>>(hist, (uint32_t)D, P.nl, sflag, cflag, (uint32_t)G);
    scan_excl_u32(hist, cnt_scan, (uint32_t)D, d_tot + 0, dev_->scan, stream_);
    scan_excl_u32(sflag, sflag, (uint32_t)D, d_tot + 1, dev_->scan, stream_);
    scan_excl_u32(cflag, cscan, (uint32_t)G, d_tot + 2, dev_->scan, stream_);
    uint32_t tots[3];
    Counters hc;
    HIP_CHECK(hipMemcpyAsync(tots, d_tot, 12, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    if (hc.err) return fail(-34, "level-0 binning: point outside the bounding grid (internal error)");
    if (tots[0] != n_) return fail(-5, "level-0 histogram mismatch");
    Level* L = new Level();
    L->dev = dev_;
    levels_.push_back(L);
    L->h = 0;
    L->ncells = tots[2];
    L->nslabs = tots[1];
    L->arena = 0;
    L->alloc(L->cell_idx, 3ull * L->ncells);
    L->alloc(L->cell_sb, L->ncells);
    L->alloc(L->cell_slab0, L->ncells + 1ull);
    L->alloc(L->slab_cell, L->nslabs);
    L->alloc(L->slab_layer, L->nslabs);
    L->alloc(L->slab_off, L->nslabs);
    L->alloc(L->slab_n, L->nslabs);
    L->alloc(L->big_list, L->nslabs);
    L->alloc(L->small_list, L->nslabs);
    k_l0_tables<<<grid_for(std::max<uint64_t>(D, G), 256, 1u << 30), 256, 0, stream_>>>(
        hist, cnt_scan, sflag, cflag, cscan, (uint32_t)D, (uint32_t)G, P, L->cell_idx, L->cell_sb, L->cell_slab0, L->slab_cell,
        L->slab_layer, L->slab_off, L->slab_n, L->big_list, L->small_list, dev_->ctr);
    k_set_u32<<<1, 1, 0, stream_>>>(L->cell_slab0 + L->ncells, L->nslabs);
    // keys = slab id (ordered by (cell, layer)), stable radix sort, gather into arena 0
    Arena& A0 = dev_->ar[0];
    Arena& A1 = dev_->ar[1];
    k_l0_keys<<<grid_for(n_, 256, 1 << 20), 256, 0, stream_>>>(d_in_, n_, P, sflag, A1.k, A1.e);
    int bits = 0;
    while ((1ull << bits) < L->nslabs) bits++;
    const int where = radix_sort_pairs(A1.k, A1.e, A1.x ? reinterpret_cast<uint32_t*>(A1.x) : nullptr,
                                       reinterpret_cast<uint32_t*>(A1.y), (uint32_t)n_, bits, dev_->sort, stream_);
    const uint32_t* perm = where ? reinterpret_cast<uint32_t*>(A1.y) : A1.e;
    k_l0_gather<<<grid_for(n_, 256, 1 << 20), 256, 0, stream_>>>(d_in_, perm, n_, A0, dev_->files,
                                                                   (uint32_t)file_start_.size());
    HIP_CHECK(hipGetLastError());
    ev_end(ST_L0);
    HIP_CHECK(hipMemcpyAsync(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    L->nbig = hc.nbig;
    L->nsmall = hc.nsmall;
    stats_.cells += L->ncells;
    stats_.slabs += L->nslabs;
    stats_.arrivals += n_;
    return 0;
}

int Engine::run_level(uint32_t h) {
    Level* L = levels_[h];
    const uint32_t dim = cfg_.sub_grid_dimension;
    const SlabGeom g = slab_geom(dim);
    const float cs = cell_size(cfg_.max_cell_size, h), csc = cell_size(cfg_.max_cell_size, h + 1);
    const Arena& in = dev_->ar[L->arena];
    const Arena& nx = dev_->ar[1 - L->arena];
    L->alloc(L->slab_grid_off, L->nslabs);
    L->alloc(L->slab_grid_n, L->nslabs);
    L->alloc(L->dest_off, (uint64_t)L->nslabs * kDests);
    L->alloc(L->dest_n, (uint64_t)L->nslabs * kDests);
    L->alloc(L->bkt_state, 8ull * L->ncells);
    L->alloc(L->bkt_off, 8ull * L->ncells);
    L->alloc(L->bkt_n, 8ull * L->ncells);
    L->alloc(L->bkt_sb, 8ull * L->ncells);
    L->alloc(L->bkt_nd, 8ull * L->ncells);
    // reset the next-arena cursor and the next-level counters (keep out_cur)
    {
        Counters hc;
        HIP_CHECK(hipMemcpyAsync(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        hc.arena_cur = 0;
        hc.nbig = hc.nsmall = 0;
        hc.arrivals_next = 0;
        HIP_CHECK(hipMemcpyAsync(dev_->ctr, &hc, sizeof hc, hipMemcpyHostToDevice, stream_));
    }
    SlabParams SP;
    SP.in = in;
    SP.nx = nx;
    SP.out = dev_->out;
    SP.cell_idx = L->cell_idx;
    SP.cell_sb = L->cell_sb;
    SP.slab_cell = L->slab_cell;
    SP.slab_layer = L->slab_layer;
    SP.slab_off = L->slab_off;
    SP.slab_n = L->slab_n;
    SP.slab_grid_off = L->slab_grid_off;
    SP.slab_grid_n = L->slab_grid_n;
    SP.dest_off = L->dest_off;
    SP.dest_n = L->dest_n;
    SP.ctr = dev_->ctr;
    SP.cs = cs;
    SP.cr = hex_radius(sub_cell_size(cs, dim));
    SP.cs_child = csc;
    SP.cr_child = hex_radius(sub_cell_size(csc, dim));
    SP.tx = g.tx;
    SP.ty = g.ty;
    if (L->nbig) {
        SP.list = L->big_list;
        ev_begin(ST_DENSE);
        k_slab<true><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        ev_end(ST_DENSE);
    }
    if (L->nsmall) {
        SP.list = L->small_list;
        ev_begin(ST_SMALL);
        k_slab<false><<<L->nsmall, kSmallBS, 0, stream_>>>(SP);
        ev_end(ST_SMALL);
    }
    HIP_CHECK(hipGetLastError());
    BucketParams BP;
    BP.nx = nx;
    BP.out = dev_->out;
    BP.cell_slab0 = L->cell_slab0;
    BP.slab_layer = L->slab_layer;
    BP.dest_off = L->dest_off;
    BP.dest_n = L->dest_n;
    BP.bkt_state = L->bkt_state;
    BP.bkt_off = L->bkt_off;
    BP.bkt_n = L->bkt_n;
    BP.bkt_sb = L->bkt_sb;
    BP.bkt_nd = L->bkt_nd;
    BP.ctr = dev_->ctr;
    BP.L = cfg_.cell_point_overflow_limit;
    const uint32_t nb = 8 * L->ncells;
    ev_begin(ST_BUCKET);
    k_bucket<<<nb, kBktBS, 0, stream_>>>(BP);
    ev_end(ST_BUCKET);
    HIP_CHECK(hipGetLastError());
    ev_begin(ST_NEXT);
    // next level
    uint32_t* flag = static_cast<uint32_t*>(dev_->get(nb * 4ull));
    uint32_t* ndv = static_cast<uint32_t*>(dev_->get(nb * 4ull));
    uint32_t* tots = static_cast<uint32_t*>(dev_->get(16));
    k_next_flags<<<grid_for(nb, 256, 1u << 30), 256, 0, stream_>>>(L->bkt_state, L->bkt_nd, nb, flag, ndv);
    scan_excl_u32(flag, flag, nb, tots + 0, dev_->scan, stream_);
    scan_excl_u32(ndv, ndv, nb, tots + 1, dev_->scan, stream_);
    ev_end(ST_NEXT);
    uint32_t ht[2];
    Counters hc;
    HIP_CHECK(hipMemcpyAsync(ht, tots, 8, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    stats_.grid_points = hc.grid_total;
    stats_.kept_points = hc.out_cur - hc.grid_total;
    if (hc.err) {
        char buf[160];
        snprintf(buf, sizeof buf, "device error flags 0x%x at level %u (slot range/layer/octant/sel/kept-cap)", hc.err, h);
        return fail(-5, buf);
    }
    if (ht[0] > 0) {
        Level* N = new Level();
        N->dev = dev_;
        levels_.push_back(N);
        N->h = h + 1;
        N->ncells = ht[0];
        N->nslabs = ht[1];
        N->arena = 1 - L->arena;
        N->alloc(N->cell_idx, 3ull * N->ncells);
        N->alloc(N->cell_sb, N->ncells);
        N->alloc(N->cell_slab0, N->ncells + 1ull);
        N->alloc(N->slab_cell, N->nslabs);
        N->alloc(N->slab_layer, N->nslabs);
        N->alloc(N->slab_off, N->nslabs);
        N->alloc(N->slab_n, N->nslabs);
        N->alloc(N->big_list, N->nslabs);
        N->alloc(N->small_list, N->nslabs);
        {
            Counters z = hc;
            z.nbig = z.nsmall = 0;
            HIP_CHECK(hipMemcpyAsync(dev_->ctr, &z, sizeof z, hipMemcpyHostToDevice, stream_));
        }
        NextParams Q;
        Q.bkt_state = L->bkt_state;
        Q.bkt_sb = L->bkt_sb;
        Q.rank = flag;
        Q.sbase = ndv;
        Q.cell_idx = L->cell_idx;
        Q.cell_slab0 = L->cell_slab0;
        Q.slab_layer = L->slab_layer;
        Q.dest_off = L->dest_off;
        Q.dest_n = L->dest_n;
        Q.ncell_idx = N->cell_idx;
        Q.ncell_sb = N->cell_sb;
        Q.ncell_slab0 = N->cell_slab0;
        Q.nslab_cell = N->slab_cell;
        Q.nslab_layer = N->slab_layer;
        Q.nslab_off = N->slab_off;
        Q.nslab_n = N->slab_n;
        Q.nbig_list = N->big_list;
        Q.nsmall_list = N->small_list;
        Q.ctr = dev_->ctr;
        k_next_emit<<<nb, 256, 0, stream_>>>(Q);
        k_set_u32<<<1, 1, 0, stream_>>>(N->cell_slab0 + N->ncells, N->nslabs);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        N->nbig = hc.nbig;
        N->nsmall = hc.nsmall;
        stats_.arrivals += hc.arrivals_next;
        stats_.cells += N->ncells;
        stats_.slabs += N->nslabs;
    }
    return 0;
}

int Engine::download(std::vector<LevelHost>& out, std::vector<Point>& grid, std::vector<Point>& kept) {
    out.clear();
    Counters hc;
    HIP_CHECK(hipMemcpyAsync(&hc, dev_->ctr, sizeof hc, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    grid.resize(hc.out_cur);
    if (hc.out_cur) HIP_CHECK(hipMemcpyAsync(grid.data(), dev_->out, (uint64_t)hc.out_cur * sizeof(Point), hipMemcpyDeviceToHost, stream_));
    kept.clear();   // kept lists share the output arena with the grid points
    for (Level* L : levels_) {
        LevelHost H;
        H.h = L->h;
        auto cp = [&](auto& vec, auto* dptr, uint64_t n) {
            vec.resize(n);
            if (n) HIP_CHECK(hipMemcpyAsync(vec.data(), dptr, n * sizeof(vec[0]), hipMemcpyDeviceToHost, stream_));
        };
        cp(H.cell_idx, L->cell_idx, 3ull * L->ncells);
        cp(H.cell_slab0, L->cell_slab0, L->ncells + 1ull);
        cp(H.slab_grid_off, L->slab_grid_off, L->nslabs);
        cp(H.slab_grid_n, L->slab_grid_n, L->nslabs);
        cp(H.bkt_state, L->bkt_state, 8ull * L->ncells);
        cp(H.bkt_off, L->bkt_off, 8ull * L->ncells);
        cp(H.bkt_n, L->bkt_n, 8ull * L->ncells);
        HIP_CHECK(hipStreamSynchronize(stream_));
        out.push_back(std::move(H));
    }
    return 0;
}

}  // namespace pcc
