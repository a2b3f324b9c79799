// engine.hip — MI355X-native hierarchy/LOD build (gfx950).
//
// Replaces the per-batch, per-point loop of point-converter/src/converter.rs:96-139
// and cell.rs:70-153 with the level-synchronous restatement of SURVEY.md
// Appendix C (validated in oracle/pyref.py::convert_keyed):
//
//   level-0 binning  : input points -> slabs (cell, hex z-layer), stable in key
//                      order: LSD radix sort whose keys are recomputed from the
//                      positions in every pass and which carries the payload
//                      (no key array, no random gather)
//   per level h      : one workgroup per slab, slot table in LDS, ONE pass in
//                      key order: per chunk, the earliest pending arrival of
//                      every slot is applied (cell.rs:70-94), the loser is
//                      emitted at the arrival's key straight into its child
//                      slab; winners are written at the end
//   bucket resolve   : per (cell, octant) bucket: keep (Some) or spill (None),
//                      spill batch by counting over key-ordered child slabs
//   next level       : spilled buckets become the next level's cells; their
//                      child slabs are already laid out contiguously.
//
// Every output range is known before the kernel that fills it: the parent
// level counts, per child slab, how many of its arrivals go to each of ITS
// child slabs ("capacities"), so emission and winner regions come from
// exclusive scans, not from same-address atomics.
//
// Key facts this relies on:
//   * child hex z-layer u comes from parent layer t = u/2 (truncating) because
//     r_{h+1} = r_h / 2 exactly, so each child slab has exactly ONE parent slab
//     and inherits its key order;
//   * keys (input indices) are unique at every level; event batches are
//     monotone in key inside every cell.
#include "engine.h"

#include <sys/mman.h>
#include <cerrno>
#include <memory>

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "hip_check.h"
#include "pcc_math.h"
#include "prims.h"
#include "synth.h"

namespace pcc {

// ------------------------------------------------------------------ device memory
// Large device buffers (arenas, input, pool chunks, merge seeds) are kept in a
// process-wide cache when a converter releases them and handed to the next
// converter on the same device: right after hipFree of tens of GB, the next
// hipMalloc of that size stalled for about 5 s on the MI355X boxes
// (scripts/second_conv.py).  A failed hipMalloc empties the cache and retries.
namespace {
constexpr size_t kCacheMin = size_t(64) << 20;
constexpr size_t kCacheMaxDefault = size_t(96) << 30;   // cached bytes per process, beyond: hipFree
size_t g_dev_cached = 0;
// PCC_DEVICE_CACHE_GB overrides the cap (0 disables the cache)
size_t cache_max() {
    static const size_t m = [] {
        const char* e = getenv("PCC_DEVICE_CACHE_GB");
        return e ? (size_t)(strtod(e, nullptr) * double(size_t(1) << 30)) : kCacheMaxDefault;
    }();
    return m;
}
// PCC_POISON_CACHE=1 (debug): a reused block is filled with 0xFF before it is
// handed out, so a read of memory the build never wrote shows up in parity tests.
bool poison_cache() {
    const char* e = getenv("PCC_POISON_CACHE");
    return e && e[0] == '1';
}
struct DevBlock { void* p; size_t bytes; int device; };
std::mutex g_dev_mu;
std::vector<DevBlock> g_dev_free;                 // cached, unused
std::unordered_map<void*, DevBlock> g_dev_live;   // handed out by dev_alloc
}  // namespace

static void* dev_alloc(size_t bytes) {
    bytes = std::max<size_t>(bytes, 1);
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    {
        std::lock_guard<std::mutex> g(g_dev_mu);
        size_t best = SIZE_MAX;
        for (size_t i = 0; i < g_dev_free.size(); i++) {   // the smallest cached block that fits, not far larger
            const DevBlock& b = g_dev_free[i];
            if (b.device == dev && b.bytes >= bytes && b.bytes <= bytes + bytes / 4 + kCacheMin &&   // (not far larger)
                (best == SIZE_MAX || b.bytes < g_dev_free[best].bytes))
                best = i;
        }
        if (best != SIZE_MAX) {
            const DevBlock b = g_dev_free[best];
            g_dev_free.erase(g_dev_free.begin() + (ptrdiff_t)best);
            g_dev_cached -= b.bytes;
            g_dev_live[b.p] = b;
            if (poison_cache()) { HIP_CHECK(hipMemset(b.p, 0xFF, b.bytes)); HIP_CHECK(hipDeviceSynchronize()); }
            return b.p;
        }
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {   // out of memory: give the cached blocks back and retry
        (void)hipGetLastError();
        std::vector<DevBlock> drop;
        {
            std::lock_guard<std::mutex> g(g_dev_mu);
            for (size_t i = 0; i < g_dev_free.size();) {
                if (g_dev_free[i].device == dev) {
                    drop.push_back(g_dev_free[i]);
                    g_dev_cached -= g_dev_free[i].bytes;
                    g_dev_free.erase(g_dev_free.begin() + (ptrdiff_t)i);
                } else {
                    i++;
                }
            }
        }
        for (const DevBlock& b : drop) (void)hipFree(b.p);
        HIP_CHECK(hipMalloc(&p, bytes));
    }
    std::lock_guard<std::mutex> g(g_dev_mu);
    g_dev_live[p] = DevBlock{p, bytes, dev};
    return p;
}

static void dev_release(void* p) {
    if (!p) return;
    DevBlock b{};
    {
        std::lock_guard<std::mutex> g(g_dev_mu);
        auto it = g_dev_live.find(p);
        if (it == g_dev_live.end()) {   // not ours
            (void)hipFree(p);
            return;
        }
        b = it->second;
        g_dev_live.erase(it);
        if ((b.bytes >= kCacheMin || poison_cache()) && g_dev_cached + b.bytes <= cache_max()) {   // poison: cache all
            g_dev_free.push_back(b);
            g_dev_cached += b.bytes;
            return;
        }
    }
    (void)hipFree(b.p);
}

size_t release_device_cache() {
    std::vector<DevBlock> drop;
    {
        std::lock_guard<std::mutex> g(g_dev_mu);
        drop.swap(g_dev_free);
        g_dev_cached = 0;
    }
    size_t bytes = 0;
    int cur = 0;
    HIP_CHECK(hipGetDevice(&cur));
    for (const DevBlock& b : drop) {
        if (b.device != cur) (void)hipSetDevice(b.device);
        (void)hipFree(b.p);
        if (b.device != cur) (void)hipSetDevice(cur);
        bytes += b.bytes;
    }
    return bytes;
}

template <class T>
static void dev_alloc_t(T*& p, size_t bytes) {
    p = static_cast<T*>(dev_alloc(bytes));
}

// ------------------------------------------------------------------ constants
constexpr uint64_t kEmpty64 = ~0ull;
constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;
constexpr int kDenseBS = 1024;
constexpr int kDenseTab = 116 * 132;  // one z-layer of a dim-96 cell (slab_geom)
#ifndef PCC_SLAB_PF
#define PCC_SLAB_PF 2
#endif
#ifndef PCC_L0_SWZ
#define PCC_L0_SWZ 1        // level-0 pass 1: padded pair-count rows
#endif
#ifndef PCC_STREAM_MAX
#define PCC_STREAM_MAX 24576
#endif
#ifndef PCC_STREAM_V
#define PCC_STREAM_V 4
#endif
#ifndef PCC_LPT
#define PCC_LPT 1   // dense slabs of skewed levels launched largest first
#endif
constexpr uint32_t kDenseStreamMax = PCC_STREAM_MAX;   // k_slab: stream (not gather) the grid points up to this many arrivals
constexpr int kSmallBS = 256;
constexpr uint32_t kSmallMax = 1024;  // slabs with fewer arrivals use the hashed kernel
constexpr int kSmallTab = 2048;
constexpr int kSmallClaim = 512;
constexpr int kKeptMax = 8192;        // LDS sort capacity for kept (Some) buckets
constexpr int kDests = 24;            // 8 octants x 3 child layers per slab
constexpr uint32_t kMaxDepth = 31;    // 2u32.pow(h) overflows at h = 32 (metadata.rs:92)
constexpr uint64_t kWideMax = 1ull << 24;  // points per build with a sub-grid beyond the dense table (build_wide)
constexpr int kInfSaturated = -10022;   // build_infinite: finite cells could meet the infinite ones (-EINVAL to callers)

enum ErrBits : uint32_t {
    ERR_SLOT_RANGE = 1u << 0,
    ERR_LAYER = 1u << 1,
    ERR_OCTANT = 1u << 2,
    ERR_SEL = 1u << 3,
    ERR_KEPT_CAP = 1u << 4,
    ERR_L0_RANGE = 1u << 5,
    ERR_CAPACITY = 1u << 6,
    ERR_CLAIM = 1u << 7,
    ERR_SLAB_SIZE = 1u << 8,
    ERR_ARENA = 1u << 9,   // child-slab capacities beyond the next arena (their regions are clamped to it)
};

struct Counters {
    uint32_t kept_cur;    // kept-list cursor inside the level's kept region
    uint32_t err;
    uint32_t nbig, nsmall;
    uint32_t max_slab, pad0;
    unsigned long long arrivals_next;  // sum of next-level slab sizes
    unsigned long long grid_total;     // grid winners written so far (all levels)
    unsigned long long kept_total;
    unsigned long long dense_arrivals, small_arrivals;
};

// One level's arrivals: the 16-B record (x, y, z, rgba bits) as one float4 so
// every load/store of a point is a single dwordx4, and the key (input index)
// apart.  The event batch is not stored: inside a level-h cell it is
// max(eb0(key), cell_sb) (lib.rs:31-52 batches, SURVEY.md Appendix C.3
// eb' = max(eb, sb) along the cell's ancestor chain, whose spill batches only
// grow), recomputed where it is needed (k_bucket).
struct Arena {
    float4* p;
    uint32_t* k;
};

struct Engine::Dev {
    Arena ar[2] = {};
    Counters* ctr = nullptr;
    float* bbox_part = nullptr;     // per-block min/max partials
    uint32_t* bbox_flag = nullptr;
    uint32_t* hst = nullptr;        // pinned host staging of the level-0 segment starts
    uint64_t hst_cap = 0;
    uint32_t* files = nullptr;      // per file: start_lo, start_hi, eb0, batch
    uint32_t* rb_dev = nullptr;     // readback: small device values gathered into one block,
    uint32_t* rb_host = nullptr;    //   copied in one transfer to pinned host memory
    ScanTemp scan;
    uint64_t cap = 0;
    // chunked bump allocator for per-build tables and output regions (reset at
    // every build, chunks kept for the next build)
    std::vector<std::pair<uint8_t*, uint64_t>> chunks;
    size_t chunk_i = 0;
    uint64_t chunk_used = 0;
    void* get(uint64_t bytes) {
        bytes = (std::max<uint64_t>(bytes, 1) + 255) & ~255ull;
        while (chunk_i < chunks.size() && chunk_used + bytes > chunks[chunk_i].second) { chunk_i++; chunk_used = 0; }
        if (chunk_i == chunks.size()) {
            uint64_t sz = std::max<uint64_t>(bytes, 256ull << 20);
            uint8_t* p = nullptr;
            dev_alloc_t(p, sz);
            chunks.push_back({p, sz});
            chunk_used = 0;
        }
        void* r = chunks[chunk_i].first + chunk_used;
        chunk_used += bytes;
        return r;
    }
    void reset_pool() { chunk_i = 0; chunk_used = 0; }
    // scratch taken after a build (downloads) is returned with release(mark())
    uint64_t mark() const { return ((uint64_t)chunk_i << 40) | chunk_used; }
    void release(uint64_t m) { chunk_i = (size_t)(m >> 40); chunk_used = m & ((1ull << 40) - 1); }
};

struct Engine::Level {
    uint32_t h = 0, ncells = 0, nslabs = 0, nbig = 0, nsmall = 0;
    uint64_t arrivals = 0;           // sum of slab_n
    int arena = 0;
    Engine::Dev* dev = nullptr;
    int32_t* cell_idx = nullptr;     // 3 * ncells
    uint32_t* cell_sb = nullptr;     // spill batch of the parent bucket (running max along the ancestors)
    uint32_t* cell_slab0 = nullptr;  // ncells + 1
    uint32_t* slab_cell = nullptr;
    int32_t* slab_layer = nullptr;
    uint32_t* slab_off = nullptr;
    uint32_t* slab_n = nullptr;
    uint32_t* big_list = nullptr;
    uint32_t* small_list = nullptr;
    uint32_t* dcap = nullptr;        // 24 * nslabs: arrivals of this slab per child slab (capacity)
    uint32_t* dest_off = nullptr;    // 24 * nslabs: exclusive scan of dcap = emission regions (next arena)
    uint32_t* dest_n = nullptr;      // 24 * nslabs: emissions actually written
    uint32_t max_slab = 0;           // largest slab (arrivals)
    uint32_t* gcap = nullptr;        // 24 * 24 * nslabs: capacities of the child slabs' own child slabs
    uint32_t* grid_off = nullptr;    // exclusive scan of slab_n = winner regions (capacity n)
    uint32_t* slab_grid_n = nullptr;
    Point* grid = nullptr;           // this level's winner region (arrivals entries)
    Point* kept = nullptr;           // this level's kept-list region
    uint64_t kept_cap = 0;
    unsigned long long* ksort = nullptr;   // limit > kKeptMax: sort scratch of the kept lists (2 words per point)
    uint32_t kept_used = 0;
    uint32_t* bkt_state = nullptr;   // 8 * ncells
    uint32_t* bkt_off = nullptr;
    uint32_t* bkt_n = nullptr;
    uint32_t* bkt_sb = nullptr;
    uint32_t* bkt_nd = nullptr;
    uint32_t* slab_prior = nullptr;  // merge: the existing cloud's record of each slab (kNoPriorSlab: none)
    uint32_t* room = nullptr;        // merge: 24 per slab, seeds injected in front of each child slab's emissions
    template <class T>
    void alloc(T*& p, uint64_t n) { p = static_cast<T*>(dev->get(n * sizeof(T))); }
};

// ------------------------------------------------------------------ diagnostics
// Diagnostic build only (-DPCC_STAMPS): per-wave s_memtime phase sums of the
// slab kernel, added into P.stamps[phase]; never compiled into the product.
#ifdef PCC_STAMPS
#define STAMP_DECL unsigned long long st_t0 = __builtin_amdgcn_s_memtime(), st_acc[16] = {};
#define STAMP(ph) do { const unsigned long long st_n = __builtin_amdgcn_s_memtime(); st_acc[ph] += st_n - st_t0; st_t0 = st_n; } while (0)
#define STAMP_COUNT(ph, v) do { st_acc[ph] += (v); } while (0)
#define STAMP_FLUSH(ptr) do { if ((threadIdx.x & 63) == 0 && (blockIdx.x & 63) == 0) for (int q_ = 0; q_ < 16; q_++) atomicAdd((ptr) + q_, st_acc[q_]); } while (0)
#else
#define STAMP_DECL
#define STAMP(ph) do {} while (0)
#define STAMP_COUNT(ph, v) do {} while (0)
#define STAMP_FLUSH(ptr) do {} while (0)
#endif

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ void set_err(Counters* c, uint32_t bit) { atomicOr(&c->err, bit); }

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }

// A per-lane select that stays one v_cndmask: both operands are computed on
// every lane first.  (A conditional operator with arms of a few instructions
// is emitted as a branch, i.e. an exec-mask region of 2-3 SALU per wave; the
// dense slab kernel's 16 waves share the CU's scalar unit.)
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t t, uint32_t f) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(c);
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
__device__ __forceinline__ int32_t vsel(bool c, int32_t t, int32_t f) {
    return (int32_t)vsel(c, (uint32_t)t, (uint32_t)f);
}

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

// Child slab of a point living in slab (cell c, layer t) at the current level:
// octant from cell_index at the next level (metadata.rs:100-102; child index =
// 2*parent + bit since floor(2q) = 2 floor(q) + {0,1}) and child layer
// u = trunc(z / r_child) in {2t-1, 2t, 2t+1} -> sel = u - 2t + 1.
// Returns 0..23 or -1 (sets err); also returns the child cell index and layer.
__device__ __forceinline__ int route(float csc, float crc, int32_t cx, int32_t cy, int32_t cz, int32_t t, float x,
                                     float y, float z, int32_t& ix, int32_t& iy, int32_t& iz, int32_t& u,
                                     uint32_t& err) {
    ix = cell_index1(x, csc);
    iy = cell_index1(y, csc);
    iz = cell_index1(z, csc);
    u = sat_i32(z / crc);
    const int32_t bx = ix - 2 * cx, by = iy - 2 * cy, bz = iz - 2 * cz;
    const int32_t sel = u - 2 * t + 1;
    const bool bad_oct = ((bx | by | bz) & ~1) != 0;
    const bool bad_sel = sel < 0 || sel > 2;
    err |= bad_oct ? (uint32_t)ERR_OCTANT : (bad_sel ? (uint32_t)ERR_SEL : 0u);
    return (bad_oct || bad_sel) ? -1 : (bx | (by << 1) | (bz << 2)) * 3 + sel;
}

// Per-level constants for the slot / routing arithmetic (all computed on the
// host with the reference's own f32 formulas; see pcc_math.h).
struct LevelGeo {
    float cr, crx, cry, inv_cr;          // hex radius, cr*S3, (-cr)*S3 (hex.rs:69-70), 1/cr
    float inv_crx, inv_cry;              // RN(1/crx), RN(1/cry)
    float csc, inv_csc, crc, inv_crc;    // child level cell size / hex radius
    float csg, inv_csg, crg, inv_crg;    // grandchild level
    int32_t exact;                       // a divisor outside [2^-60, 2^60]: IEEE divisions only
};

// floorf(fl(a / b)) and truncf(fl(a / b)) without a full division in the common
// case: the product with the correctly rounded reciprocal differs from the
// correctly rounded quotient by at most ~4 ulp, so unless it lies within a
// (16x wider) margin of an integer, both have the same floor/trunc.  Lanes near
// an integer are recomputed with the exact IEEE division.
// Same quotients with the ambiguity test only accumulated: callers OR the flags
// of all their divisions and resolve flagged lanes with exact IEEE divisions
// behind ONE wave-uniform branch (one ballot per point instead of one per
// division).  (k_dcap; the slab kernels use the exact quotients of div_rc.)
// An integer lies within m = |q| 2^-20 + 2^-126 of q: fract(q + m) <= 2m, tested
// against 3m to absorb the rounding of q + m (conservative; any |q| >= 2^23 is
// flagged).
__device__ __forceinline__ bool near_int(float q) {
    const float m = fmaf(fabsf(q), 0x1p-20f, 0x1p-126f);
    const float m3 = fmaf(fabsf(q), 0x3p-20f, 0x3p-126f);
    return __builtin_amdgcn_fractf(q + m) <= m3;
}
__device__ __forceinline__ float floor_q(float a, float inv_b, bool& amb) {
    const float q = a * inv_b;
    amb |= near_int(q);
    return floorf(q);
}
__device__ __forceinline__ float trunc_q(float a, float inv_b, bool& amb) {
    const float q = a * inv_b;
    amb |= near_int(q);
    return truncf(q);
}
// a / b correctly rounded from y = RN(1/b): q0 = RN(a*y) is within an ulp of
// a/b, the residual a - b*q0 is exact with an FMA, and RN(q0 + r*y) = RN(a/b)
// (Markstein; tests/div_rc_check.c compares it with IEEE division).  Valid
// without over/underflow of the intermediates: the callers keep the operands
// in {0} U [2^-60, 2^60] and the divisors in [2^-60, 2^60] (rc_ok, G.exact), so
// every quotient is normal or zero.
__device__ __forceinline__ float div_rc(float a, float b, float y) {
    const float q0 = a * y;
    const float r = fmaf(-b, q0, a);
    return fmaf(r, y, q0);
}
__device__ __forceinline__ bool rc_ok(float a) {   // 0, or |a| in [2^-60, 2^60]
    return fabsf(a) <= 0x1p60f && (uint32_t)(__builtin_amdgcn_frexp_expf(a) + 58) <= 118u;
}
// hex.rs:67-85 with the exact quotients; the sums t1 + t3 and t1 + t2 are 0 or
// at least 2^-24 in magnitude for coordinates in range, so /3 stays normal.
__device__ __forceinline__ I3 hex_q(float px, float py, float pz, const LevelGeo& G) {
    const float x = div_rc(px, G.crx, G.inv_crx);
    const float y = div_rc(py, G.cry, G.inv_cry);
    const float t = (kSqrt3 * y) + 1.0f;
    const float t1 = floorf(t + x);
    const float t2 = t - x;
    const float t3 = (2.0f * x) + 1.0f;
    const int32_t q = sat_i32(floorf(div_rc(t1 + t3, 3.0f, 0x1.555556p-2f)));
    const int32_t r = (int32_t)(0u - (uint32_t)sat_i32(floorf(div_rc(t1 + t2, 3.0f, 0x1.555556p-2f))));
    const int32_t h = sat_i32(truncf(div_rc(pz, G.cr, G.inv_cr)));
    I3 o = {q + (r - (r & 1)) / 2, r, h};
    return o;
}
// child cell index and hex layer of a point at the next level (metadata.rs:100-102, hex.rs:83)
struct RouteIdx { int32_t ix, iy, iz, u; };
__device__ __forceinline__ RouteIdx route_idx_q(float cs, float inv_cs, float inv_cr, float x, float y, float z,
                                               bool& amb) {
    RouteIdx R;
    R.ix = sat_i32(floor_q(x, inv_cs, amb));
    R.iy = sat_i32(floor_q(y, inv_cs, amb));
    R.iz = sat_i32(floor_q(z, inv_cs, amb));
    R.u = sat_i32(trunc_q(z, inv_cr, amb));
    return R;
}
__device__ __forceinline__ RouteIdx route_idx_exact(float cs, float cr, float x, float y, float z) {
    RouteIdx R;
    R.ix = cell_index1(x, cs);
    R.iy = cell_index1(y, cs);
    R.iz = cell_index1(z, cs);
    R.u = sat_i32(z / cr);
    return R;
}
// child slab (octant * 3 + layer select) of a point with child index R inside
// parent cell (cx, cy, cz) / layer t; -1 (and err) if inconsistent
__device__ __forceinline__ int route_dest(const RouteIdx& R, int32_t cx, int32_t cy, int32_t cz, int32_t t,
                                          uint32_t& err) {
    const int32_t bx = R.ix - 2 * cx, by = R.iy - 2 * cy, bz = R.iz - 2 * cz;
    const int32_t sel = R.u - 2 * t + 1;
    const bool bad_oct = ((bx | by | bz) & ~1) != 0;
    const bool bad_sel = sel < 0 || sel > 2;
    err |= bad_oct ? (uint32_t)ERR_OCTANT : (bad_sel ? (uint32_t)ERR_SEL : 0u);
    return (bad_oct || bad_sel) ? -1 : (bx | (by << 1) | (bz << 2)) * 3 + sel;
}
// route_dest without the error code (callers derive the codes on the rare
// failing lanes only)
__device__ __forceinline__ int route_dest_nc(const RouteIdx& R, int32_t cx, int32_t cy, int32_t cz, int32_t t) {
    const int32_t bx = R.ix - 2 * cx, by = R.iy - 2 * cy, bz = R.iz - 2 * cz;
    const int32_t sel = R.u - 2 * t + 1;
    const bool bad = (((bx | by | bz) & ~1) != 0) || (uint32_t)sel > 2u;
    return bad ? -1 : (bx | (by << 1) | (bz << 2)) * 3 + sel;
}
struct SlotRoute;
__device__ __forceinline__ uint32_t slot_route_errs(const SlotRoute& sr, bool layer_ok, bool range_ok, int32_t cx,
                                                    int32_t cy, int32_t cz, int32_t t, bool check_g);
// slot, child route and grandchild route of one point, one ballot for all
// divisions.  The grandchild level halves cell size and hex radius exactly
// (metadata.rs:92,96: powers of two), so x / cs_g = 2 * RN(x / cs_c) exactly and
// one quotient per axis gives both: grandchild index ig = floor(2q), child index
// floor(q) = ig >> 1; layers u_g = trunc(2q), u_c = u_g / 2 (C division
// truncates).  Quotients with |2q| >= 2^30 take the exact path.
struct SlotRoute { I3 sl; RouteIdx rc, rg; };
__device__ __forceinline__ SlotRoute slot_route(float x, float y, float z, const LevelGeo& G) {
    bool amb = G.exact || !(rc_ok(x) && rc_ok(y) && rc_ok(z));
    SlotRoute S;
    S.sl = hex_q(x, y, z, G);
    const float qx = div_rc(x, G.csg, G.inv_csg), qy = div_rc(y, G.csg, G.inv_csg);
    const float qz = div_rc(z, G.csg, G.inv_csg), qu = div_rc(z, G.crg, G.inv_crg);
    amb |= fmaxf(fmaxf(fabsf(qx), fabsf(qy)), fmaxf(fabsf(qz), fabsf(qu))) >= 0x1p30f;
    S.rg.ix = sat_i32(floorf(qx));
    S.rg.iy = sat_i32(floorf(qy));
    S.rg.iz = sat_i32(floorf(qz));
    S.rg.u = sat_i32(truncf(qu));
    S.rc.ix = S.rg.ix >> 1;
    S.rc.iy = S.rg.iy >> 1;
    S.rc.iz = S.rg.iz >> 1;
    S.rc.u = S.rg.u / 2;
    if (__ballot(amb)) {
        if (amb) {
            S.sl = hex_from_world(x, y, z, G.cr);
            S.rc = route_idx_exact(G.csc, G.crc, x, y, z);
            S.rg = route_idx_exact(G.csg, G.crg, x, y, z);
        }
    }
    return S;
}

// Error codes of a point whose slot or routes failed (computed on those rare
// lanes only; the common path uses route_dest_nc).
__device__ __forceinline__ uint32_t slot_route_errs(const SlotRoute& sr, bool layer_ok, bool range_ok, int32_t cx,
                                                    int32_t cy, int32_t cz, int32_t t, bool check_g) {
    uint32_t rerr = 0, gerr = 0;
    const uint32_t e = !layer_ok ? (uint32_t)ERR_LAYER : (!range_ok ? (uint32_t)ERR_SLOT_RANGE : 0u);
    const int d = route_dest(sr.rc, cx, cy, cz, t, rerr);
    (void)route_dest(sr.rg, sr.rc.ix, sr.rc.iy, sr.rc.iz, sr.rc.u, gerr);
    return e | rerr | ((check_g && d >= 0) ? gerr : 0u);
}

// Slot, child slab and grandchild slab of a point of one slab (cell c, layer t):
// the per-arrival routine of the slab kernels.  Same quotients as slot_route,
// fewer instructions on the common path:
//  * grandchild indices relative to the cell, lg = floor(q_g) - 4c in [0, 4):
//    child octant bit lg >> 1 (= floor(q_g) >> 1 - 2c), grandchild bit lg & 1;
//    grandchild layer u_g = trunc(z / cr_g), child layer u_c = u_g / 2 (C
//    division truncates), so the grandchild select u_g - 2 u_c + 1 is always in
//    [0, 2] and a valid child route implies a valid grandchild route;
//  * the point's own layer trunc(z / cr) = u_g / 4: cr_g = cr / 4 exactly
//    (metadata.rs:92,96 divide by powers of two), RN(z / cr_g) = 4 RN(z / cr),
//    and trunc(trunc(a) / 4) = trunc(a / 4);
//  * the operand range of div_rc from the exponents (frexp) and one max: the
//    exact IEEE path also takes every non-finite coordinate.
// Lanes outside the range take the exact divisions of slot_route (one ballot).
struct SlabCtx {
    int32_t cx, cy, cz, t;
    int32_t uglo;    // lowest grandchild layer of the slab's points: u_g in [uglo, uglo + 6]
    uint32_t uspan;  // 3 (t != 0) or 6 (t == 0): u_g - uglo <= uspan <=> the point's layer is t
    uint32_t sel;    // per u_g - uglo, 4 bits: child select | grandchild select << 2
    __device__ __forceinline__ SlabCtx(int32_t cx_, int32_t cy_, int32_t cz_, int32_t t_) : cx(cx_), cy(cy_), cz(cz_), t(t_) {
        // trunc(z / cr) = t <=> u_g in [4t, 4t+3] (t > 0), [-3, 3] (t = 0), [4t-3, 4t] (t < 0)
        uglo = t_ > 0 ? 4 * t_ : 4 * t_ - 3;
        uspan = t_ == 0 ? 6u : 3u;
        sel = 0;
        for (uint32_t o = 0; o <= uspan; o++) {
            const int32_t ug = uglo + (int32_t)o, uc = ug / 2;
            sel |= (uint32_t)((uc - 2 * t_ + 1) | ((ug - 2 * uc + 1) << 2)) << (4 * o);
        }
    }
};
struct SlotDest {
    int32_t ox, oy;   // offset index (hex.rs:45-51)
    int32_t qa;       // axial q (hex.rs:18-24 to_axial of ox, oy)
    bool layer_ok;    // the point's z layer is the slab's
    int32_t d, g;     // child slab 0..23 / grandchild slab 0..23 inside it, -1: no valid route
};
// Without the exact path: `amb` flags the lanes slot_dest_exact must redo.
__device__ __forceinline__ SlotDest slot_dest_fast(float x, float y, float z, const LevelGeo& G, const SlabCtx& C,
                                                   bool& amb) {
    const int32_t ex = __builtin_amdgcn_frexp_expf(x), ey = __builtin_amdgcn_frexp_expf(y),
                  ez = __builtin_amdgcn_frexp_expf(z);
    // (non-short-circuit & and |: a && / || chain is emitted as branches, i.e.
    // exec-mask regions of scalar instructions, in the dense kernel's hot loop)
    amb = ((int)(G.exact != 0) | (int)!(fmaxf(fmaxf(fabsf(x), fabsf(y)), fabsf(z)) < 0x1p60f) |
           (int)(min(min(ex, ey), ez) < -58)) != 0;
    SlotDest S;
    {   // hex.rs:67-85
        const float xq = div_rc(x, G.crx, G.inv_crx);
        const float yq = div_rc(y, G.cry, G.inv_cry);
        const float tt = (kSqrt3 * yq) + 1.0f;
        const float t1 = floorf(tt + xq);
        const float t2 = tt - xq;
        const float t3 = (2.0f * xq) + 1.0f;
        S.qa = sat_i32(floorf(div_rc(t1 + t3, 3.0f, 0x1.555556p-2f)));
        S.oy = (int32_t)(0u - (uint32_t)sat_i32(floorf(div_rc(t1 + t2, 3.0f, 0x1.555556p-2f))));
        S.ox = S.qa + ((S.oy - (S.oy & 1)) >> 1);
    }
    const float qx = div_rc(x, G.csg, G.inv_csg), qy = div_rc(y, G.csg, G.inv_csg);
    const float qz = div_rc(z, G.csg, G.inv_csg), qu = div_rc(z, G.crg, G.inv_crg);
    amb |= fmaxf(fmaxf(fabsf(qx), fabsf(qy)), fmaxf(fabsf(qz), fabsf(qu))) >= 0x1p30f;
    const int32_t lgx = sat_i32(floorf(qx)) - 4 * C.cx, lgy = sat_i32(floorf(qy)) - 4 * C.cy,
                  lgz = sat_i32(floorf(qz)) - 4 * C.cz;
    const uint32_t off = (uint32_t)(sat_i32(truncf(qu)) - C.uglo);
    S.layer_ok = off <= C.uspan;
    const uint32_t sl = __builtin_amdgcn_ubfe(C.sel, (off & 7u) * 4u, 4u);
    const bool bad = (((lgx | lgy | lgz) & ~3) != 0) | !S.layer_ok;
    const uint32_t octc = (uint32_t)((lgx >> 1) | (lgy & 2) | ((lgz & 2) << 1));
    const uint32_t octg = (uint32_t)((lgx & 1) | ((lgy & 1) << 1) | ((lgz & 1) << 2));
    S.d = vsel(bad, -1, (int32_t)((octc << 1) + octc + (sl & 3u)));
    S.g = vsel(bad, -1, (int32_t)((octg << 1) + octg + (sl >> 2)));
    return S;
}
// The exact IEEE divisions of slot_route for one lane.
__device__ __forceinline__ void slot_dest_exact(float x, float y, float z, const LevelGeo& G, const SlabCtx& C,
                                                SlotDest& S) {
    const I3 hs = hex_from_world(x, y, z, G.cr);
    const RouteIdx rc = route_idx_exact(G.csc, G.crc, x, y, z);
    const RouteIdx rg = route_idx_exact(G.csg, G.crg, x, y, z);
    S.ox = hs.x;
    S.oy = hs.y;
    S.layer_ok = hs.z == C.t;
    S.qa = hs.x - (hs.y - (hs.y & 1)) / 2;
    S.d = route_dest_nc(rc, C.cx, C.cy, C.cz, C.t);
    S.g = S.d < 0 ? -1 : route_dest_nc(rg, rc.ix, rc.iy, rc.iz, rc.u);
}
__device__ __forceinline__ SlotDest slot_dest(float x, float y, float z, const LevelGeo& G, const SlabCtx& C) {
    bool amb;
    SlotDest S = slot_dest_fast(x, y, z, G, C, amb);
    if (__ballot(amb)) {
        if (amb) slot_dest_exact(x, y, z, G, C, S);
    }
    return S;
}
// hex.rs:55-65 centre of the slot (z layer t: the point's own layer when it belongs to the slab)
__device__ __forceinline__ void slot_centre(const SlotDest& S, float cr, float zt, float& X, float& Y, float& Z) {
    const float qf = (float)S.qa, rf = (float)S.oy;
    X = cr * ((kSqrt3 * qf) + ((kSqrt3 / 2.0f) * rf));
    Y = ((cr * 3.0f) / 2.0f) * rf;
    Z = zt;
}

// Buffer descriptor of a wave-uniform range.  Base and size are forced into
// SGPRs (readfirstlane): values loaded from global memory are otherwise kept
// in VGPRs and every buffer op becomes a readfirstlane "waterfall" loop.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd(const void* base, uint64_t bytes) {
    const uint64_t a = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint32_t nr = __builtin_amdgcn_readfirstlane((uint32_t)(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes));
    void* p = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)nr, 0x00020000);
}
__device__ __forceinline__ uint32_t bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0);
}

// ------------------------------------------------------------------ input kernels
__global__ void k_synth(Point* out, uint64_t first, uint64_t n, uint64_t seed, int kind, float lo, float ext) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        float x, y, z;
        uint32_t c;
        synth_point(seed, kind, j, lo, ext, x, y, z, c);
        float4 v = make_float4(x, y, z, __uint_as_float(c));
        reinterpret_cast<float4*>(out)[first + j] = v;
    }
}

// stream points idx0 .. idx0+n of a synthetic file into out[0 .. n)
__global__ void k_synth_at(Point* out, uint64_t idx0, uint64_t n, uint64_t seed, int kind, float lo, float ext) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
        float x, y, z;
        uint32_t c;
        synth_point(seed, kind, idx0 + j, lo, ext, x, y, z, c);
        reinterpret_cast<float4*>(out)[j] = make_float4(x, y, z, __uint_as_float(c));
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

// Reduces the per-block partials (min xyz, max xyz) into part[0..6); one block
// of 256 threads, strided over the partials.
__global__ __launch_bounds__(256) void k_bbox_final(float* part, uint32_t nb) {
    __shared__ float sb[4][6];
    float r[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (uint32_t b = threadIdx.x; b < nb; b += 256)
        for (int a = 0; a < 6; a++) r[a] = a < 3 ? fminf(r[a], part[b * 6 + a]) : fmaxf(r[a], part[b * 6 + a]);
    for (int d = 32; d > 0; d >>= 1)
        for (int a = 0; a < 6; a++) {
            const float o = __shfl_xor(r[a], d, 64);
            r[a] = a < 3 ? fminf(r[a], o) : fmaxf(r[a], o);
        }
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 6; a++) sb[threadIdx.x / 64][a] = r[a];
    __syncthreads();
    if (threadIdx.x < 6) {
        const int a = threadIdx.x;
        float v = sb[0][a];
        for (int q = 1; q < 4; q++) v = a < 3 ? fminf(v, sb[q][a]) : fmaxf(v, sb[q][a]);
        part[a] = v;
    }
}

// Non-finite coordinates (the reference's semantics: f32::min/max skip NaN,
// `as i32` saturates with NaN -> 0, a NaN distance never compares less):
// 1 = a NaN coordinate and no infinite one (such a point enters finite cells:
// index 0 on the NaN axes), 2 = an infinite coordinate (its cell index
// saturates on that axis at every level: cells of their own, built apart).
constexpr uint32_t kNfNan = 1u, kNfInf = 2u, kNfLayer = 4u;
__device__ __forceinline__ uint32_t nf_class(float x, float y, float z) {
    const bool inf = isinf(x) || isinf(y) || isinf(z);
    const bool nan = isnan(x) || isnan(y) || isnan(z);
    return inf ? kNfInf : (nan ? kNfNan : 0u);
}

// ------------------------------------------------------------------ level-0 binning
struct L0Params {
    float cs, cr, csc, crc;   // level 0 and level 1 cell size / hex radius
    float inv_cs, inv_cr;     // reciprocals for the fast floor/trunc quotients
    float inv_csc, inv_crc;
    int32_t exact;            // a divisor outside div_rc's range: IEEE divisions only
    int32_t lo[3];
    int32_t g[3];
    int32_t nl;
    int32_t dim2;   // 2 * sub_grid_dimension
    // sparse mode (bounding box spans > 2^20 level-0 cells): occupied cells in a
    // hash set keyed by the packed grid offset, compact cell id instead of the
    // dense linear index
    int32_t hashed;
    uint32_t hmask;
    const unsigned long long* hkeys;
    const uint32_t* hcid;
    const unsigned long long* ckeys;   // packed grid offset per compact cell id
};

constexpr unsigned long long kHashEmpty = ~0ull;
__device__ __forceinline__ unsigned long long l0_pack(int32_t gx, int32_t gy, int32_t gz) {
    return (unsigned long long)gx | ((unsigned long long)gy << 21) | ((unsigned long long)gz << 42);
}
__device__ __forceinline__ uint32_t l0_hash(unsigned long long k) {
    k ^= k >> 31;
    k *= 0x7fb5d329728ea185ull;
    k ^= k >> 27;
    k *= 0x81dadef4bc2dd44dull;
    k ^= k >> 33;
    return (uint32_t)k;
}

// Dense slab id of a point: ((cell - lo) linearised) * kL0Layers + (layer -
// (dim2*iz - 2)); ordered by (cell, layer) exactly like the compact slab ids.
// The layer part (< nl <= 194) is a function of z alone, so the radix pass on
// the low 6 bits needs no bounding box and runs fused with its reduction.
constexpr int kL0LayerBits = 8;
constexpr uint32_t kL0Layers = 1u << kL0LayerBits;
__device__ __forceinline__ int64_t l0_layer(const L0Params& P, float z, int32_t& iz) {
    iz = cell_index1(z, P.cs);
    const int32_t t = sat_i32(z / P.cr);   // hex.rs:83 z slot (truncation)
    return (int64_t)t - ((int64_t)P.dim2 * iz - 2);
}
// The same quotients from the correctly rounded reciprocals (div_rc: the IEEE
// quotient for operands 0 or in [2^-60, 2^60]); `amb` flags a lane whose
// operand is outside that range or a level whose divisors are, and the caller
// redoes such lanes with l0_layer / l0_dense / l0_dense_dest behind one ballot.
#ifndef PCC_L0_RC
#define PCC_L0_RC 1
#endif
__device__ __forceinline__ int64_t l0_layer_rc(const L0Params& P, float z, int32_t& iz, bool& amb) {
    amb |= P.exact || !rc_ok(z);
    iz = sat_i32(floorf(div_rc(z, P.cs, P.inv_cs)));
    const int32_t t = sat_i32(truncf(div_rc(z, P.cr, P.inv_cr)));
    return (int64_t)t - ((int64_t)P.dim2 * iz - 2);
}
// the layer digit of pass 0 / pass 1 (exact either way)
__device__ __forceinline__ int64_t l0_layer_any(const L0Params& P, float z, int32_t& iz) {
    if (!PCC_L0_RC) return l0_layer(P, z, iz);
    bool amb = false;
    int64_t ll = l0_layer_rc(P, z, iz, amb);
    if (__ballot(amb)) {
        if (amb) ll = l0_layer(P, z, iz);
    }
    return ll;
}
// HASHED: -1 = decided by P.hashed at run time, 0 / 1 = known at compile time
// (the pipelined downsweep must not carry the hash probe loop: its waits would
// drain the prefetched tile)
template <int HASHED = -1>
__device__ __forceinline__ int64_t l0_dense(const L0Params& P, float x, float y, float z) {
    int32_t iz, ix, iy;
    int64_t ll;
    if (HASHED == 0 && PCC_L0_RC) {   // reciprocal quotients, exact lanes redone below
        bool amb = !rc_ok(x) || !rc_ok(y);
        ll = l0_layer_rc(P, z, iz, amb);
        ix = sat_i32(floorf(div_rc(x, P.cs, P.inv_cs)));
        iy = sat_i32(floorf(div_rc(y, P.cs, P.inv_cs)));
        if (__ballot(amb)) {
            if (amb) {
                ll = l0_layer(P, z, iz);
                ix = cell_index1(x, P.cs);
                iy = cell_index1(y, P.cs);
            }
        }
    } else {
        ll = l0_layer(P, z, iz);
        ix = cell_index1(x, P.cs);
        iy = cell_index1(y, P.cs);
    }
    int32_t gx = ix - P.lo[0], gy = iy - P.lo[1], gz = iz - P.lo[2];
    if (gx < 0 || gy < 0 || gz < 0 || gx >= P.g[0] || gy >= P.g[1] || gz >= P.g[2] || ll < 0 || ll >= P.nl) return -1;
    if (HASHED == 1 || (HASHED == -1 && P.hashed)) {
        const unsigned long long key = l0_pack(gx, gy, gz);
        uint32_t h = l0_hash(key) & P.hmask;
        for (uint32_t probe = 0; probe <= P.hmask; probe++) {
            const unsigned long long k = P.hkeys[h];
            if (k == key) return (int64_t)P.hcid[h] * kL0Layers + ll;
            if (k == kHashEmpty) return -1;
            h = (h + 1) & P.hmask;
        }
        return -1;
    }
    return (((int64_t)gz * P.g[1] + gy) * P.g[0] + gx) * kL0Layers + ll;
}

// sparse mode: insert every point's level-0 cell into the hash set (a plain read
// first, so repeated cells cost no atomic); counts distinct cells
__global__ __launch_bounds__(256) void k_l0_hash_insert(const Point* __restrict__ in, uint64_t n, L0Params P,
                                                        unsigned long long* hkeys, uint32_t* count, uint32_t* bad) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const float4 v = reinterpret_cast<const float4*>(in)[i];
        const int32_t gx = cell_index1(v.x, P.cs) - P.lo[0], gy = cell_index1(v.y, P.cs) - P.lo[1];
        const int32_t gz = cell_index1(v.z, P.cs) - P.lo[2];
        if (gx < 0 || gy < 0 || gz < 0 || gx >= P.g[0] || gy >= P.g[1] || gz >= P.g[2]) { atomicOr(bad, 1u); continue; }
        const unsigned long long key = l0_pack(gx, gy, gz);
        uint32_t h = l0_hash(key) & P.hmask;
        uint32_t probe = 0;
        for (; probe <= P.hmask; probe++) {
            unsigned long long k = hkeys[h];
            if (k == kHashEmpty) {
                k = atomicCAS(&hkeys[h], kHashEmpty, key);
                if (k == kHashEmpty) { atomicAdd(count, 1u); break; }
            }
            if (k == key) break;
            h = (h + 1) & P.hmask;
        }
        if (probe > P.hmask) atomicOr(bad, 2u);   // table full: the host grows it and retries
    }
}

// compact ids of the occupied hash entries
__global__ void k_l0_hash_flags(const unsigned long long* hkeys, uint32_t cap, uint32_t* flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap) flag[i] = hkeys[i] != kHashEmpty ? 1u : 0u;
}
__global__ void k_l0_hash_ids(const unsigned long long* hkeys, uint32_t cap, uint32_t* hcid,
                              unsigned long long* ckeys) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap && hkeys[i] != kHashEmpty) ckeys[hcid[i]] = hkeys[i];
}

#ifndef PCC_L0_PF
#define PCC_L0_PF 1   // level-0 downsweeps: register tiles in flight ahead (1 or 2)
#endif
#ifndef PCC_L0BS
#define PCC_L0BS 1024
#define PCC_L0IPT 3
#endif
constexpr int kL0BS = PCC_L0BS, kL0IPT = PCC_L0IPT, kL0Tile = kL0BS * kL0IPT, kL0W = kL0BS / 64;
constexpr int kHistLds = 16384;   // dense level-0 slabs counted in LDS (64 KB): 64 cells x 256 layers
constexpr uint32_t kL0DownGrid = 512;   // persistent blocks of the fused upsweep (2 per CU)

// Pass 0 over the tile groups of k_l0_down6g, fused with the bounding box
// (converter.rs:96-104, bounding-volume/src/lib.rs:38-52): per group the
// histogram of the low 6 layer bits (a function of z alone, no bbox needed) and
// the group's min/max partials (finished by k_bbox_final).  Nothing per tile, so
// the loop is a plain stream with 4 loads in flight per thread.
__global__ __launch_bounds__(kL0BS) void k_l0_up0g(const Point* __restrict__ in, uint64_t n, L0Params P, uint32_t tpg,
                                                   uint32_t ngroups, uint32_t* __restrict__ gcnt0, float* part,
                                                   uint32_t* flag) {
    constexpr int R = 1 << 6, U = 4, NWV = kL0BS / 64;
    __shared__ uint32_t dh[NWV][R];   // per wave: one LDS add per point, no ranks
    __shared__ float sb[kL0BS / 64][6];
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (uint32_t i = threadIdx.x; i < NWV * R; i += kL0BS) (&dh[0][0])[i] = 0;
    __syncthreads();
    const uint32_t wv = threadIdx.x / 64;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nf = 0;
    const uint64_t lo = (uint64_t)blockIdx.x * tpg * kL0Tile;
    const uint64_t hi = min((uint64_t)(blockIdx.x + 1) * tpg * kL0Tile, n);
    for (uint64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (uint64_t)U * kL0BS) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = p4[min(i0 + (uint64_t)u * kL0BS, hi - 1)];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool valid = i0 + (uint64_t)u * kL0BS < hi;
            uint32_t d6 = 0;
            if (valid) {
                nf |= nf_class(v[u].x, v[u].y, v[u].z);
                mn[0] = fminf(mn[0], v[u].x); mn[1] = fminf(mn[1], v[u].y); mn[2] = fminf(mn[2], v[u].z);
                mx[0] = fmaxf(mx[0], v[u].x); mx[1] = fmaxf(mx[1], v[u].y); mx[2] = fmaxf(mx[2], v[u].z);
                int32_t iz;
                d6 = (uint32_t)l0_layer_any(P, v[u].z, iz) & (R - 1);
            }
            if (valid) atomicAdd(&dh[wv][d6], 1u);
        }
    }
    for (int d = 32; d > 0; d >>= 1)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
        }
    const int w = threadIdx.x / 64;
    if (nf) atomicOr(flag, nf);
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; a++) { sb[w][a] = mn[a]; sb[w][3 + a] = mx[a]; }
    __syncthreads();
    if (threadIdx.x < 6) {
        float r = sb[0][threadIdx.x];
        for (int q = 1; q < kL0BS / 64; q++) r = threadIdx.x < 3 ? fminf(r, sb[q][threadIdx.x]) : fmaxf(r, sb[q][threadIdx.x]);
        part[blockIdx.x * 6 + threadIdx.x] = r;
    }
    if (threadIdx.x < (uint32_t)R) {
        uint32_t c = 0;
        for (int q = 0; q < NWV; q++) c += dh[q][threadIdx.x];
        gcnt0[(uint64_t)threadIdx.x * ngroups + blockIdx.x] = c;
    }
}

// Pass 0 while a host input uploads (Engine::pre0_count): per tile of kL0Tile
// points the histogram of the low 6 layer bits (the digit k_l0_up0g counts per
// group), per block the bounding box of its tiles behind the running box in
// part[0..5] (k_bbox_final folds them).  Grid-stride over tiles [t0, t1); the
// build sums the tiles of each group (k_l0_group_from_tiles) instead of reading
// the points again.
__global__ __launch_bounds__(kL0BS) void k_l0_tiles0(const Point* __restrict__ in, uint64_t n, L0Params P, uint64_t t0,
                                                     uint64_t t1, uint16_t* __restrict__ tile6, float* part,
                                                     uint32_t* flag) {
    constexpr int R = 1 << 6, NWV = kL0BS / 64;
    __shared__ uint32_t dh[NWV][R];
    __shared__ float sb[NWV][6];
    const float4* p4 = reinterpret_cast<const float4*>(in);
    const uint32_t tid = threadIdx.x, wv = tid / 64;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nf = 0;
    for (uint64_t t = t0 + blockIdx.x; t < t1; t += gridDim.x) {
        for (uint32_t i = tid; i < NWV * R; i += kL0BS) (&dh[0][0])[i] = 0;
        __syncthreads();
        const uint64_t base = t * kL0Tile;
        float4 v[kL0IPT];
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) v[r] = p4[min(base + (uint64_t)r * kL0BS + tid, n - 1)];
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            if (base + (uint64_t)r * kL0BS + tid >= n) continue;
            nf |= nf_class(v[r].x, v[r].y, v[r].z);
            mn[0] = fminf(mn[0], v[r].x); mn[1] = fminf(mn[1], v[r].y); mn[2] = fminf(mn[2], v[r].z);
            mx[0] = fmaxf(mx[0], v[r].x); mx[1] = fmaxf(mx[1], v[r].y); mx[2] = fmaxf(mx[2], v[r].z);
            int32_t iz;
            atomicAdd(&dh[wv][(uint32_t)l0_layer_any(P, v[r].z, iz) & (R - 1)], 1u);
        }
        __syncthreads();
        if (tid < (uint32_t)R) {
            uint32_t c = 0;
            for (int q = 0; q < NWV; q++) c += dh[q][tid];
            tile6[t * R + tid] = (uint16_t)c;
        }
        __syncthreads();
    }
    for (int d = 32; d > 0; d >>= 1)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
        }
    if (nf) atomicOr(flag, nf);
    if ((tid & 63) == 0)
        for (int a = 0; a < 3; a++) { sb[wv][a] = mn[a]; sb[wv][3 + a] = mx[a]; }
    __syncthreads();
    if (tid < 6) {
        float r = sb[0][tid];
        for (int q = 1; q < NWV; q++) r = tid < 3 ? fminf(r, sb[q][tid]) : fmaxf(r, sb[q][tid]);
        part[(1 + blockIdx.x) * 6 + tid] = r;
    }
}

// per (group, digit): the sum of its tiles' counts, as k_l0_up0g's gcnt0
__global__ void k_l0_group_from_tiles(const uint16_t* __restrict__ tile6, uint64_t ntiles, uint32_t tpg,
                                      uint32_t ngroups, uint32_t* __restrict__ gcnt0) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;   // g * 64 + digit
    if (i >= ngroups * 64u) return;
    const uint32_t g = i / 64, d = i % 64;
    const uint64_t a = (uint64_t)g * tpg, b = min(a + tpg, ntiles);
    uint32_t c = 0;
    for (uint64_t t = a; t < b; t++) c += tile6[t * 64 + d];
    gcnt0[(uint64_t)d * ngroups + g] = c;
}

// Pass-1 upsweep from the arena: per-tile digit histogram + the full dense-slab
// histogram (LDS-privatised when it fits), grid-stride over the tiles.
// Global histogram increment with one atomic per distinct bin of the active
// lanes when they all hit the same bin (a run of one slab: clustered or
// partially sorted input), else one per lane.
__device__ __forceinline__ void wave_aggregated_add(uint32_t* hist, uint32_t d) {
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
    const unsigned long long same = __ballot(d == d0), act = __ballot(1);
    if (same == act) {
        if (__lane_id() == (uint32_t)__ffsll((long long)act) - 1) atomicAdd(&hist[d0], (uint32_t)__popcll(act));
    } else {
        atomicAdd(&hist[d], 1u);
    }
}

template <int BITS>
__global__ __launch_bounds__(kL0BS) void k_l0_up_hist(Arena A, uint64_t n, L0Params P, int shift,
                                                      uint32_t* __restrict__ counts, uint32_t ntiles, uint32_t* hist,
                                                      uint32_t D, Counters* ctr) {
    constexpr int R = 1 << BITS;
    __shared__ uint32_t dh[R];
    __shared__ uint32_t h[kHistLds];
    const bool lds = D <= (uint32_t)kHistLds;
    if (lds) for (uint32_t i = threadIdx.x; i < D; i += kL0BS) h[i] = 0;
    uint32_t err = 0;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = threadIdx.x; i < R; i += kL0BS) dh[i] = 0;
        __syncthreads();
        const uint64_t base = (uint64_t)tile * kL0Tile;
        float4 v[kL0IPT];
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
            if (i < n) v[r] = A.p[i];
        }
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
            if (i < n) {
                const int64_t d = l0_dense(P, v[r].x, v[r].y, v[r].z);
                if (d < 0) { err = ERR_L0_RANGE; continue; }
                atomicAdd(&dh[((uint64_t)d >> shift) & (R - 1)], 1u);
                if (lds) atomicAdd(&h[d], 1u);
                else wave_aggregated_add(hist, (uint32_t)d);   // clustered input: few hot slabs
            }
        }
        __syncthreads();
        for (int d = threadIdx.x; d < R; d += kL0BS) counts[(uint64_t)d * ntiles + tile] = dh[d];
    }
    if (err) set_err(ctr, err);
    __syncthreads();
    if (lds)
        for (uint32_t i = threadIdx.x; i < D; i += kL0BS)
            if (h[i]) atomicAdd(&hist[i], h[i]);
}

// Pass-1 upsweep fused with the level-0 capacities (replaces k_dcap when the
// level-1 grid is small): per point the LEVEL-1 slab (cell index at h = 1,
// metadata.rs:100-102, and hex layer hex.rs:83) is counted in an LDS histogram.
// Its level-0 slab follows exactly (cell_size and the hex radius halve exactly,
// metadata.rs:92,96, so x / cs0 = RN(x / cs1) / 2: ix0 = ix1 >> 1, t0 = u1 / 2),
// so the per-tile digit counts come from the same 4 divisions, and every
// level-0 slab's 24 capacities are level-1 histogram bins (k_l0_dcap_from1).
constexpr int kHist1Lds = 16384;   // level-1 dense slabs held in LDS (64 KB)
struct L1Grid { int32_t lo[3], g[3]; };
__device__ __forceinline__ int64_t l1_dense(const L0Params& P, const L1Grid& Q, float x, float y, float z, int64_t& d0) {
    // IEEE divisions (exact reciprocal quotients measured slower here: 5.1 vs 4.2 ms)
    const int32_t ix1 = cell_index1(x, P.csc), iy1 = cell_index1(y, P.csc), iz1 = cell_index1(z, P.csc);
    const int32_t u1 = sat_i32(z / P.crc);
    const int32_t gx1 = ix1 - Q.lo[0], gy1 = iy1 - Q.lo[1], gz1 = iz1 - Q.lo[2];
    const int64_t ll1 = (int64_t)u1 - ((int64_t)P.dim2 * iz1 - 2);
    // level 0 from level 1: floor halves (arithmetic shift), the layer truncates (u1 / 2)
    const int32_t gx0 = (ix1 >> 1) - P.lo[0], gy0 = (iy1 >> 1) - P.lo[1], iz0 = iz1 >> 1, gz0 = iz0 - P.lo[2];
    const int64_t ll0 = (int64_t)(u1 / 2) - ((int64_t)P.dim2 * iz0 - 2);
    const bool ok1 = gx1 >= 0 && gy1 >= 0 && gz1 >= 0 && gx1 < Q.g[0] && gy1 < Q.g[1] && gz1 < Q.g[2] && ll1 >= 0 &&
                     ll1 < (int64_t)kL0Layers;
    const bool ok0 = gx0 >= 0 && gy0 >= 0 && gz0 >= 0 && gx0 < P.g[0] && gy0 < P.g[1] && gz0 < P.g[2] && ll0 >= 0 &&
                     ll0 < P.nl;
    d0 = ok0 ? (((int64_t)gz0 * P.g[1] + gy0) * P.g[0] + gx0) * kL0Layers + ll0 : -1;
    return ok1 ? (((int64_t)gz1 * Q.g[1] + gy1) * Q.g[0] + gx1) * kL0Layers + ll1 : -1;
}

template <int BITS>
__global__ __launch_bounds__(kL0BS) void k_l0_up_hist1(Arena A, uint64_t n, L0Params P, L1Grid Q, int shift,
                                                       uint32_t* __restrict__ counts, uint32_t ntiles,
                                                       uint32_t* hist1, uint32_t D1, Counters* ctr) {
    constexpr int R = 1 << BITS;
    __shared__ uint32_t dh[R];
    __shared__ uint32_t h[kHist1Lds];
    for (uint32_t i = threadIdx.x; i < D1; i += kL0BS) h[i] = 0;
    uint32_t err = 0;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = threadIdx.x; i < R; i += kL0BS) dh[i] = 0;
        __syncthreads();
        const uint64_t base = (uint64_t)tile * kL0Tile;
        float4 v[kL0IPT];
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
            if (i < n) v[r] = A.p[i];
        }
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
            if (i < n) {
                int64_t d0;
                const int64_t d1 = l1_dense(P, Q, v[r].x, v[r].y, v[r].z, d0);
                if (d1 < 0 || d0 < 0) { err = ERR_L0_RANGE; continue; }
                atomicAdd(&dh[((uint64_t)d0 >> shift) & (R - 1)], 1u);
                atomicAdd(&h[d1], 1u);
            }
        }
        __syncthreads();
        for (int d = threadIdx.x; d < R; d += kL0BS) counts[(uint64_t)d * ntiles + tile] = dh[d];
    }
    if (err) set_err(ctr, err);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < D1; i += kL0BS)
        if (h[i]) atomicAdd(&hist1[i], h[i]);
}

// level-0 dense histogram from the level-1 one (each level-1 slab has exactly one parent slab)
__global__ void k_l0_hist_from1(const uint32_t* __restrict__ hist1, uint32_t D1, L0Params P, L1Grid Q,
                                uint32_t* __restrict__ hist) {
    const uint32_t d1 = blockIdx.x * blockDim.x + threadIdx.x;
    if (d1 >= D1 || !hist1[d1]) return;
    const uint32_t c1 = d1 / kL0Layers, ll1 = d1 % kL0Layers;
    const int32_t gx1 = (int32_t)(c1 % (uint32_t)Q.g[0]), gy1 = (int32_t)((c1 / (uint32_t)Q.g[0]) % (uint32_t)Q.g[1]);
    const int32_t gz1 = (int32_t)(c1 / ((uint32_t)Q.g[0] * (uint32_t)Q.g[1]));
    const int32_t iz1 = Q.lo[2] + gz1, iz0 = iz1 >> 1;
    const int32_t u1 = (int32_t)ll1 + (P.dim2 * iz1 - 2);
    const int32_t ll0 = u1 / 2 - (P.dim2 * iz0 - 2);
    const uint64_t d0 = (((uint64_t)(iz0 - P.lo[2]) * P.g[1] + (uint32_t)(((Q.lo[1] + gy1) >> 1) - P.lo[1])) * P.g[0] +
                         (uint32_t)(((Q.lo[0] + gx1) >> 1) - P.lo[0])) * kL0Layers + (uint32_t)ll0;
    atomicAdd(&hist[d0], hist1[d1]);
}

// capacities of the level-0 slabs: arrivals per child slab (octant, layer select)
// = the level-1 histogram bin of that child slab
__global__ void k_l0_dcap_from1(const uint32_t* __restrict__ hist1, L0Params P, L1Grid Q, const int32_t* cell_idx,
                                const uint32_t* slab_cell, const int32_t* slab_layer, uint32_t nslabs, uint32_t* dcap) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= (uint64_t)nslabs * kDests) return;
    const uint32_t s = (uint32_t)(i / kDests), dest = (uint32_t)(i % kDests), o = dest / 3, sel = dest % 3;
    const uint32_t c = slab_cell[s];
    const int32_t t = slab_layer[s];
    const int32_t cx = 2 * cell_idx[3 * c] + (int32_t)(o & 1), cy = 2 * cell_idx[3 * c + 1] + (int32_t)((o >> 1) & 1);
    const int32_t cz = 2 * cell_idx[3 * c + 2] + (int32_t)((o >> 2) & 1);
    const int32_t u = 2 * t - 1 + (int32_t)sel;
    const int64_t ll1 = (int64_t)u - ((int64_t)P.dim2 * cz - 2);
    uint32_t v = 0;
    // a child layer has ONE parent layer, u / 2 (C division): sel 0 exists only for
    // t <= 0 and sel 2 only for t >= 0, so (t, 2) and (t + 1, 0) never both count u
    if (u / 2 == t && ll1 >= 0 && ll1 < (int64_t)kL0Layers) {
        const uint64_t d1 = (((uint64_t)(cz - Q.lo[2]) * Q.g[1] + (uint32_t)(cy - Q.lo[1])) * Q.g[0] + (uint32_t)(cx - Q.lo[0])) *
                                kL0Layers + (uint64_t)ll1;
        v = hist1[d1];
    }
    dcap[i] = v;
}

// later-pass upsweep from a SoA arena
template <int BITS>
__global__ __launch_bounds__(kL0BS) void k_l0_up(Arena A, uint64_t n, L0Params P, int shift,
                                                 uint32_t* __restrict__ counts, uint32_t ntiles) {
    constexpr int R = 1 << BITS;
    __shared__ uint32_t dh[R];
    for (int i = threadIdx.x; i < R; i += kL0BS) dh[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kL0Tile;
#pragma unroll 4
    for (int r = 0; r < kL0IPT; r++) {
        const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
        if (i < n) {
            const float4 v = A.p[i];
            const int64_t d = l0_dense(P, v.x, v.y, v.z);
            atomicAdd(&dh[((uint64_t)(d < 0 ? 0 : d) >> shift) & (R - 1)], 1u);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < R; d += kL0BS) counts[(uint64_t)d * ntiles + blockIdx.x] = dh[d];
}

// Stable downsweep carrying the payload (x, y, z, rgba, input index); the key is
// recomputed from the position.  SRC_AOS: read the 16-B input records (index =
// position); FINAL: also write the event batch of every point.
template <int BITS, bool SRC_AOS, bool FINAL>
__global__ __launch_bounds__(kL0BS) void k_l0_down(const Point* __restrict__ in, const uint32_t* __restrict__ keys,
                                                   Arena S, Arena O, uint64_t n,
                                                   L0Params P, int shift, const uint32_t* __restrict__ offs,
                                                   uint32_t ntiles, const uint32_t* files, uint32_t nfiles) {
    constexpr int R = 1 << BITS;
    __shared__ float4 sp[kL0Tile];
    __shared__ uint32_t sk[kL0Tile];
    __shared__ uint16_t sd[kL0Tile];
    // per (row r, wave) digit counts of the whole tile, then ONE prefix pass in
    // key order (r-major, wave, lane): two barriers per tile
    __shared__ uint16_t wcnt[kL0IPT][kL0W][R], wpre[kL0IPT][kL0W][R];
    __shared__ uint32_t tot[R], dbase[R], goff[R];
    __shared__ uint32_t lds[kL0W + 1];
    const uint32_t w = threadIdx.x / 64;
    for (int i = threadIdx.x; i < R; i += kL0BS) goff[i] = offs[(uint64_t)i * ntiles + blockIdx.x];
    for (int i = threadIdx.x; i < kL0IPT * kL0W * R; i += kL0BS) (&wcnt[0][0][0])[i] = 0;
    const uint64_t base = (uint64_t)blockIdx.x * kL0Tile;
    float4 v[kL0IPT];
    uint32_t k[kL0IPT], rw[kL0IPT];
    uint16_t dg[kL0IPT];
#pragma unroll
    for (int r = 0; r < kL0IPT; r++) {
        const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
        dg[r] = 0;
        k[r] = 0;
        v[r] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < n) {
            if constexpr (SRC_AOS) {
                v[r] = reinterpret_cast<const float4*>(in)[i];
                k[r] = keys ? keys[i] : (uint32_t)i;   // sharded input carries global keys
            } else {
                v[r] = S.p[i];
                k[r] = S.k[i];
            }
            const int64_t d = l0_dense(P, v[r].x, v[r].y, v[r].z);
            dg[r] = (uint16_t)(((uint64_t)(d < 0 ? 0 : d) >> shift) & (R - 1));
        }
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int r = 0; r < kL0IPT; r++) {
        const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
        const bool valid = i < n;
        const uint32_t d = dg[r];
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; b++) {
            const uint64_t bb = __ballot(valid && ((d >> b) & 1));
            same &= ((d >> b) & 1) ? bb : ~bb;
        }
        rw[r] = __popcll(same & lt);
        if (valid && rw[r] == 0) wcnt[r][w][d] = (uint16_t)__popcll(same);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < R; t += kL0BS) {
        uint32_t acc = 0;
#pragma unroll
        for (int r = 0; r < kL0IPT; r++)
#pragma unroll
            for (int q = 0; q < kL0W; q++) { const uint32_t cc = wcnt[r][q][t]; wpre[r][q][t] = (uint16_t)acc; acc += cc; }
        tot[t] = acc;
    }
    __syncthreads();
    {
        uint32_t tt;
        const uint32_t cc = threadIdx.x < (uint32_t)R ? tot[threadIdx.x] : 0;
        const uint32_t e = block_excl_scan<kL0BS>(cc, lds, &tt);
        if (threadIdx.x < (uint32_t)R) dbase[threadIdx.x] = e;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kL0IPT; r++) {
        const uint64_t i = base + (uint64_t)r * kL0BS + threadIdx.x;
        if (i < n) {
            const uint32_t p = dbase[dg[r]] + wpre[r][w][dg[r]] + rw[r];
            sp[p] = v[r]; sk[p] = k[r]; sd[p] = dg[r];
        }
    }
    __syncthreads();
    const uint32_t tn = (uint32_t)((n - base) < (uint64_t)kL0Tile ? (n - base) : (uint64_t)kL0Tile);
    for (uint32_t j = threadIdx.x; j < tn; j += kL0BS) {
        const uint32_t d = sd[j];
        const uint32_t dst = goff[d] + (j - dbase[d]);
        O.p[dst] = sp[j];
        O.k[dst] = sk[j];
    }
}

// ---- level-0 binning with one upsweep (at most 8 level-0 cells: the dense-id
// bits above the 6 low layer bits fit one 5-bit pass).  Pass 1 (k_l0_down6g)
// runs kL0Groups persistent blocks, block g over a contiguous group of tiles,
// and counts every point's (low 6 bits d6, high bits d5) pair in LDS.  Its
// output is ordered by (d6, tile), so the points of group g with low bits d6
// are one contiguous segment, and those counts give pass 2 the exact output
// offset of every (segment, d5) run: no second upsweep.  Pass 2 (k_l0_down5g)
// walks units of consecutive segments of one d6 bucket with running offsets and
// counts the level-0 capacities (arrivals per child slab) on the way, which
// replaces the level-1 histogram pass.
constexpr uint32_t kL0Groups = 2048;
constexpr uint32_t kL0Groups6 = 256;   // the modulo-4 fold (k_l0_tile6 CB = 6: 64 KB pair table per group)
struct L0Unit { uint32_t d6, g0, g1, pad; };

// Per-tile wave counts, digit-major: cnt[d][r * kL0W + q] = lanes of wave q in
// row r with digit d (<= 64), pre[d][..] = their exclusive prefix in key order.
constexpr int kL0RW = kL0IPT * kL0W;   // 48 (row, wave) pairs per tile
static_assert(kL0RW % 16 == 0, "16-byte rows");
// Row strides of the count (bytes) and prefix (u16) rows: PCC_L0_PAD skews the
// rows across LDS banks for wave 0's row reads / writes (56 B = 14 words, 112 B =
// 28 words against 48 B = 12 and 96 B = 24: half the lanes per bank)
#ifndef PCC_L0_PAD
#define PCC_L0_PAD 0
#endif
constexpr int kL0RC = kL0RW + (PCC_L0_PAD ? 8 : 0), kL0RP = kL0RW + (PCC_L0_PAD ? 8 : 0);
static_assert(kL0RC % 8 == 0 && (kL0RP * 2) % 16 == 0, "8-byte count rows, 16-byte prefix rows");
// Wave 0 of a tile: lane t < R reads digit t's 48 counts as 16-byte words,
// writes their prefixes and clears them for the next tile, then the tile's digit
// bases by a wave scan; returns the digit's total.
template <int R>
__device__ __forceinline__ uint32_t l0_tile_prefix(uint8_t (*cnt)[kL0RC], uint16_t (*pre)[kL0RP], uint32_t lane,
                                                   uint32_t& excl) {
    uint32_t acc = 0;
    if (lane < (uint32_t)R) {
        uint2* c2 = reinterpret_cast<uint2*>(cnt[lane]);
        uint4* p4 = reinterpret_cast<uint4*>(pre[lane]);
#pragma unroll 1
        for (int c = 0; c < kL0RW / 8; c++) {   // 8 counts per step: one 8-byte read, one 16-byte write
            const uint2 wv = c2[c];
            c2[c] = make_uint2(0u, 0u);
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const uint32_t wd = k ? wv.y : wv.x;
                const uint32_t b0 = wd & 0xFFu, b1 = (wd >> 8) & 0xFFu, b2 = (wd >> 16) & 0xFFu, b3 = wd >> 24;
                o[2 * k] = acc | ((acc + b0) << 16);
                acc += b0 + b1;
                o[2 * k + 1] = acc | ((acc + b2) << 16);
                acc += b2 + b3;
            }
            p4[c] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
    uint32_t x = acc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    excl = x - acc;
    return acc;
}

// l0_tile_prefix for R > 64 digits: lane t handles the R / 64 consecutive digits
// t * R / 64 + k, their totals and exclusive bases in tot[k], excl[k].
template <int R>
__device__ __forceinline__ void l0_tile_prefix_n(uint8_t (*cnt)[kL0RC], uint16_t (*pre)[kL0RP], uint32_t lane,
                                                 uint32_t* tot, uint32_t* excl) {
    constexpr int DPL = R / 64;
    static_assert(R % 64 == 0 && DPL >= 1, "whole digits per lane");
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
        const uint32_t d = lane * DPL + k;
        uint2* c2 = reinterpret_cast<uint2*>(cnt[d]);
        uint4* p4 = reinterpret_cast<uint4*>(pre[d]);
        uint32_t acc = 0;
#pragma unroll 2
        for (int c = 0; c < kL0RW / 8; c++) {
            const uint2 wv = c2[c];
            c2[c] = make_uint2(0u, 0u);
            uint32_t o[4];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t wd = h ? wv.y : wv.x;
                const uint32_t b0 = wd & 0xFFu, b1 = (wd >> 8) & 0xFFu, b2 = (wd >> 16) & 0xFFu, b3 = wd >> 24;
                o[2 * h] = acc | ((acc + b0) << 16);
                acc += b0 + b1;
                o[2 * h + 1] = acc | ((acc + b2) << 16);
                acc += b2 + b3;
            }
            p4[c] = make_uint4(o[0], o[1], o[2], o[3]);
        }
        tot[k] = acc;
        excl[k] = sum;   // (lane-local so far)
        sum += acc;
    }
    uint32_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
#pragma unroll
    for (int k = 0; k < DPL; k++) excl[k] += x - sum;
}

// Stores shaped like one tile's output stores (kL0IPT x (16 B + 4 B)) into a
// scratch area: issued once before a tile loop so the loop is entered with the
// pending memory ops of its back-edge (the compiler's waits at the loop header
// then never cover the previous tile's stores).
__device__ __forceinline__ void l0_dummy_stores(const Arena& dummy, const float4* v) {
    const uint32_t slot = (blockIdx.x % 256) * kL0BS + threadIdx.x;
#pragma unroll
    for (int r = 0; r < kL0IPT; r++) {
        dummy.p[slot * kL0IPT + r] = v[r];
        dummy.k[slot * kL0IPT + r] = 0u;
    }
}

// Pass 1.  Per tile: stable LDS partition on the low 6 layer bits, the (d6, d5)
// pair counted per group; the next tile's loads are issued before this tile's
// stores and only LDS barriers are used, so no wait ever covers a store.
// KEYS: global keys from `keys` (sharded input), staged in LDS beside the
// points (then R5 <= 16 keeps the LDS under half a CU); else key = index.
template <int R5, bool KEYS>
__global__ __launch_bounds__(kL0BS, 8) void k_l0_down6g(const Point* __restrict__ in, const uint32_t* __restrict__ keys,
                                                        Arena O, uint64_t n, L0Params P,
                                                        const uint32_t* __restrict__ offs, uint32_t ntiles, uint32_t tpg,
                                                        uint32_t ngroups, uint32_t* __restrict__ gcnt, int pairs,
                                                        Arena dummy, Counters* ctr) {
    constexpr int R = 64;
    using KT = typename std::conditional<KEYS, uint32_t, uint16_t>::type;
    __shared__ float4 sp[kL0Tile];
    __shared__ KT sk[kL0Tile];
    __shared__ uint8_t sd[kL0Tile];
    __shared__ alignas(16) uint8_t wcnt[R][kL0RC];
    __shared__ alignas(16) uint16_t wpre[R][kL0RP];
    __shared__ uint32_t dbase[R], gofs[R];
    // pair counts, row d6 padded to R5 + 1 words: the lanes of a wave share few
    // d5 values, and with rows of exactly R5 words they all hit bank d5
    constexpr int HP = PCC_L0_SWZ ? R5 + 1 : R5;
    __shared__ uint32_t h[R * HP];
    const uint32_t tid = threadIdx.x, w = tid / 64, lane = tid & 63, g = blockIdx.x;
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (int i = tid; i < R * HP; i += kL0BS) h[i] = 0;
    for (int i = tid; i < kL0RC * R / 4; i += kL0BS) reinterpret_cast<uint32_t*>(&wcnt[0][0])[i] = 0;
    const uint64_t lt = lanemask_lt();
    uint32_t err = 0;
    const uint32_t t0 = g * tpg, t1 = min(t0 + tpg, ntiles);
    // wave 0, lane d: output position of digit d for the current tile (the
    // group's tiles are consecutive: the scanned pass-0 group count, then + each
    // tile's total)
    uint32_t goffr = w == 0 ? offs[(uint64_t)lane * ngroups + g] : 0u;
    gofs[lane] = goffr;   // (an LDS write: the load is complete before the loop)
    // every load and store below is issued unconditionally (indices clamped to
    // the tile), so the number of memory ops per tile is static and the waits
    // for the prefetched tiles never cover this tile's stores
    auto load_tile = [&](float4* v, uint32_t* kk, uint32_t tile) {
        const uint64_t base = (uint64_t)tile * kL0Tile;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = min(base + (uint64_t)r * kL0BS + tid, n - 1);
            v[r] = p4[i];
            if constexpr (KEYS) kk[r] = keys[i];
        }
        asm volatile("" ::: "memory");   // keep the loads ahead of the tile's stores
    };
    // one tile from registers v: digits and wave ranks, the tile's digit
    // prefix, the LDS partition; then v is refilled with tile `pf` (PCC_L0_PF
    // tiles ahead) before the partitioned tile is stored
    auto body = [&](uint32_t tile, float4* v, uint32_t* kk, uint32_t pf) {
        const uint64_t base = (uint64_t)tile * kL0Tile;
        lds_barrier();   // the last tile's stores have read the staging arrays
        uint32_t dgp = 0, rwp = 0;
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + tid;
            const bool valid = i < n;
            uint32_t d6 = 0;
            if (valid && pairs) {
                int64_t d = l0_dense<0>(P, v[r].x, v[r].y, v[r].z);
                if (d < 0) { err = ERR_L0_RANGE; d = 0; }
                d6 = (uint32_t)d & (R - 1);
                atomicAdd(&h[d6 * HP + (((uint32_t)d >> 6) & (R5 - 1))], 1u);
            } else if (valid) {   // the digit alone (a later pass checks the grid)
                int32_t iz;
                d6 = (uint32_t)l0_layer_any(P, v[r].z, iz) & (R - 1);
            }
            const uint64_t same = wave_peers<6>(d6, valid);
            const uint32_t rw = (uint32_t)__popcll(same & lt);
            if (valid && rw == 0) wcnt[d6][r * kL0W + w] = (uint8_t)__popcll(same);
            dgp |= d6 << (8 * r);
            rwp |= rw << (8 * r);
        }
        lds_barrier();
        if (w == 0) {
            uint32_t ex;
            const uint32_t tot = l0_tile_prefix<R>(wcnt, wpre, lane, ex);
            dbase[lane] = ex;
            gofs[lane] = goffr - ex;
            goffr += tot;
        }
        lds_barrier();
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + tid;
            if (i < n) {
                const uint32_t d6 = (dgp >> (8 * r)) & 0xFFu;
                const uint32_t q = dbase[d6] + wpre[d6][r * kL0W + w] + ((rwp >> (8 * r)) & 0xFFu);
                sp[q] = v[r];
                if constexpr (KEYS) sk[q] = kk[r];
                else sk[q] = (uint16_t)(r * kL0BS + tid);
                sd[q] = (uint8_t)d6;
            }
        }
        load_tile(v, kk, pf);   // past the group's end: its last tile again, no branch
        lds_barrier();
        const uint32_t tn = (uint32_t)((n - base) < (uint64_t)kL0Tile ? (n - base) : (uint64_t)kL0Tile);
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {   // past tn: a duplicate of the last store
            const uint32_t j = min((uint32_t)r * kL0BS + tid, tn - 1);
            const uint32_t dst = gofs[sd[j]] + j;
            O.p[dst] = sp[j];
            if constexpr (KEYS) O.k[dst] = sk[j];
            else O.k[dst] = (uint32_t)(base + sk[j]);
        }
    };
#if PCC_L0_PF == 2
    // two register tiles: tile t + 2 is loaded while tiles t + 1 and t run
    float4 va[kL0IPT], vb[kL0IPT];
    uint32_t ka[kL0IPT], kb[kL0IPT];
    load_tile(va, ka, t0);
    l0_dummy_stores(dummy, va);   // enter the loop with the back-edge's pending ops
    load_tile(vb, kb, min(t0 + 1, t1 - 1));
    l0_dummy_stores(dummy, vb);
    for (uint32_t tile = t0; tile < t1; tile += 2) {
        body(tile, va, ka, min(tile + 2, t1 - 1));
        if (tile + 1 >= t1) break;
        body(tile + 1, vb, kb, min(tile + 3, t1 - 1));
    }
#else
    float4 v[kL0IPT];
    uint32_t kk[kL0IPT];
    load_tile(v, kk, t0);
    l0_dummy_stores(dummy, v);   // enter the loop with the back-edge's pending ops
    for (uint32_t tile = t0; tile < t1; tile++) body(tile, v, kk, min(tile + 1, t1 - 1));
#endif
    lds_barrier();
    if (pairs)
        for (int i = tid; i < R * R5; i += kL0BS)
            gcnt[((uint64_t)(i / R5) * ngroups + g) * R5 + (i % R5)] = h[(i / R5) * HP + (i % R5)];
    if (err) set_err(ctr, err);
}

// ---- level-0 binning with pass 0 folded into pass 1 (grids of at most two
// level-0 cells per axis).  k_l0_tile6 writes every tile IN PLACE, partitioned by
// the low 6 layer bits d6 (tile-major: a tile's output range is its input range,
// so no global digit offsets and no counting pass are needed), and records per
// tile its digit counts (cnt6, digit-major: the exclusive scan of cnt6 is the
// position of each tile's run in the digit-partitioned order k_l0_down6g writes)
// and each run's physical start (ph6, digit-major too); per group the (d6, d5) pair counts,
// with the cell part of d5 taken from the PARITY of the absolute cell indices
// (the grid is unknown until the bounding box is; parities name the cells of a
// grid of at most two cells per axis, which the host checks after the pass and
// otherwise falls back to the three-pass binning); and the bounding box
// (converter.rs:96-104).  k_l0_down5g<., true> then walks each d6 bucket as the
// sequence of that digit's runs, tile after tile, i.e. in key order.  Without
// external keys a point's key is its tile's base plus its index in the tile, so
// pass 1 writes that 16-bit index only.
// RB1: the low layer bits of pass 1 (6: 64 digits, runs of ~48 points for pass
// 2; 5: 32 digits, runs of ~96), the pair's high part then the cell parity and
// the layer's other kL0LayerBits - RB1 bits.
// CB: the pair's cell bits, the absolute cell indices modulo 2 (CB = 3: a grid
// of at most two cells per axis) or modulo 4 (CB = 6: at most four, config 3).
template <bool KEYS, int RB1 = 6, int CB = 3>
__global__ __launch_bounds__(kL0BS, CB == 3 ? 8 : 1) void k_l0_tile6(const Point* __restrict__ in, const uint32_t* __restrict__ keys,
                                                       Arena O, uint64_t n, L0Params P, uint32_t ntiles, uint32_t tpg,
                                                       uint32_t ngroups, uint32_t* __restrict__ cnt6,
                                                       uint32_t* __restrict__ ph6, uint32_t* __restrict__ gcnt,
                                                       float* __restrict__ part, uint32_t* __restrict__ flag,
                                                       Arena dummy, uint32_t g0, uint32_t cstride,
                                                       const uint32_t* __restrict__ glist = nullptr) {
    constexpr int R = 1 << RB1, HB = kL0LayerBits - RB1, R5 = (1 << CB) << HB, HP = R5 + 1;
    constexpr uint32_t PB = CB / 3, PM = (1u << PB) - 1u;
    static_assert(CB == 3 || CB == 6, "cell bits: parity or modulo 4 per axis");
    using KT = typename std::conditional<KEYS, uint32_t, uint16_t>::type;
    __shared__ float4 sp[kL0Tile];
    __shared__ KT sk[kL0Tile];
    __shared__ alignas(16) uint8_t wcnt[R][kL0RC];
    __shared__ alignas(16) uint16_t wpre[R][kL0RP];
    __shared__ uint32_t dbase[R];
    __shared__ uint32_t h[R * HP];
    __shared__ float sb[kL0W][6];
    // g0: the first group of this launch (uploads, Engine::pre0_count), or glist:
    // the launch's groups (input landing in pieces, Engine::input_landed); the run
    // records' rows are cstride tiles apart and the pair-count rows ngroups groups
    const uint32_t tid = threadIdx.x, w = tid / 64, lane = tid & 63;
    const uint32_t g = glist ? glist[blockIdx.x] : g0 + blockIdx.x;
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (int i = tid; i < R * HP; i += kL0BS) h[i] = 0;
    for (int i = tid; i < kL0RC * R / 4; i += kL0BS) reinterpret_cast<uint32_t*>(&wcnt[0][0])[i] = 0;
    const uint64_t lt = lanemask_lt();
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nf = 0;
    const uint32_t t0 = g * tpg, t1 = min(t0 + tpg, ntiles);
    // per-tile run records through buffer descriptors (scalar bases, 32-bit offsets)
    const __amdgpu_buffer_rsrc_t rC = srd(cnt6, 4ull * R * cstride), rH = srd(ph6, 4ull * R * cstride);
    auto load_tile = [&](float4* v, uint32_t* kk, uint32_t tile) {   // unconditional, clamped (see k_l0_down6g)
        const uint64_t base = (uint64_t)tile * kL0Tile;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = min(base + (uint64_t)r * kL0BS + tid, n - 1);
            v[r] = p4[i];
            if constexpr (KEYS) kk[r] = keys[i];
        }
        asm volatile("" ::: "memory");
    };
    auto body = [&](uint32_t tile, float4* v, uint32_t* kk, uint32_t pf) {
        const uint64_t base = (uint64_t)tile * kL0Tile;
        lds_barrier();   // the last tile's stores have read the staging arrays
        uint32_t dgp = 0, rwp = 0;
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + tid;
            const bool valid = i < n;
            uint32_t d6 = 0;
            if (valid) {
                const float x = v[r].x, y = v[r].y, z = v[r].z;
                nf |= nf_class(x, y, z);
                mn[0] = fminf(mn[0], x); mn[1] = fminf(mn[1], y); mn[2] = fminf(mn[2], z);
                mx[0] = fmaxf(mx[0], x); mx[1] = fmaxf(mx[1], y); mx[2] = fmaxf(mx[2], z);
            }
            // cell indices (metadata.rs:100-102) and the layer relative to the
            // cell's first one, exact quotients, IEEE lanes behind one ballot
            bool amb = !rc_ok(v[r].x) || !rc_ok(v[r].y);
            int32_t iz;
            int64_t ll = l0_layer_rc(P, v[r].z, iz, amb);
            int32_t ix = sat_i32(floorf(div_rc(v[r].x, P.cs, P.inv_cs)));
            int32_t iy = sat_i32(floorf(div_rc(v[r].y, P.cs, P.inv_cs)));
            if (__ballot(valid && amb)) {
                if (valid && amb) {
                    ll = l0_layer(P, v[r].z, iz);
                    ix = cell_index1(v[r].x, P.cs);
                    iy = cell_index1(v[r].y, P.cs);
                }
            }
            if (valid) {
                nf |= (ll < 0 || ll >= (int64_t)kL0Layers) ? kNfLayer : 0u;   // (an infinite z too: rebinned apart)
                d6 = (uint32_t)ll & (R - 1);
                const uint32_t par = ((uint32_t)ix & PM) | (((uint32_t)iy & PM) << PB) | (((uint32_t)iz & PM) << (2 * PB));
                atomicAdd(&h[d6 * HP + ((par << HB) | (((uint32_t)ll >> RB1) & ((1u << HB) - 1u)))], 1u);
            }
            const uint64_t same = wave_peers<RB1>(d6, valid);
            const uint32_t rw = (uint32_t)__popcll(same & lt);
            if (valid && rw == 0) wcnt[d6][r * kL0W + w] = (uint8_t)__popcll(same);
            dgp |= d6 << (8 * r);
            rwp |= rw << (8 * r);
        }
        lds_barrier();
        if (w == 0) {
            uint32_t ex;
            const uint32_t tot = l0_tile_prefix<R>(wcnt, wpre, lane, ex);
            uint32_t ln = lane;   // (recomputed addresses: see k_l0_down5g)
            asm volatile("" : "+v"(ln));
            if (ln < (uint32_t)R) {
                dbase[ln] = ex;
                const uint32_t ro = (ln * cstride + tile) * 4;   // this tile's run of digit `lane`: length, start
                bst(rC, ro, tot);
                bst(rH, ro, tile * (uint32_t)kL0Tile + ex);
            }
        }
        lds_barrier();
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint64_t i = base + (uint64_t)r * kL0BS + tid;
            if (i < n) {
                const uint32_t d6 = (dgp >> (8 * r)) & 0xFFu;
                const uint32_t q = dbase[d6] + wpre[d6][r * kL0W + w] + ((rwp >> (8 * r)) & 0xFFu);
                sp[q] = v[r];
                if constexpr (KEYS) sk[q] = kk[r];
                else sk[q] = (uint16_t)(r * kL0BS + tid);
            }
        }
        load_tile(v, kk, pf);   // past the group's end: its last tile again, no branch
        lds_barrier();
        const uint32_t tn = (uint32_t)((n - base) < (uint64_t)kL0Tile ? (n - base) : (uint64_t)kL0Tile);
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {   // past tn: a duplicate of the last store
            const uint32_t j = min((uint32_t)r * kL0BS + tid, tn - 1);
            O.p[base + j] = sp[j];
            if constexpr (KEYS) O.k[base + j] = sk[j];
            else reinterpret_cast<uint16_t*>(O.k)[base + j] = sk[j];   // key - tile base (k_l0_down5g adds it back)
        }
    };
    if (t0 < t1) {
        float4 v[kL0IPT];
        uint32_t kk[kL0IPT];
        load_tile(v, kk, t0);
        l0_dummy_stores(dummy, v);   // enter the loop with the back-edge's pending ops
        for (uint32_t tile = t0; tile < t1; tile++) body(tile, v, kk, min(tile + 1, t1 - 1));
    }
    for (int d = 32; d > 0; d >>= 1)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
        }
    if (lane == 0)
        for (int a = 0; a < 3; a++) { sb[w][a] = mn[a]; sb[w][3 + a] = mx[a]; }
    if (nf) atomicOr(flag, nf);
    __syncthreads();
    if (tid < 6) {
        float r = sb[0][tid];
        for (int q = 1; q < kL0W; q++) r = tid < 3 ? fminf(r, sb[q][tid]) : fmaxf(r, sb[q][tid]);
        part[g * 6 + tid] = r;
    }
    for (int i = tid; i < R * R5; i += kL0BS)
        gcnt[((uint64_t)(i / R5) * ngroups + g) * R5 + (i % R5)] = h[(i / R5) * HP + (i % R5)];
}

// Segment starts of the digit-partitioned order from the tile-major pass 1:
// start of (d6, group g) = the scanned run position of the group's first tile.
__global__ void k_l0_tstarts(const uint32_t* __restrict__ voff, uint32_t ntiles, uint32_t tpg, uint32_t ngroups,
                             uint64_t n, uint32_t* __restrict__ starts, uint32_t R1) {   // R1: pass-1 digits
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R1 * (ngroups + 1)) return;
    const uint32_t d6 = i / (ngroups + 1), g = i % (ngroups + 1);
    const uint64_t t = (uint64_t)g * tpg;
    starts[i] = g < ngroups ? voff[(uint64_t)d6 * ntiles + t] : (d6 + 1 < R1 ? voff[(uint64_t)(d6 + 1) * ntiles] : (uint32_t)n);
}

// Per (d6, d5): exclusive prefix over the groups of the pair counts of
// k_l0_tile6, read from their parity slots (pmap: dense d5 -> parity slot, 0xFF
// none) into the dense-d5 layout k_l0_down5g reads, and the dense histogram
// bin (d5 << 6 | d6).  A count in a parity slot no dense d5 names is a point
// outside the grid (pass 2 reports it).
struct L0PMap { uint16_t s[256]; };   // 0xFFFF: none
template <int LB = 6, int CB = 3>
__global__ __launch_bounds__(1024) void k_l0_gprefix_par(const uint32_t* __restrict__ gsrc, uint32_t* __restrict__ gdst,
                                                         uint32_t ngroups, uint32_t D, L0PMap pm,
                                                         uint32_t* __restrict__ hist, Counters* ctr) {
    constexpr int R5 = (1 << CB) << (kL0LayerBits - LB), NC = 1024 / R5;
    __shared__ uint32_t part[NC][R5];
    const uint32_t d6 = blockIdx.x, d5 = threadIdx.x % R5, c = threadIdx.x / R5;
    const uint32_t gpc = (ngroups + NC - 1) / NC, g0 = min(c * gpc, ngroups), g1 = min(g0 + gpc, ngroups);
    const uint32_t ps = pm.s[d5];
    const uint32_t* row = gsrc + (uint64_t)d6 * ngroups * R5 + (ps < (uint32_t)R5 ? ps : 0u);
    uint32_t* orow = gdst + (uint64_t)d6 * ngroups * R5 + d5;
    uint32_t acc = 0;
    if (ps < (uint32_t)R5)
        for (uint32_t g = g0; g < g1; g++) acc += row[(uint64_t)g * R5];
    part[c][d5] = acc;
    __syncthreads();
    if (c == 0) {
        uint32_t a = 0;
        for (int q = 0; q < NC; q++) { const uint32_t v = part[q][d5]; part[q][d5] = a; a += v; }
        const uint32_t d0 = (d5 << LB) | d6;
        if (d0 < D) hist[d0] = a;
        else if (a) set_err(ctr, ERR_L0_RANGE);
    }
    __syncthreads();
    acc = part[c][d5];
    for (uint32_t g = g0; g < g1; g++) {
        orow[(uint64_t)g * R5] = acc;
        if (ps < (uint32_t)R5) acc += row[(uint64_t)g * R5];
    }
}

// Pass-2 windows over the tile-major pass-1 output: window k of unit u covers the
// unit's points [a + k T, min(a + (k+1) T, b)) of its d6 bucket; per window the
// tiles holding its first and last point (the largest tile whose scanned run
// start is <= the position), found by binary search over the unit's tiles.
struct L0UnitW { uint32_t d6, a, b, t0, t1, w0, pad_g0, pad; };   // pad_g0: the unit's first group
__device__ __forceinline__ uint32_t l0_tile_of(const uint32_t* __restrict__ vrow, uint32_t t0, uint32_t t1, uint32_t v) {
    uint32_t lo = t0, hi = t1 - 1;   // vrow[t0] <= v (the unit's first run starts at a <= v)
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (vrow[mid] <= v) lo = mid; else hi = mid - 1;
    }
    return lo;
}
// (dcnt: the unit and window counts on the device, k_l0_uplan; else the arguments)
__global__ void k_l0_wplan(const L0UnitW* __restrict__ units, uint32_t nunits, uint32_t nwin,
                           const uint32_t* __restrict__ voff, uint32_t ntiles, uint2* __restrict__ wt,
                           const uint32_t* __restrict__ dcnt) {
    const uint32_t wi = blockIdx.x * blockDim.x + threadIdx.x;
    if (dcnt) { nunits = dcnt[0]; nwin = dcnt[1]; }
    if (wi >= nwin) return;
    uint32_t lo = 0, hi = nunits - 1;   // the unit of window wi: last with w0 <= wi
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (units[mid].w0 <= wi) lo = mid; else hi = mid - 1;
    }
    const L0UnitW U = units[lo];
    const uint32_t v0 = U.a + (wi - U.w0) * (uint32_t)kL0Tile;
    const uint32_t v1 = min(v0 + (uint32_t)kL0Tile, U.b) - 1;
    const uint32_t* vrow = voff + (uint64_t)U.d6 * ntiles;
    wt[wi] = make_uint2(l0_tile_of(vrow, U.t0, U.t1, v0), l0_tile_of(vrow, U.t0, U.t1, v1));
}

// The pass-2 units of the folded binning, planned on the device (no host round
// trip between the passes): row d6 of the segment starts is cut into
// ceil(size / target) units, unit k taking the groups whose segment starts at
// [k target, (k + 1) target) from the row's first point (a segment is never
// split; a unit no segment starts in is empty and its block exits).  Units are
// numbered row after row, one thread each; umax >= their count (64 + n /
// target) is the launch size.  wn[u]: the unit's windows of kL0Tile points,
// whose exclusive scan is each unit's first window (k_l0_uplan_w0); out[0]: the
// unit count.
__global__ __launch_bounds__(256) void k_l0_uplan(const uint32_t* __restrict__ starts, uint32_t ngroups, uint32_t tpg,
                                                  uint32_t ntiles, uint32_t target, uint32_t umax,
                                                  L0UnitW* __restrict__ uw, uint32_t* __restrict__ wn,
                                                  uint32_t* __restrict__ out, uint32_t R1, int cols) {   // R1 <= 64 rows
    __shared__ uint32_t ub[65];
    const uint32_t tid = threadIdx.x, u = blockIdx.x * 256 + tid;
    if (tid < 64) {   // units per row, exclusive scan over the rows (wave 0)
        const uint32_t* row = starts + (uint64_t)min(tid, R1 - 1) * (ngroups + 1);
        const uint32_t nu = tid < R1 ? (row[ngroups] - row[0] + target - 1) / target : 0u;
        uint32_t x = nu;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (tid >= (uint32_t)d) x += y;
        }
        ub[tid] = x - nu;
        if (tid == 63) ub[64] = x;
    }
    __syncthreads();
    const uint32_t nunits = ub[64];
    if (u == 0) out[0] = nunits;
    if (u >= umax) return;
    L0UnitW W{0, 0, 0, 0, 0, 0, 0, 0};
    if (u < nunits) {
        uint32_t lo = 0, hi = 63;   // the row: last with ub[d] <= u
        while (lo < hi) {
            const uint32_t m = (lo + hi + 1) >> 1;
            if (ub[m] <= u) lo = m; else hi = m - 1;
        }
        const uint32_t d = lo, k = u - ub[d];
        const uint32_t* row = starts + (uint64_t)d * (ngroups + 1);
        const uint32_t r0 = row[0];
        auto first_at = [&](uint64_t off) {   // first group whose segment starts >= r0 + off (ngroups: none)
            uint32_t a = 0, b = ngroups;
            while (a < b) {
                const uint32_t m = (a + b) >> 1;
                if ((uint64_t)(row[m] - r0) >= off) b = m; else a = m + 1;
            }
            return a;
        };
        const uint32_t g0 = first_at((uint64_t)k * target), g1 = first_at((uint64_t)(k + 1) * target);
        W.d6 = d;
        W.a = row[g0];
        W.b = row[g1];
        W.t0 = g0 * tpg;
        W.t1 = min(g1 * tpg, ntiles);
        W.pad_g0 = min(g0, ngroups - 1);
    }
    uint32_t p = u;
    if (cols && u < nunits) {
        // launch position column by column: unit k of every row, then unit k + 1
        // (concurrent blocks read the same tiles' runs of all 64 digits, whose
        // boundary lines they share), and in a full column the 8 digits 8x .. 8x + 7
        // on the blocks of one XCD (block i runs on XCD i mod 8), so neighbours
        // share the XCD's L2
        const uint32_t d = W.d6, k = u - ub[d];
        uint32_t base = 0, q = 0, present = 0;
        for (uint32_t r = 0; r < 64; r++) {
            const uint32_t nr = ub[r + 1] - ub[r];
            base += min(nr, k);
            present += nr > k ? 1u : 0u;
            q += (r < d && nr > k) ? 1u : 0u;
        }
        p = base + (present == 64 ? (d % 8) * 8 + d / 8 : q);
    }
    uw[p] = W;
    wn[p] = (W.b - W.a + kL0Tile - 1) / kL0Tile;
}
__global__ void k_l0_uplan_w0(L0UnitW* __restrict__ uw, const uint32_t* __restrict__ w0, uint32_t umax) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < umax) uw[u].w0 = w0[u];
}

// start of segment (d6, g) of the pass-1 output, g = 0..ngroups (the end)
__global__ void k_l0_gstarts(const uint32_t* __restrict__ offs, uint32_t ngroups, uint64_t n,
                             uint32_t* __restrict__ starts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 64 * (ngroups + 1)) return;
    const uint32_t d6 = i / (ngroups + 1), g = i % (ngroups + 1);
    const uint64_t idx = (uint64_t)d6 * ngroups + g;   // (d6, ngroups) = (d6 + 1, 0)
    starts[i] = idx < 64ull * ngroups ? offs[idx] : (uint32_t)n;
}

// per (d6, d5): exclusive prefix of the group counts (in place) and the dense
// histogram bin (d5 << 6 | d6).  One block per d6, thread = (chunk, d5).
template <int R5>
__global__ __launch_bounds__(1024) void k_l0_gprefix(uint32_t* __restrict__ gcnt, uint32_t ngroups, uint32_t D,
                                                     uint32_t* __restrict__ hist, Counters* ctr) {
    constexpr int NC = 1024 / R5;
    __shared__ uint32_t part[NC][R5];
    const uint32_t d6 = blockIdx.x, d5 = threadIdx.x % R5, c = threadIdx.x / R5;
    const uint32_t gpc = (ngroups + NC - 1) / NC, g0 = min(c * gpc, ngroups), g1 = min(g0 + gpc, ngroups);
    uint32_t* row = gcnt + (uint64_t)d6 * ngroups * R5 + d5;
    uint32_t acc = 0;
    for (uint32_t g = g0; g < g1; g++) acc += row[(uint64_t)g * R5];
    part[c][d5] = acc;
    __syncthreads();
    if (c == 0) {
        uint32_t a = 0;
        for (int q = 0; q < NC; q++) { const uint32_t v = part[q][d5]; part[q][d5] = a; a += v; }
        const uint32_t d0 = (d5 << 6) | d6;
        if (d0 < D) hist[d0] = a;
        else if (a) set_err(ctr, ERR_L0_RANGE);
    }
    __syncthreads();
    acc = part[c][d5];
    for (uint32_t g = g0; g < g1; g++) {
        const uint32_t v = row[(uint64_t)g * R5];
        row[(uint64_t)g * R5] = acc;
        acc += v;
    }
}

// Level-0 dense id from the level-1 quotients (exact halving, see l1_dense) and
// the point's child slab among the slab's 24 (octant * 3 + layer select, as
// k_l0_dcap_from1 numbers them); -1 outside the grid.
__device__ __forceinline__ int64_t l0_dense_dest(const L0Params& P, float x, float y, float z, uint32_t& dest) {
    int32_t ix1, iy1, iz1, u1;
    bool amb = !PCC_L0_RC;
    if (PCC_L0_RC) {   // reciprocal quotients, exact lanes redone below
        amb = P.exact || !rc_ok(x) || !rc_ok(y) || !rc_ok(z);
        ix1 = sat_i32(floorf(div_rc(x, P.csc, P.inv_csc)));
        iy1 = sat_i32(floorf(div_rc(y, P.csc, P.inv_csc)));
        iz1 = sat_i32(floorf(div_rc(z, P.csc, P.inv_csc)));
        u1 = sat_i32(truncf(div_rc(z, P.crc, P.inv_crc)));
    }
    if (__ballot(amb)) {
        if (amb) {
            ix1 = cell_index1(x, P.csc);
            iy1 = cell_index1(y, P.csc);
            iz1 = cell_index1(z, P.csc);
            u1 = sat_i32(z / P.crc);
        }
    }
    const int32_t iz0 = iz1 >> 1, t0 = u1 / 2;
    const int32_t gx0 = (ix1 >> 1) - P.lo[0], gy0 = (iy1 >> 1) - P.lo[1], gz0 = iz0 - P.lo[2];
    const int64_t ll0 = (int64_t)t0 - ((int64_t)P.dim2 * iz0 - 2);
    const int64_t ll1 = (int64_t)u1 - ((int64_t)P.dim2 * iz1 - 2);
    dest = (uint32_t)(((ix1 & 1) | ((iy1 & 1) << 1) | ((iz1 & 1) << 2)) * 3 + (u1 - (2 * t0 - 1)));
    const bool ok = gx0 >= 0 && gy0 >= 0 && gz0 >= 0 && gx0 < P.g[0] && gy0 < P.g[1] && gz0 < P.g[2] && ll0 >= 0 &&
                    ll0 < P.nl && ll1 >= 0 && ll1 < (int64_t)kL0Layers;
    return ok ? (((int64_t)gz0 * P.g[1] + gy0) * P.g[0] + gx0) * kL0Layers + ll0 : -1;
}

// Pass 2 over one unit (consecutive segments of one d6 bucket), running
// offsets per d5 kept in wave-0 registers; the same pipelining as pass 1.
// TM: the pass-1 output is tile-major (k_l0_tile6).  The unit is then read in
// windows of one tile's size; window k's positions map to the runs of the tiles
// wt[k] = (first, last) through a slice of their scanned run starts (voff) and
// physical starts (tile base + lp6) staged in LDS, fetched one window ahead and
// stored one step before use.
struct L0Slice { uint32_t tf, ntl, sv, sp; };
// LB: the low digit's bits (pass 1: 6, or 5 with R5 = 64 high digits)
// R5 = 256 (fold over at most four cells per axis): one workgroup per CU (LDS).
template <int R5, bool TM, bool K16 = false, int LB = 6>
__global__ __launch_bounds__(kL0BS, R5 > 64 ? 1 : 8) void k_l0_down5g(Arena S, Arena O, L0Params P, const L0Unit* __restrict__ units,
                                                        const uint32_t* __restrict__ starts, uint32_t ngroups,
                                                        const uint32_t* __restrict__ gpre,
                                                        const uint32_t* __restrict__ cnt_scan,
                                                        const uint32_t* __restrict__ sid, uint32_t D,
                                                        uint32_t* __restrict__ dcap, Arena dummy, Counters* ctr,
                                                        const L0UnitW* __restrict__ uw, const uint2* __restrict__ wt,
                                                        const uint32_t* __restrict__ voff,
                                                        const uint32_t* __restrict__ ph6, uint32_t ntiles) {
    constexpr int R = R5, RB = R5 == 256 ? 8 : R5 == 64 ? 6 : R5 == 32 ? 5 : R5 == 16 ? 4 : R5 == 8 ? 3 : 2;
    static_assert((1 << RB) == R5, "R5 is a power of two in 4..64, or 256");
    constexpr int DPL = R > 64 ? R / 64 : 1;   // wave 0: digits per lane
    constexpr uint32_t LM = (1u << LB) - 1u;
    // slice entries (tiles per window) staged in LDS; a window over more tiles
    // (a sparse digit) searches the run starts in memory
    constexpr uint32_t kSl = R5 == 64 ? 128 : kL0BS;
    __shared__ float4 sp[kL0Tile];
    __shared__ uint32_t sk[kL0Tile];
    __shared__ uint8_t sd[kL0Tile];
    __shared__ alignas(16) uint8_t wcnt[R][kL0RC];
    __shared__ alignas(16) uint16_t wpre[R][kL0RP];
    __shared__ uint32_t dbase[R], gofs[R];
    __shared__ uint32_t hc[R * kDests];
    __shared__ uint32_t slv[TM ? kSl : 1], slp[TM ? kSl : 1];
    const uint32_t tid = threadIdx.x, w = tid / 64, lane = tid & 63;
    uint32_t d6u, a, b, g0u, w0 = 0, nwin = 0;
    if constexpr (TM) {
        const L0UnitW U = uw[blockIdx.x];
        d6u = U.d6; a = U.a; b = U.b; g0u = U.pad_g0; w0 = U.w0;
        nwin = (b - a + kL0Tile - 1) / kL0Tile;
    } else {
        const L0Unit U = units[blockIdx.x];
        d6u = U.d6; g0u = U.g0;
        a = starts[U.d6 * (ngroups + 1) + U.g0];
        b = starts[U.d6 * (ngroups + 1) + U.g1];
    }
    uint32_t runr[DPL];   // wave 0, lane t: next output position of digit t (R <= 64) or t * DPL + k
#pragma unroll
    for (int k = 0; k < DPL; k++) {
        const uint32_t dg = R > 64 ? lane * DPL + k : lane;
        runr[k] = 0;
        if (w == 0 && dg < (uint32_t)R) {
            const uint32_t d0 = (dg << LB) | d6u;
            runr[k] = d0 < D ? cnt_scan[d0] + gpre[((uint64_t)d6u * ngroups + g0u) * R + dg] : 0u;
        }
        gofs[dg & (R - 1)] = runr[k];   // (an LDS write of runr: its load is complete before the loop)
    }
    for (int i = tid; i < R * kDests; i += kL0BS) hc[i] = 0;
    for (int i = tid; i < kL0RC * R / 4; i += kL0BS) reinterpret_cast<uint32_t*>(&wcnt[0][0])[i] = 0;
    const uint64_t lt = lanemask_lt();
    uint32_t err = 0;
    const uint32_t* vrow = TM ? voff + (uint64_t)d6u * ntiles : nullptr;
    const uint32_t* prow = TM ? ph6 + (uint64_t)d6u * ntiles : nullptr;
    const __amdgpu_buffer_rsrc_t rV = srd(vrow, TM ? 4ull * ntiles : 0), rPh = srd(prow, TM ? 4ull * ntiles : 0);
    // TM: this thread's entry of the slice of window k (run start, physical
    // start), loaded into registers; the window's tiles come from wt (scalar)
    auto slice_fetch = [&](uint32_t k, L0Slice& q) {
        k = min(k, nwin - 1);
        const uint2 t = wt[w0 + k];
        q.tf = __builtin_amdgcn_readfirstlane(t.x);
        q.ntl = __builtin_amdgcn_readfirstlane(t.y - t.x + 1);
        const uint32_t o = (q.tf + min(tid, q.ntl - 1)) * 4;
        q.sv = bld(rV, o);
        q.sp = bld(rPh, o);
    };
    auto slice_store = [&](const L0Slice& q) {
        if (tid < q.ntl && tid < kSl) {
            uint32_t t = tid;   // the LDS addresses recomputed here, not kept live (spilled at the 64-VGPR cap)
            asm volatile("" : "+v"(t));
            slv[t] = q.sv;
            slp[t] = q.sp;
        }
    };
    // physical position of the unit's point at virtual position v (window of q)
    // physical positions of this thread's kL0IPT points of the window at `base`:
    // one binary search per row over the window's slice, the rows' LDS reads
    // interleaved (a uniform number of halvings); a sparse digit's window of more
    // than kSl tiles searches the run starts in memory
    auto xlate3 = [&](const L0Slice& q, uint32_t base, uint32_t* ix) {
        uint32_t vv[kL0IPT];
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) vv[r] = min(base + (uint32_t)r * kL0BS + tid, b - 1);
        if (q.ntl <= kSl) {
            uint32_t lo[kL0IPT], step = 1;
            while (step < q.ntl) step <<= 1;
#pragma unroll
            for (int r = 0; r < kL0IPT; r++) lo[r] = 0;
            for (step >>= 1; step; step >>= 1) {   // largest lo with slv[lo] <= v (slv[0] <= v)
#pragma unroll
                for (int r = 0; r < kL0IPT; r++) {
                    const uint32_t m = lo[r] + step;
                    lo[r] = (m < q.ntl && slv[m < q.ntl ? m : 0] <= vv[r]) ? m : lo[r];
                }
            }
#pragma unroll
            for (int r = 0; r < kL0IPT; r++) ix[r] = slp[lo[r]] + (vv[r] - slv[lo[r]]);
        } else {
#pragma unroll
            for (int r = 0; r < kL0IPT; r++) {
                const uint32_t t = l0_tile_of(vrow, q.tf, q.tf + q.ntl, vv[r]);
                ix[r] = prow[t] + (vv[r] - vrow[t]);
            }
        }
    };
    auto load_tile = [&](float4* v, uint32_t* kk, uint32_t base, const uint32_t* ixp) {   // unconditional, clamped (see k_l0_down6g)
        uint32_t ix[kL0IPT];
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            if constexpr (TM) ix[r] = ixp[r];
            else ix[r] = min(base + (uint32_t)r * kL0BS + tid, b - 1);
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            v[r] = S.p[ix[r]];
            if constexpr (K16) {   // key = tile base + 16-bit index in the tile (k_l0_tile6)
                const uint32_t tb = __umulhi(ix[r], 0xAAAAAAABu) >> 11;   // ix / 3072 (ix < 2^32)
                kk[r] = tb * (uint32_t)kL0Tile + reinterpret_cast<const uint16_t*>(S.k)[ix[r]];
            } else {
                kk[r] = S.k[ix[r]];
            }
        }
        asm volatile("" ::: "memory");   // keep the loads ahead of the tile's stores
    };
    if (a >= b) return;   // (units are never empty)
    auto body = [&](uint32_t base, float4* v, uint32_t* kk, uint32_t pf, L0Slice& qn, L0Slice& qf) {
        const uint32_t tn = min(b - base, (uint32_t)kL0Tile);
        lds_barrier();
        uint32_t dgp = 0, rwp = 0;
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint32_t j = (uint32_t)r * kL0BS + tid;
            const bool valid = j < tn;
            uint32_t d5 = 0;
            if (valid) {
                uint32_t dest;
                const int64_t d = l0_dense_dest(P, v[r].x, v[r].y, v[r].z, dest);
                if (d < 0 || ((uint32_t)d & LM) != d6u || dest >= (uint32_t)kDests) {
                    err = ERR_L0_RANGE;
                } else {
                    d5 = ((uint32_t)d >> LB) & (R - 1);
                    atomicAdd(&hc[d5 * kDests + dest], 1u);
                }
            }
            const uint64_t same = wave_peers<RB>(d5, valid);
            const uint32_t rw = (uint32_t)__popcll(same & lt);
            if (valid && rw == 0) wcnt[d5][r * kL0W + w] = (uint8_t)__popcll(same);
            dgp |= d5 << (8 * r);
            rwp |= rw << (8 * r);
        }
        lds_barrier();
        if (w == 0) {
            if constexpr (R > 64) {
                uint32_t tot[DPL], ex[DPL];
                l0_tile_prefix_n<R>(wcnt, wpre, lane, tot, ex);
#pragma unroll
                for (int k = 0; k < DPL; k++) {
                    dbase[lane * DPL + k] = ex[k];
                    gofs[lane * DPL + k] = runr[k] - ex[k];
                    runr[k] += tot[k];
                }
            } else {
                uint32_t ex;
                const uint32_t tot = l0_tile_prefix<R>(wcnt, wpre, lane, ex);
                // the LDS addresses are recomputed here, not kept live across the loop
                // (at the 64-VGPR cap they were spilled, and each reload drained vmcnt)
                uint32_t ln = lane;
                asm volatile("" : "+v"(ln));
                if (ln < (uint32_t)R) {
                    dbase[ln] = ex;
                    gofs[ln] = runr[0] - ex;
                    runr[0] += tot;
                }
            }
        }
        lds_barrier();
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {
            const uint32_t j = (uint32_t)r * kL0BS + tid;
            if (j < tn) {
                const uint32_t d5 = (dgp >> (8 * r)) & 0xFFu;
                const uint32_t q = dbase[d5] + wpre[d5][r * kL0W + w] + ((rwp >> (8 * r)) & 0xFFu);
                sp[q] = v[r];
                sk[q] = kk[r];
                sd[q] = (uint8_t)d5;
            }
        }
        {
            uint32_t ixn[kL0IPT];   // TM: the next window's physical positions (its slice is in LDS)
            if constexpr (TM) xlate3(qn, pf, ixn);
            load_tile(v, kk, pf, ixn);
        }
        if constexpr (TM) slice_fetch((pf - a) / kL0Tile + 1, qf);   // the window after it
        lds_barrier();
#pragma unroll
        for (int r = 0; r < kL0IPT; r++) {   // past tn: a duplicate of the last store
            const uint32_t j = min((uint32_t)r * kL0BS + tid, tn - 1);
            const uint32_t dst = gofs[sd[j]] + j;
            O.p[dst] = sp[j];
            O.k[dst] = sk[j];
        }
        // TM: the slice of the window after `pf` (this one's last search is done;
        // searched in the next body after its third barrier)
        if constexpr (TM) slice_store(qf);
    };
    // the tile `k` tiles after `base`, clamped to the unit's last tile
    auto ahead = [&](uint32_t base, uint32_t k) {
        const uint32_t last = a + (b - 1 - a) / kL0Tile * kL0Tile;
        return min(base + k * (uint32_t)kL0Tile, last);
    };
    float4 v[kL0IPT];
    uint32_t kk[kL0IPT];
    L0Slice q0{}, q1{};
    uint32_t ix0[kL0IPT] = {};
    if constexpr (TM) {
        slice_fetch(0, q0);
        slice_store(q0);
        lds_barrier();
        xlate3(q0, a, ix0);
        lds_barrier();
    }
    load_tile(v, kk, a, ix0);
    if constexpr (TM) {
        slice_fetch(1, q1);
        slice_store(q1);   // (waits for this fetch, once; the loop stores each slice a body ahead)
    }
    l0_dummy_stores(dummy, v);
    for (uint32_t base = a; base < b; base += kL0Tile) {   // q1: the slice of the window after `base`
        body(base, v, kk, ahead(base, 1), q1, q0);
        if (base + kL0Tile >= b) break;
        base += kL0Tile;
        body(base, v, kk, ahead(base, 1), q0, q1);
    }
    lds_barrier();
    for (int i = tid; i < R * kDests; i += kL0BS) {
        const uint32_t c = hc[i];
        if (!c) continue;
        const uint32_t d0 = ((uint32_t)(i / kDests) << LB) | d6u;
        if (d0 < D) atomicAdd(&dcap[(uint64_t)sid[d0] * kDests + (uint32_t)(i % kDests)], c);
    }
    if (err) set_err(ctr, err);
}

// per dense slab: non-empty flag; per grid cell: non-empty flag
__global__ void k_l0_flags(const uint32_t* hist, uint32_t D, int32_t nl, uint32_t* sflag, uint32_t* cflag, uint32_t G) {
    uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d < D) sflag[d] = hist[d] ? 1u : 0u;
    if (d < G) {
        uint32_t any = 0;
        for (int32_t l = 0; l < nl; l++) any |= hist[(uint64_t)d * kL0Layers + l];
        cflag[d] = any ? 1u : 0u;
    }
}

__global__ void k_l0_tables(const uint32_t* hist, const uint32_t* cnt_scan, const uint32_t* sflag_scan,
                            const uint32_t* cflag, const uint32_t* cflag_scan, uint32_t D, uint32_t G, L0Params P,
                            int32_t* cell_idx, uint32_t* cell_sb, uint32_t* cell_slab0, uint32_t* slab_cell,
                            int32_t* slab_layer, uint32_t* slab_off, uint32_t* slab_n, const uint32_t* d_tot) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d_tot && d == 0) cell_slab0[d_tot[2]] = d_tot[1];   // (else k_set_u32 from the host totals)
    if (d < G && cflag[d]) {
        const uint32_t r = cflag_scan[d];
        int32_t gx, gy, gz;
        if (P.hashed) {
            const unsigned long long key = P.ckeys[d];
            gx = (int32_t)(key & 0x1FFFFF);
            gy = (int32_t)((key >> 21) & 0x1FFFFF);
            gz = (int32_t)(key >> 42);
        } else {
            gx = (int32_t)(d % (uint32_t)P.g[0]);
            gy = (int32_t)((d / (uint32_t)P.g[0]) % (uint32_t)P.g[1]);
            gz = (int32_t)(d / ((uint32_t)P.g[0] * (uint32_t)P.g[1]));
        }
        cell_idx[3 * r] = P.lo[0] + gx;
        cell_idx[3 * r + 1] = P.lo[1] + gy;
        cell_idx[3 * r + 2] = P.lo[2] + gz;
        cell_sb[r] = 0;
        cell_slab0[r] = sflag_scan[(uint64_t)d * kL0Layers];
    }
    if (d < D && hist[d]) {
        const uint32_t sid = sflag_scan[d];
        const uint32_t g = d / kL0Layers;
        const int32_t ll = (int32_t)(d % kL0Layers);
        const int32_t gz = P.hashed ? (int32_t)(P.ckeys[g] >> 42) : (int32_t)(g / ((uint32_t)P.g[0] * (uint32_t)P.g[1]));
        const int32_t iz = P.lo[2] + gz;
        slab_cell[sid] = cflag_scan[g];
        slab_layer[sid] = ll + (P.dim2 * iz - 2);
        slab_off[sid] = cnt_scan[d];
        slab_n[sid] = hist[d];
    }
}

// Sub-tree build rooted below level 0 (set_root_level): each root cell takes the
// spill batch of the parent bucket it came from (exported with the arrivals,
// export_pending), found by binary search in the (x, y, z)-sorted root table.
__global__ void k_root_sb(const int32_t* __restrict__ cell_idx, uint32_t ncells, const int32_t* __restrict__ rxyz,
                          const uint32_t* __restrict__ rsb, uint32_t nroot, uint32_t* __restrict__ cell_sb,
                          Counters* ctr) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    const int32_t x = cell_idx[3 * c], y = cell_idx[3 * c + 1], z = cell_idx[3 * c + 2];
    uint32_t lo = 0, hi = nroot;
    while (lo < hi) {
        const uint32_t m = (lo + hi) / 2;
        const int32_t* q = rxyz + 3ull * m;
        const bool less = q[0] != x ? q[0] < x : q[1] != y ? q[1] < y : q[2] < z;
        if (less) lo = m + 1;
        else hi = m;
    }
    const int32_t* q = rxyz + 3ull * lo;
    if (lo < nroot && q[0] == x && q[1] == y && q[2] == z) cell_sb[c] = rsb[lo];
    else atomicOr(&ctr->err, (uint32_t)ERR_L0_RANGE);
}

// Pending level (set_max_levels): its slabs' arrivals, concatenated in slab
// order (a cell's slabs are consecutive, so every cell is one range).
__global__ __launch_bounds__(256) void k_export_slabs(Arena A, const uint32_t* __restrict__ slab_off,
                                                      const uint32_t* __restrict__ slab_n,
                                                      const uint32_t* __restrict__ out_off, uint32_t nslabs,
                                                      float4* __restrict__ dp, uint32_t* __restrict__ dk) {
    for (uint32_t s = blockIdx.x; s < nslabs; s += gridDim.x) {
        const uint32_t o = slab_off[s], n = slab_n[s], d = out_off[s];
        for (uint32_t i = threadIdx.x; i < n; i += 256) {
            dp[d + i] = A.p[o + i];
            dk[d + i] = A.k[o + i];
        }
    }
}

// ------------------------------------------------------------------ slab kernels
// Per-slab launch descriptor (one 48-B record: the slab kernels' prologue is
// one load instead of a chain of dependent table loads).
struct SmallDesc {
    uint32_t s, off, n, dbase;
    int32_t t, cx, cy, cz;
    uint32_t sb, dlen, pad0, pad1;
    uint32_t ng;   // merge, dense slabs of levels >= 1: the first ng seeds are grid points (one per slot)
};

struct SlabParams {
    Arena in, nx;
    Point* grid;
    const int32_t* cell_idx;
    const uint32_t* cell_sb;
    const uint32_t* slab_cell;
    const int32_t* slab_layer;
    const uint32_t* slab_off;
    const uint32_t* slab_n;
    const uint32_t* list;
    const uint32_t* grid_off;
    const uint32_t* dcap;
    const uint32_t* dest_off;
    uint32_t* slab_grid_n;
    uint32_t* dest_n;
    uint32_t* gcap;       // 24 x 24 per slab: arrivals of each child slab per grandchild slab
    const struct SmallDesc* sdesc;   // small-slab descriptors (k_slab_small)
    uint32_t nlist;
    const struct SmallDesc* wdesc;   // one-wave slab descriptors (k_slab_wave)
    const struct SmallDesc* ddesc;   // dense slab descriptors (k_slab), by block
    uint32_t nwave;
    Counters* ctr;
    float cs;
    LevelGeo G;
    int32_t tx, ty;
    int32_t check_gchild;
    uint32_t kf_lo, kf_n;         // merge mode: keys in [kf_lo, kf_lo + kf_n) are forced emissions (engine.h PriorState)
    const float4* inj;            // merge mode: seeds of levels >= 1 (a small slab reads its own in place)
    const unsigned long long* inj_rec;   // merge mode: per grid seed its slot-table record (k_seed_rec)
    const uint32_t* inj_keys;
    unsigned long long* stamps;   // diagnostic build only
};

// Dense slabs (>= kSmallMax arrivals): one 1024-thread workgroup per slab, the
// slab's whole hex layer as a direct-mapped slot table in LDS.
struct DenseLds {
    static constexpr int BS = kDenseBS, TAB = kDenseTab, NW = BS / 64;
    unsigned long long tab[TAB];   // occupant: (d2 bits << 33) | (child slab << 28) | j
    static constexpr int HW = (TAB + 1) / 2;
    uint32_t head[HW];             // per slot, 16 bits: (chunk tag << 11) | head of the slot's candidate list
    uint32_t cd2[BS];              // candidates of the current chunk, by thread: d2 bits,
    uint16_t cnext[BS];            //   next candidate of the same slot (kNil: end),
    uint16_t cdg[BS];              //   own child slab | (grandchild slab + 1) << 5
    uint32_t gcnt[kDests * kDests / 2];   // 16 bits each, folded into registers every 32 steps
    uint32_t dcur[2][kDests];      // emissions per child slab before chunk c: dcur[c & 1]
    alignas(16) uint32_t wcnt[kDests][NW / 4];   // emissions per child slab and wave, one byte per wave (<= 64)
    uint32_t nwin, err;
    uint32_t fj;                   // NaN points in the slot (0, 0) outside the table: the first one's arrival index
    uint32_t nanc[2];              // per chunk parity: a NaN-distance candidate pushed (the walk's NaN rules apply)
};
static_assert(sizeof(DenseLds) <= 163840, "the dense slab kernel's LDS");

__device__ __forceinline__ uint32_t hash_slot(uint32_t k) { return (k * 2654435761u) >> 15; }

// Per-chunk claim table keyed by slot: entry = (slot << 11) | min pending thread
// (0x7FF once that thread has been applied).  Slots < 2^14, threads < 2^10.
constexpr uint32_t kClaimDone = 0x7FFu;
// Claim table of CLAIM entries (a power of two), linear probing from the
// multiplicative hash's middle bits.  CAS first: an empty entry (the common
// case) costs one LDS round trip.
template <int CLAIM>
__device__ __forceinline__ int claim_insert(uint32_t* H, uint32_t local, uint32_t tid) {
    static_assert((CLAIM & (CLAIM - 1)) == 0, "claim table: a power of two");
    const uint32_t mine = (local << 11) | tid;
    uint32_t h = hash_slot(local) & (CLAIM - 1);
    for (int probe = 0; probe < CLAIM; probe++) {
        const uint32_t e = atomicCAS(&H[h], kEmpty32, mine);
        if (e == kEmpty32) return (int)h;
        if ((e >> 11) == local) {
            atomicMin(&H[h], mine);
            return (int)h;
        }
        h = (h + 1) & (CLAIM - 1);
    }
    return -1;
}

// end of a dense slab's per-slot candidate list (k_slab)
constexpr uint32_t kNil = 0x7FFu;
// a NaN distance in the candidate list: never less than another (cell.rs:77-80)
constexpr uint32_t kNanKey = 0x7FFFFFFFu;
// The slot key of a foreign slot in the hashed tables of the small-slab
// kernels: a NaN x or y maps to offset slot (0, 0), outside the cell's slot
// range unless the cell touches the origin (k_slab's "foreign" slots); above
// every slot of a dim-96 layer, below the wave kernel's reserved 0x3FFF.
constexpr uint32_t kForeignSlot = 0x3FFEu;
static_assert(kDenseTab < (int)kForeignSlot, "foreign slot key above the table");
// the table key of a distance: a NaN point that takes an empty slot keeps it
// (nothing compares less than it, cell.rs:77-80), i.e. key 0
__device__ __forceinline__ uint32_t dist_key(float d2) { return d2 == d2 ? f2u(d2) : 0u; }


// Slot-table entry: (d2 bits << 33) | (dest << 28) | ((g + 1) << 23) | j.  d2 >= +0
// so its sign bit is free; dest (0..23) and g (grandchild slab inside dest, -1
// none) route a displaced occupant without its payload; j < 2^23 indexes the
// slab's arrivals.  Slabs of 2^23 arrivals or more ("wide") use j < 2^28 in
// place of g and recompute a displaced occupant's g from its gathered payload.
constexpr uint32_t kJBits = 28;
constexpr uint32_t kJMask = (1u << kJBits) - 1;
constexpr uint32_t kJMaskNarrow = (1u << 23) - 1;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ void bst4(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

// A dense slab's arrivals.  Merge mode (SEEDS): arrivals 0 .. ns-1 are the
// slab's seeds, read in place from the seed array (the room reserved for them
// in front of the emissions is never written); every load is issued to both
// sources with the other one out of range (a buffer load out of range returns
// 0), so no lane branches.  Offsets are byte offsets (16 j / 4 j) or ~0u.
template <bool SEEDS>
struct ArrSrc {
    __amdgpu_buffer_rsrc_t rP, rK, rS, rT;
    uint32_t ns16;   // 16 * ns
    __device__ __forceinline__ u32x4 p(uint32_t o) const {
        if constexpr (!SEEDS) {
            return bld4(rP, o);
        } else {
            const bool sd = o < ns16;
            const u32x4 a = bld4(rS, sd ? o : 0xFFFFFFFFu), b = bld4(rP, sd ? 0xFFFFFFFFu : o);
            return u32x4{a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w};
        }
    }
    __device__ __forceinline__ uint32_t k(uint32_t o) const {
        if constexpr (!SEEDS) {
            return bld(rK, o);
        } else {
            const bool sd = o < ns16 / 4;
            return bld(rT, sd ? o : 0xFFFFFFFFu) | bld(rK, sd ? 0xFFFFFFFFu : o);
        }
    }
};

// Grid points of a dense slab: the slot table's occupants, compacted into the
// slab's grid region (cell.rs:158-160: order inside a cell file is free).
#ifdef PCC_STAMPS
#define GSTAMP(ph) do { const unsigned long long st_n = __builtin_amdgcn_s_memtime(); st_acc[ph] += st_n - st_t0; st_t0 = st_n; } while (0)
#else
#define GSTAMP(ph) do {} while (0)
#endif
template <bool NF, class L, class SRC>
__device__ __forceinline__ void dense_grid_points(const SlabParams& P, L& S, uint32_t* bm, const SRC& rP,
                                                  uint32_t s, uint32_t n, uint32_t jmask, uint32_t tid, uint32_t lane,
                                                  unsigned long long* st_acc, unsigned long long& st_t0) {
    constexpr int BS = L::BS, TAB = L::TAB;
    // ---- grid points: the table's occupants, compacted into the slab's grid
    // region (cell.rs:158-160: order inside a cell file is free).
    constexpr int U = (TAB + BS - 1) / BS;
    const uint64_t lt = lanemask_lt();
    const __amdgpu_buffer_rsrc_t rG = srd(P.grid + P.grid_off[s], (uint64_t)n * 16);
    if (n <= kDenseStreamMax) {
        // Small slab: clear the winners' bits in a bitmap over the arrivals (bm:
        // the head words, all ones after the last step), then stream the arrivals
        // once in order, coalesced, instead of gathering the winners.  The first
        // V chunks are loaded before the table scan and stay in flight across
        // the LDS-only barrier.
        constexpr int V = PCC_STREAM_V;
        u32x4 pv[V];
#pragma unroll
        for (int u = 0; u < V; u++) pv[u] = rP.p((u * BS + tid) * 16);   // past n: zero (buffer range)
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = u * BS + (int)tid;
            const unsigned long long occ = i < TAB ? S.tab[i] : kEmpty64;
            if (occ != kEmpty64) {
                const uint32_t jw = (uint32_t)occ & jmask;
                atomicAnd(&bm[jw >> 5], ~(1u << (jw & 31u)));
            }
        }
        if constexpr (NF)   // a foreign slot's point
            if (tid == 0 && S.fj != kEmpty32) atomicAnd(&bm[S.fj >> 5], ~(1u << (S.fj & 31u)));
        GSTAMP(14);
        lds_barrier();
        GSTAMP(15);
        for (uint32_t j0 = 0; j0 < n; j0 += V * BS) {
            if (j0) {
#pragma unroll
                for (int u = 0; u < V; u++) pv[u] = rP.p((j0 + u * BS + tid) * 16);
            }
            uint64_t m[V];
            uint32_t tot = 0;
#pragma unroll
            for (int u = 0; u < V; u++) {
                const uint32_t jj = j0 + u * BS + tid;
                m[u] = __ballot(jj < n && !((bm[jj >> 5] >> (jj & 31u)) & 1u));
                tot += (uint32_t)__popcll(m[u]);
            }
            uint32_t wb = 0;
            if (lane == 0 && tot) wb = atomicAdd(&S.nwin, tot);
            wb = __shfl(wb, 0, 64);
#pragma unroll
            for (int u = 0; u < V; u++) {
                const bool win = (m[u] >> lane) & 1ull;
                bst4(rG, win ? (wb + (uint32_t)__popcll(m[u] & lt)) * 16 : 0xFFFFFFFFu, pv[u]);
                wb += (uint32_t)__popcll(m[u]);
            }
        }
    } else {
        // Large slab: gather the winners' payloads, U loads in flight per thread,
        // one LDS atomic per wave for the positions.
        uint32_t wpos[U], src[U];
        uint64_t m[U];
        uint32_t tot = 0;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = u * BS + (int)tid;
            const unsigned long long occ = i < TAB ? S.tab[i] : kEmpty64;
            const bool win = occ != kEmpty64;
            m[u] = __ballot(win);
            tot += (uint32_t)__popcll(m[u]);
            src[u] = win ? ((uint32_t)occ & jmask) * 16 : 0xFFFFFFFFu;
        }
        uint32_t wb = 0;
        if (lane == 0 && tot) wb = atomicAdd(&S.nwin, tot);
        wb = __shfl(wb, 0, 64);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const bool win = (m[u] >> lane) & 1ull;
            wpos[u] = win ? (wb + (uint32_t)__popcll(m[u] & lt)) * 16 : 0xFFFFFFFFu;
            wb += (uint32_t)__popcll(m[u]);
        }
        GSTAMP(14);
        u32x4 pv[U];
#pragma unroll
        for (int u = 0; u < U; u++) pv[u] = rP.p(src[u]);
#ifdef PCC_STAMPS
        if (pv[U - 1].x == 0x7FC00001u) S.err = 1u << 28;   // the stamp below waits for the gathers
        GSTAMP(15);
#endif
#pragma unroll
        for (int u = 0; u < U; u++) bst4(rG, wpos[u], pv[u]);
        if constexpr (NF) {
            if (tid == 0 && S.fj != kEmpty32) {   // the point holding a foreign slot (NaN coordinates)
                const uint32_t wf = atomicAdd(&S.nwin, 1u);
                bst4(rG, wf * 16, rP.p(S.fj * 16));
            }
        }
    }
}

// One pass over the slab in key order (cell.rs:70-94), one chunk of BS arrivals
// per step and exactly two barriers per step:
//   phase A : slot / d2 / routes of chunk i.  An arrival that does not beat its
//             slot's occupant overflows at once (occupants only improve); the
//             others (candidates) push themselves onto their slot's list.  Wave
//             ranks of chunk i-1's emissions per child slab.
//   barrier
//   phase B : chunk i-1's emissions are stored (positions from per-wave prefixes
//             of the wave counts).  Every candidate walks its slot's list: it is
//             a record iff no earlier candidate has d2 <= its own; a record is
//             the new occupant iff no later candidate has a smaller d2, and it
//             emits, at its own key, the record before it (the earlier
//             candidate with the least (d2, key)) or, if it is the first record,
//             the slot's previous occupant.  Everything else overflows at its key.
//   barrier
// The payload of a displaced record is gathered from the slab's arrivals and
// stored one step later with the rest of the chunk's emissions.  After the last
// chunk the table's occupants are the slab's grid points (cell.rs:158-160:
// order inside a cell file is free).  Grandchild capacities count every
// emission's (child, grandchild) slab when its rank is taken.
// NF: the input has NaN coordinates (the NaN rules below; Engine::nf_mode_).
// KF: a merge level with forced emissions (kept seeds, P.kf_n > 0).
// WIDEOK: a slab of the launch may have 2^23 arrivals or more ("wide"); false
// compiles the wide paths out of the common launch.
template <bool SEEDS, bool NF, bool KF, bool WIDEOK = true>
__global__ __launch_bounds__(kDenseBS) void k_slab(SlabParams P) {
    using L = DenseLds;
    constexpr int BS = L::BS, TAB = L::TAB, NW = L::NW;
    __shared__ L S;
    STAMP_DECL
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid / 64);   // (an SGPR)
    const SmallDesc D = P.ddesc[blockIdx.x];
    const uint32_t s = D.s;
    const int32_t t = D.t;
    const uint32_t off = D.off, n = D.n, nm1 = n - 1;
    const int32_t cx = D.cx, cy = D.cy, cz = D.cz;
    const LevelGeo& G = P.G;
    if (n > kJMask) {   // the entry packs j in 28 bits
        if (tid == 0) set_err(P.ctr, ERR_SLAB_SIZE);
        return;
    }
    const bool wide = WIDEOK && n > kJMaskNarrow;
    if (!WIDEOK && n > kJMaskNarrow) {   // (the host launches WIDEOK for such a level)
        if (tid == 0) set_err(P.ctr, ERR_SLAB_SIZE);
        return;
    }
    const uint32_t wide_u = __builtin_amdgcn_readfirstlane(wide ? 1u : 0u);   // (an SGPR: uniform branches)
    const uint32_t jmask = wide ? kJMask : kJMaskNarrow;
    // merge: the first ng arrivals are the slab's grid seeds (below)
    const uint32_t ng = SEEDS ? min(D.ng, n) : 0u;
    // reference slot: the one holding the cell centre (metadata.rs:104-106)
    const I3 c0 = hex_from_world(cell_pos1(cx, P.cs), cell_pos1(cy, P.cs), cell_pos1(cz, P.cs), G.cr);
    const int32_t rx = c0.x - P.tx / 2, ry = c0.y - P.ty / 2;
    const SlabCtx SC{cx, cy, cz, t};
    const float zt = (float)t * G.cr;   // slot centre z of the slab's layer (hex.rs:63)
    uint32_t err = 0;
    // buffer descriptors: this slab's arrivals and the contiguous region of its
    // 24 child slabs in the next arena (out-of-range offsets drop a store)
    const uint64_t nb = (uint64_t)n * 4;
    ArrSrc<SEEDS> A_;
    A_.rP = srd(P.in.p + off, nb * 4);
    A_.rK = srd(P.in.k + off, nb);
    if constexpr (SEEDS) {
        A_.rS = srd(P.inj + D.pad0, (uint64_t)D.pad1 * 16);
        A_.rT = srd(P.inj_keys + D.pad0, (uint64_t)D.pad1 * 4);
        A_.ns16 = D.pad1 * 16;
    } else {
        A_.rS = A_.rP;
        A_.rT = A_.rK;
        A_.ns16 = 0;
    }
    const ArrSrc<SEEDS>& rP = A_;
    const uint32_t dbase = D.dbase;
    const uint64_t db = (uint64_t)D.dlen * 4;
    const __amdgpu_buffer_rsrc_t oP = srd(P.nx.p + dbase, db * 4), oK = srd(P.nx.k + dbase, db);
    // child-slab regions of this slab, one per lane < 24, kept in registers:
    // unconditional buffer loads (lanes >= 24 read 0) issued before the first
    // chunks', so the prologue never waits for them (dbase is subtracted at use)
    const __amdgpu_buffer_rsrc_t rDo = srd(P.dest_off + (uint64_t)s * kDests, kDests * 4),
                                 rDc = srd(P.dcap + (uint64_t)s * kDests, kDests * 4);
    uint32_t my_doff = bld(rDo, lane < kDests ? lane * 4 : 0xFFFFFFFFu);
    uint32_t my_dcap = bld(rDc, lane < kDests ? lane * 4 : 0xFFFFFFFFu);

    // Slot of an arrival: computed one step ahead, in the phase B before the
    // step that replays it (software pipelining: the arithmetic of chunk i+1
    // fills the LDS latency chains of chunk i's emissions and list walks).
    struct SlotInfo {
        uint32_t local;   // slot table index (0 when not slotted)
        float d2;         // distance to the slot centre
        uint32_t dn;      // own child slab
        int32_t gn;       // own grandchild slab
        bool slotted;     // valid, layer and range ok
        bool isn;         // NF: NaN distance
        bool foreign;     // NF: NaN slot outside the table
    };
    struct Stage {
        int32_t em;     // -1 none, 0 self, 1 displaced record / occupant
        uint32_t d;     // child slab of the emitted point
        int32_t g;      // its grandchild slab (-1 none, -2 unknown: wide slab, from gp)
        u32x4 gp;       // gathered payload of a displaced point
        SlotInfo si;    // slot of this stage's chunk (written one step before its replay)
    };
    Stage A;
    A.em = -1; A.d = 0; A.g = -1;
    A.gp = u32x4{0u, 0u, 0u, 0u};
    A.si.local = 0; A.si.d2 = 0.0f; A.si.dn = 0; A.si.gn = -1;
    A.si.slotted = A.si.isn = A.si.foreign = false;
    Stage B = A;
    // Arrivals are prefetched two chunks ahead into a ring of four register
    // buffers: chunk i lives in buf[i % 4] from its load (step i-2) to its
    // emission store (step i+1), so no loaded register is ever copied (a copy
    // would wait for the load, and vmcnt also counts the stores issued since).
    struct Pre { u32x4 p; uint32_t k; };
    constexpr int PF = PCC_SLAB_PF;   // chunks loaded ahead; the ring holds PF + 2
    Pre pre[PF + 2];
#pragma unroll
    for (int q = 0; q < PF + 2; q++) {
        const uint32_t jo = min(ng + (uint32_t)(q * BS) + tid, nm1);
        if (q < PF) {
            pre[q].p = rP.p(jo * 16);
            pre[q].k = rP.k(jo * 4);
        } else {
            pre[q].p = u32x4{0u, 0u, 0u, 0u};
            pre[q].k = 0;
        }
    }
    // merge: the first seed records (below) are loaded before the LDS
    // initialisation too
    constexpr int SQ = 4;
    const __amdgpu_buffer_rsrc_t rR = srd(P.inj_rec + D.pad0, SEEDS ? (uint64_t)ng * 8 : 0ull);
    uint32_t rl[SQ], rh[SQ];
    auto seed_batch = [&](uint32_t j0) {
#pragma unroll
        for (int k = 0; k < SQ; k++) {
            const uint32_t jg = j0 + k * BS + tid;
            const bool v = jg < ng;
            rl[k] = bld(rR, v ? jg * 8 : 0xFFFFFFFFu);
            rh[k] = bld(rR, v ? jg * 8 + 4 : 0xFFFFFFFFu);
        }
    };
    if constexpr (SEEDS) seed_batch(0);
    // the LDS initialisation overlaps the first two chunks' loads
    for (int i = tid; i < TAB; i += BS) S.tab[i] = kEmpty64;
    for (int i = tid; i < L::HW; i += BS) S.head[i] = kEmpty32;   // tag 31, head kNil
    for (int i = tid; i < kDests * kDests / 2; i += BS) S.gcnt[i] = 0;
    uint32_t gacc0 = 0, gacc1 = 0;   // thread t < 288: counts of (child, grandchild) pairs 2t, 2t + 1
    if (tid < kDests) {
        S.dcur[0][tid] = 0;
        S.dcur[1][tid] = 0;
    }
    if (tid == 0) { S.nwin = 0; S.err = 0; S.fj = kEmpty32; S.nanc[0] = S.nanc[1] = 0; }
    lds_barrier();   // LDS only: the first chunks' loads stay in flight
    if constexpr (SEEDS) {
        // Merge: the slab's grid seeds (its first ng arrivals: keys below every
        // other arrival, one per slot, cell.rs:183-229) are the occupants the
        // replay would install, with no emission; they go straight into the table.
        // a seed whose record (k_seed_rec) is flagged: its slot and route again,
        // with the error codes (never expected)
        auto seed_exact = [&](uint32_t jg) {
            const bool v = jg < ng;
            const u32x4 q = rP.p(v ? jg * 16 : 0xFFFFFFFFu);
            const float x = __uint_as_float(q.x), y = __uint_as_float(q.y), z = __uint_as_float(q.z);
            const SlotDest sd = slot_dest(x, y, z, G, SC);
            const int32_t lx = sd.ox - rx, ly = sd.oy - ry;
            const bool layer_ok = sd.layer_ok;
            const bool range_ok = lx >= 0 && ly >= 0 && lx < P.tx && ly < P.ty;
            const bool slotted = v && layer_ok && range_ok;
            float X, Y, Z;
            slot_centre(sd, G.cr, zt, X, Y, Z);
            const float d2 = dist2(X, Y, Z, x, y, z);
            const int d = sd.d;
            int32_t gn = sd.g;
            // a NaN grid seed in the foreign slot (0, 0) outside the table holds it
            const bool foreign = NF && v && layer_ok && !range_ok && d2 != d2;
            if constexpr (NF)
                if (foreign) atomicMin(&S.fj, jg);
            const bool bad = v && (!layer_ok || (!range_ok && !foreign) || d < 0 || (P.check_gchild && gn < 0));
            if (__ballot(bad)) {
                if (bad) err |= slot_route_errs(slot_route(x, y, z, G), layer_ok, range_ok, cx, cy, cz, t, P.check_gchild);
            }
            const uint32_t dn = d < 0 ? 0u : (uint32_t)d;
            if (slotted) {
                const unsigned long long e = ((unsigned long long)dist_key(d2) << 33) | ((unsigned long long)dn << kJBits) |
                                             (wide ? 0u : ((uint32_t)(gn + 1) << 23)) | jg;
                // two grid points in one slot: not a cell a converter writes
                if (atomicCAS(&S.tab[(uint32_t)(ly * P.tx + lx)], kEmpty64, e) != kEmpty64) err |= ERR_CLAIM;
            }
        };
        // the seeds' precomputed records, four chunks of loads in flight: one
        // LDS CAS per seed
        for (uint32_t j0 = 0; j0 < ng; j0 += SQ * BS) {
            if (j0) seed_batch(j0);
            bool flagged = false;
#pragma unroll
            for (int k = 0; k < SQ; k++) flagged |= (j0 + k * BS + tid < ng) && (rh[k] >> 31);
            if (__ballot(flagged)) {
#pragma unroll 1
                for (int k = 0; k < SQ; k++) seed_exact(j0 + k * BS + tid);
                continue;
            }
#pragma unroll
            for (int k = 0; k < SQ; k++) {
                const uint32_t jg = j0 + k * BS + tid;
                if (jg < ng) {
                    const uint32_t local = rh[k] & 0x3FFFu, dn = (rh[k] >> 14) & 31u, g1 = (rh[k] >> 19) & 31u;
                    const unsigned long long e = ((unsigned long long)rl[k] << 33) | ((unsigned long long)dn << kJBits) |
                                                 (wide ? 0u : (g1 << 23)) | jg;
                    if (atomicCAS(&S.tab[local], kEmpty64, e) != kEmpty64) err |= ERR_CLAIM;
                }
            }
        }
        __syncthreads();
    }
    const uint32_t nchunks = (n - ng + BS - 1) / BS;
    // Slot, distance (hex.rs:67-85, 55-65) and own child / grandchild slab of
    // chunk ci's arrival of this thread (payload c): everything of phase A that
    // does not read the table.  Error codes only on the (never expected) failing
    // lanes.  A NaN coordinate gives a NaN distance, which never compares less
    // (cell.rs:77-80), and a NaN x or y gives the slot (0, 0) (hex.rs:67-85, NaN
    // `as i32` = 0), which can lie outside this cell's table: a "foreign" slot
    // only NaN points reach, so its first arrival is the grid point and every
    // later one overflows (S.fj: the least such arrival; a min, so it may be
    // taken one step early).
    auto slot_info = [&](uint32_t ci, const Pre& c, SlotInfo& o) {
        const uint32_t j = ng + ci * BS + tid;
        const bool valid = j < n;
        const float x = __uint_as_float(c.p.x), y = __uint_as_float(c.p.y), z = __uint_as_float(c.p.z);
        bool amb = false;
        SlotDest sd = slot_dest_fast(x, y, z, G, SC, amb);
        if (__ballot(amb)) {
            if (amb) slot_dest_exact(x, y, z, G, SC, sd);
        }
        const int32_t lx = sd.ox - rx, ly = sd.oy - ry;
        const bool range_ok = (lx >= 0) & (ly >= 0) & (lx < P.tx) & (ly < P.ty);
        const bool layer_ok = sd.layer_ok;
        o.slotted = valid & layer_ok & range_ok;
        o.local = o.slotted ? (uint32_t)(ly * P.tx + lx) : 0u;
        float X, Y, Z;
        slot_centre(sd, G.cr, zt, X, Y, Z);
        o.d2 = dist2(X, Y, Z, x, y, z);
        o.isn = NF && o.d2 != o.d2;
        o.foreign = false;
        if constexpr (NF) {
            if (__ballot(o.isn && valid && layer_ok && !range_ok)) {
                o.foreign = o.isn && valid && layer_ok && !range_ok;
                const bool forced = KF && valid && c.k - P.kf_lo < P.kf_n;
                if (o.foreign && !forced) atomicMin(&S.fj, j);
            }
        }
        const int d = sd.d;
        o.gn = sd.g;
        const bool bad = valid & (!layer_ok | (!range_ok & !o.foreign) | (d < 0) | ((P.check_gchild != 0) & (o.gn < 0)));
        if (__ballot(bad)) {
            if (bad) err |= slot_route_errs(slot_route(x, y, z, G), layer_ok, range_ok, cx, cy, cz, t, P.check_gchild);
        }
        o.dn = d < 0 ? 0u : (uint32_t)d;
    };
    if (nchunks) slot_info(0, pre[0], A.si);
    STAMP(0);
    auto step = [&](uint32_t ci, Stage& cur, Stage& prv, const Pre& mine, const Pre& prvb, const Pre& nxt, Pre& pf) {
        const uint32_t par = ci & 1;
        const uint32_t tag = ci & 31u;
        const uint32_t j = ng + ci * BS + tid;
        const bool valid = j < n;
        const bool forced = KF && (valid & (mine.k - P.kf_lo < P.kf_n));
        {   // prefetch chunk i+2 (clamped)
            const uint32_t jo = min(j + PF * BS, nm1);
            pf.p = rP.p(jo * 16);
            pf.k = rP.k(jo * 4);
        }
        // ---- phase A (1): the slot's occupant and list head (the slot itself
        // was computed in the last phase B; phase B of the last step wrote the
        // table before the barrier; local 0 for lanes without a slot)
        const uint32_t local = cur.si.local;
        const bool slotted = cur.si.slotted;
        unsigned long long occ = S.tab[local];
        uint32_t hw = S.head[local >> 1];   // the slot's head word, read with the occupant
        // the last step pushes and walks nothing: the head words become the
        // winner bitmap over the arrivals (all ones; dense_grid_points).  A
        // uniform branch and one clamped store per thread (n <= kDenseStreamMax:
        // at most BS words), so no exec-mask region.
        static_assert((kDenseStreamMax + 31) / 32 <= (uint32_t)BS, "one bitmap word per thread");
        if (ci == nchunks && n <= kDenseStreamMax) S.head[min(tid, (n + 31) / 32 - 1)] = kEmpty32;
        const float d2 = cur.si.d2;
        const bool isn = cur.si.isn, foreign = cur.si.foreign;
        const uint32_t dn = cur.si.dn;
        const int32_t gn = cur.si.gn;
#ifdef PCC_STAMPS
        if (d2 == 12345.0f) err |= 1u << 29;
        STAMP(13);
#endif
        // Occupant filter (cell.rs:80 strict <: ties keep the old point); the
        // candidates push themselves onto their slot's list.
        bool cand = false;
        uint32_t myprev = kNil;
        if (slotted & !forced) {
            cand = (occ == kEmpty64) | (d2 < __uint_as_float((uint32_t)(occ >> 33)));
        } else {
            occ = kEmpty64;
        }
        if constexpr (NF) {
            if (cand && isn) S.nanc[par] = 1u;
            if (tid == 0) S.nanc[par ^ 1u] = 0u;   // the other parity's flag (read before the last barrier)
        }
        const uint32_t sh = (local & 1u) * 16u;
        if (cand) {
            // push onto the slot's list: swap this thread into the head's half of
            // the word (a CAS retried while other pushes change the word); the
            // old head belongs to this chunk only if its tag is this chunk's
            const uint32_t mineh = (tag << 11) | tid;
            for (;;) {
                const uint32_t o = atomicCAS(&S.head[local >> 1], hw, (hw & ~(0xFFFFu << sh)) | (mineh << sh));
                if (o == hw) break;
                hw = o;
            }
            const uint32_t oldh = (hw >> sh) & 0xFFFFu;
            myprev = (oldh >> 11) == tag ? (oldh & kNil) : kNil;
            S.cd2[tid] = isn ? kNanKey : f2u(d2);
            S.cnext[tid] = (uint16_t)myprev;
            S.cdg[tid] = (uint16_t)(dn | ((uint32_t)(gn + 1) << 5));
        }
        STAMP(1);
#ifdef PCC_XVALU
        // Diagnostic (issue-bound test): PCC_XVALU independent VALU per step in
        // four chains, half here and half in phase B, feeding err.
        uint32_t xv0 = j, xv1 = j ^ 1u, xv2 = j ^ 2u, xv3 = j ^ 3u;
#pragma unroll
        for (int xq = 0; xq < PCC_XVALU / 8; xq++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv0) : "v"(tid));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv1) : "v"(tid));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv2) : "v"(tid));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv3) : "v"(tid));
        }
#endif
        // ---- phase A (2): wave ranks of chunk i-1's emissions per child slab
        const bool vd = prv.em >= 0;
        const int d = vd ? (int)prv.d : 0;
        const uint64_t same = wave_peers<5>((uint32_t)d, vd);
        const uint32_t rw = mask_rank(same);
        if (lane < kDests) reinterpret_cast<uint8_t*>(S.wcnt[lane])[wv] = 0;
        if (vd & (rw == 0)) reinterpret_cast<uint8_t*>(S.wcnt[d])[wv] = (uint8_t)__popcll(same);
        // grandchild capacities: one LDS add per emission
        {
            int32_t gg = prv.g;
            if (wide_u) {   // block-uniform; a displaced occupant of a wide slab: route its payload
                if (vd && gg == -2)
                    gg = slot_dest(__uint_as_float(prv.gp.x), __uint_as_float(prv.gp.y), __uint_as_float(prv.gp.z), G,
                                   SC).g;
            }
            if (vd & (gg >= 0)) {
                const uint32_t gi = (uint32_t)(d * kDests + gg);
                atomicAdd(&S.gcnt[gi >> 1], (gi & 1u) ? 0x10000u : 1u);
            }
        }
        STAMP(2);
        lds_barrier();
        STAMP(3);
        // between the barriers nothing pushes or counts: every 16 steps, heads of
        // older chunks go back to kNil (tags are 5 bits), and every 32 steps the
        // 16-bit pair counts move into registers (at most 32 768 adds between)
        if ((ci & 15u) == 15u) {
            for (int i = tid; i < L::HW; i += BS) {
                const uint32_t w = S.head[i];
                const uint32_t lo = ((w >> 11) & 31u) == tag ? (w & 0xFFFFu) : 0xFFFFu;
                const uint32_t hi = (w >> 27) == tag ? (w >> 16) : 0xFFFFu;
                if ((lo | (hi << 16)) != w) S.head[i] = lo | (hi << 16);
            }
        }
        if ((ci & 31u) == 31u && tid < kDests * kDests / 2) {
            const uint32_t w = S.gcnt[tid];
            gacc0 += w & 0xFFFFu;
            gacc1 += w >> 16;
            S.gcnt[tid] = 0;
        }
        // ---- phase B (1): chunk i-1's emissions.  Position = emissions to the
        // same child slab before the chunk + in earlier waves + earlier lanes.
        {
            const uint32_t rp = par ^ 1;   // chunk i-1's parity
            // byte sums of the wave counts: earlier waves, all waves.  Every lane
            // reads (lanes >= 24 a copy of lane 0's row), so the reads are issued
            // before the next chunk's slot arithmetic, which hides their latency.
            const uint32_t ll = lane < kDests ? lane : 0u;
            uint32_t pre_l = S.dcur[rp][ll];
            uint32_t w[NW / 4];
            if constexpr (NW == 16) {
                const u32x4 w4 = *reinterpret_cast<const u32x4*>(S.wcnt[ll]);
                w[0] = w4.x; w[1] = w4.y; w[2] = w4.z; w[3] = w4.w;
            } else {
#pragma unroll
                for (int k = 0; k < NW / 4; k++) w[k] = S.wcnt[ll][k];
            }
            // ---- the next chunk's slots (into the stage of chunk i-1, whose slot
            // is dead; its emission fields are read below)
            if (ci + 1 < nchunks) {   // block-uniform
                slot_info(ci + 1, nxt, prv.si);
            } else {
                prv.si.local = 0; prv.si.d2 = 0.0f; prv.si.dn = 0; prv.si.gn = -1;
                prv.si.slotted = prv.si.isn = prv.si.foreign = false;
            }
            uint32_t tot_l = pre_l;
#pragma unroll
            for (uint32_t k = 0; k < (uint32_t)NW / 4; k++) {
                const uint32_t nb = wv > 4 * k ? min(wv - 4 * k, 4u) : 0u;   // wave-uniform
                const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
                pre_l = __builtin_amdgcn_udot4(w[k] & m, 0x01010101u, pre_l, false);
                tot_l = __builtin_amdgcn_udot4(w[k], 0x01010101u, tot_l, false);
            }
            if (wv == 0 && lane < kDests) S.dcur[par][lane] = tot_l;
            asm volatile("" : "+v"(my_doff));                   // keeps the load's wait out of the prologue
            const uint32_t base_l = my_doff - dbase + pre_l;    // this wave's first position in child slab `lane`
            const int32_t room_l = (int32_t)(my_dcap - pre_l);  // and the capacity left from there
            // both shuffles with every lane active (a bpermute from an inactive
            // lane reads nothing)
            const uint32_t pos = (uint32_t)__shfl((int)base_l, d, 64) + rw;
            const int32_t room = __shfl(room_l, d, 64);
            const bool ok = vd & ((int32_t)rw < room);
            if (__ballot(vd & !ok)) err |= ERR_CAPACITY;
            bst4(oP, ok ? pos * 16 : 0xFFFFFFFFu, prv.em == 1 ? prv.gp : prvb.p);
            bst(oK, ok ? pos * 4 : 0xFFFFFFFFu, prvb.k);
            STAMP(6);
        }
        // ---- phase B (2): records of chunk i (walk of the slot's candidate list)
        int32_t em = (slotted & !cand & (forced | (occ != kEmpty64))) ? 0 : -1;
        if constexpr (NF) {
            if (__ballot(foreign)) {   // a foreign slot: the first NaN point holds it, the others overflow
                if (foreign && S.fj != j) em = 0;
            }
        }
        // The decisions after the walk are selects (vsel: each divergent `if`
        // costs the wave exec-mask SALU, and the scalar unit is shared by the
        // CU's 16 waves); the LDS accesses stay on the lanes that need them.
        const uint32_t me = f2u(d2);   // d2 >= +0: the bit patterns order like the values
        // earliest least earlier candidate (the record before this one, if this
        // one is a record) and whether a later candidate beats this one
        uint32_t bd = 0xFFFFFFFFu, bt = kNil;
        bool beaten = false;
        // the own entry is skipped (known without LDS reads).  (Both arms of
        // every select below are computed first: a conditional operator whose
        // arm is more than a couple of instructions stays a branch.)
        uint32_t xk = kNil;
        if (cand) {
            xk = (S.head[local >> 1] >> sh) & kNil;
            xk = xk == tid ? myprev : xk;
        }
        uint32_t meff = me;
        if (!NF || !S.nanc[par]) {
            while (xk != kNil) {
                const uint32_t dx = S.cd2[xk];
                const uint32_t nx = S.cnext[xk];
                const bool earlier = xk < tid;
                const bool better = earlier & ((dx < bd) | ((dx == bd) & (xk < bt)));
                bd = better ? dx : bd;
                bt = better ? xk : bt;
                beaten |= !earlier & (dx < me);
                xk = nx == tid ? myprev : nx;
            }
        } else {
            // A NaN-distance candidate (the slot was empty) holds the slot iff it
            // is the earliest candidate; then nothing displaces it (key 0).  Any
            // other NaN candidate overflows (key kNanKey: never less).
            uint32_t mt = kNil;   // the earliest earlier candidate
            while (xk != kNil) {
                const uint32_t dx = S.cd2[xk];
                const uint32_t nx = S.cnext[xk];
                const bool earlier = xk < tid;
                const bool better = earlier && (dx < bd || (dx == bd && xk < bt));
                bd = better ? dx : bd;
                bt = better ? xk : bt;
                beaten |= !earlier && dx < me;
                mt = earlier && xk < mt ? xk : mt;
                xk = nx == tid ? myprev : nx;
            }
            if (cand) {
                if (mt != kNil && S.cd2[mt] == kNanKey) { bd = 0u; bt = mt; }
                if (isn) {
                    meff = bt == kNil ? 0u : kNanKey;
                    beaten = false;
                }
            }
        }
        const bool hasbt = bt != kNil;
        const bool notrec = hasbt & !(meff < bd);   // not a record: overflows at its key
        const bool rec = cand & !notrec;
        uint32_t dg = S.cdg[hasbt ? bt : tid];  // the record before this one (displaced)
        asm volatile("" : "+v"(dg));            // (not sunk into a branch of its use)
        const bool dprev = rec & hasbt, docc = rec & !hasbt & (occ != kEmpty64);
        const int32_t em_c = notrec ? 0 : ((dprev | docc) ? 1 : -1);
        em = cand ? em_c : em;
        const uint32_t d_prev = dg & 31u, d_occ = (uint32_t)(occ >> kJBits) & 31u;
        const int32_t g_prev = (int32_t)(dg >> 5) - 1, g_occ = (int32_t)(((uint32_t)occ >> 23) & 31u) - 1;
        const int32_t g_occw = wide ? -2 : g_occ;
        const uint32_t emd = vsel(dprev, d_prev, vsel(docc, d_occ, dn));
        const int32_t emg = vsel(dprev, g_prev, vsel(docc, g_occw, gn));
        // byte offset of a displaced point's payload
        const uint32_t s_prev = (ng + ci * BS + bt) * 16, s_occ = ((uint32_t)occ & jmask) * 16;
        const uint32_t gsrc = vsel(dprev, s_prev, vsel(docc, s_occ, 0xFFFFFFFFu));
        // the last record is the new occupant
        const uint32_t gbits = wide ? 0u : ((uint32_t)(gn + 1) << 23);
        const unsigned long long ent = ((unsigned long long)meff << 33) | ((unsigned long long)dn << kJBits) | gbits | j;
        if (rec & !beaten) S.tab[local] = ent;
#ifdef PCC_XVALU
#pragma unroll
        for (int xq = 0; xq < PCC_XVALU / 8; xq++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv0) : "v"(tid));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv1) : "v"(tid));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv2) : "v"(tid));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(xv3) : "v"(tid));
        }
        if ((xv0 ^ xv1 ^ xv2 ^ xv3) == 0x9E3779B9u) err |= 1u << 27;
#endif
#ifdef PCC_XSALU
        {   // Diagnostic: PCC_XSALU independent SALU per step in four chains
            uint32_t xs0 = ci, xs1 = ci ^ 1u, xs2 = ci ^ 2u, xs3 = ci ^ 3u;
#pragma unroll
            for (int xq = 0; xq < PCC_XSALU / 4; xq++) {
                asm volatile("s_add_u32 %0, %0, 0x9e37" : "+s"(xs0) : : "scc");
                asm volatile("s_add_u32 %0, %0, 0x79b9" : "+s"(xs1) : : "scc");
                asm volatile("s_add_u32 %0, %0, 0x3c6e" : "+s"(xs2) : : "scc");
                asm volatile("s_add_u32 %0, %0, 0xf1bb" : "+s"(xs3) : : "scc");
            }
            if ((xs0 ^ xs1 ^ xs2 ^ xs3) == 0x9E3779B9u) err |= 1u << 26;
        }
#endif
        STAMP(4);
        STAMP_COUNT(9, 1);
        // gather outside the divergent branches (a load into registers that
        // another branch writes would force a full vmcnt drain); stored next step
        cur.gp = rP.p(gsrc);
        cur.em = em; cur.d = emd; cur.g = emg;
        lds_barrier();
        STAMP(5);
        STAMP_COUNT(10, 1);
    };
    // nchunks + 1 steps (the last one only emits).  Chunk i lives in
    // pre[i % (PF + 2)] from its load (step i - PF) to its emission store (step i + 1).
    static_assert(PF == 2, "prefetch depth 2: a ring of four chunks");
    for (uint32_t ci = 0; ci <= nchunks; ci += 4) {
        step(ci, A, B, pre[0], pre[3], pre[1], pre[2]);
        if (ci + 1 > nchunks) break;
        step(ci + 1, B, A, pre[1], pre[0], pre[2], pre[3]);
        if (ci + 2 > nchunks) break;
        step(ci + 2, A, B, pre[2], pre[1], pre[3], pre[0]);
        if (ci + 3 > nchunks) break;
        step(ci + 3, B, A, pre[3], pre[2], pre[0], pre[1]);
    }
    STAMP(7);
    lds_barrier();   // LDS only: the last emission stores need not land
    STAMP(11);
    if (tid < kDests * kDests / 2) {
        const uint32_t w = S.gcnt[tid];
        gacc0 += w & 0xFFFFu;
        gacc1 += w >> 16;
    }
#ifndef PCC_STAMPS
    unsigned long long* st_acc = nullptr, st_t0 = 0;
#endif
    dense_grid_points<NF, L>(P, S, S.head, rP, s, n, jmask, tid, lane, st_acc, st_t0);
    STAMP(8);
    STAMP_FLUSH(P.stamps);
    if (err) atomicOr(&S.err, err);
    lds_barrier();
    const uint32_t fp = nchunks & 1;   // dcur after the last (emit-only) step
    if (tid == 0) {
        P.slab_grid_n[s] = S.nwin;
        if (S.err) set_err(P.ctr, S.err);
    }
    if (tid < kDests) P.dest_n[s * kDests + tid] = S.dcur[fp][tid] < my_dcap ? S.dcur[fp][tid] : my_dcap;   // wave 0: lane = tid
    // capacities of the child slabs' own child slabs (only rows that will exist)
    if (tid < kDests * kDests / 2) {
        const uint32_t i0 = 2 * tid, i1 = 2 * tid + 1;
        if (S.dcur[fp][i0 / kDests]) P.gcap[(uint64_t)s * kDests * kDests + i0] = gacc0;
        if (S.dcur[fp][i1 / kDests]) P.gcap[(uint64_t)s * kDests * kDests + i1] = gacc1;
    }
}

// Small slabs (< kSmallMax arrivals): at most kSmallCh chunks of kSmallBS, so a
// thread keeps its own arrivals (payload, table entry, child and grandchild
// slab) in registers from pass 1 to pass 2, all loads are issued up front, and a
// displaced record finds its emission position in LDS: pass 2 makes no global
// loads.  The slot hash table is sized to the slab (power of two >= 2n).
constexpr int kSmallCh = (int)((kSmallMax + kSmallBS - 1) / kSmallBS);
struct SmallLds {
    unsigned long long tab[kSmallTab];
    uint32_t tkey[kSmallTab];
    uint32_t claim[2][kSmallClaim];
    uint32_t fate[kSmallMax];
    uint32_t gcnt[kDests * kDests];
    uint32_t doff[kDests], dcap[kDests], dcur[kDests];
    uint32_t wcnt[kSmallBS / 64][kDests], wpre[kSmallBS / 64][kDests];
    uint32_t npend[2], nwin, err;
};

__device__ __forceinline__ int small_entry(SmallLds& S, uint32_t local, uint32_t mask) {
    uint32_t h = hash_slot(local) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
        const uint32_t k = S.tkey[h];
        if (k == local) return (int)h;
        if (k == kEmpty32) {
            const uint32_t old = atomicCAS(&S.tkey[h], kEmpty32, local);
            if (old == kEmpty32 || old == local) return (int)h;
        }
        h = (h + 1) & mask;
    }
    return -1;
}

// flattened descriptor of a small slab: one scalar load instead of the chain
// list -> slab tables -> cell tables
constexpr uint32_t kWaveMax = 512;   // small slabs below this size: one wave each (k_slab_wave)
__device__ __forceinline__ SmallDesc slab_desc(uint32_t s, const uint32_t* slab_cell, const int32_t* slab_layer,
                                               const uint32_t* slab_off, const uint32_t* slab_n, const int32_t* cell_idx,
                                               const uint32_t* cell_sb, const uint32_t* dest_off, const uint32_t* dcap,
                                               uint64_t acap) {
    const uint32_t cr_ = slab_cell[s];
    SmallDesc D;
    D.s = s;
    D.off = slab_off[s];
    D.n = slab_n[s];
    D.dbase = dest_off[s * kDests];
    D.dlen = dest_off[s * kDests + kDests - 1] + dcap[s * kDests + kDests - 1] - D.dbase;
    // never past the next arena (a capacity sum above it is ERR_ARENA, k_level_begin)
    D.dlen = (uint32_t)min((uint64_t)D.dlen, acap > D.dbase ? acap - D.dbase : 0ull);
    D.t = slab_layer[s];
    D.cx = cell_idx[3 * cr_];
    D.cy = cell_idx[3 * cr_ + 1];
    D.cz = cell_idx[3 * cr_ + 2];
    D.sb = cell_sb[cr_];
    D.pad0 = D.pad1 = 0;
    D.ng = 0;
    return D;
}

// Launch order of a level's dense slabs when their sizes are skewed: the
// largest first (LPT), by 256 size classes; the order inside a class is free
// (slabs are independent).  One block.
__global__ __launch_bounds__(1024) void k_lpt_order(const uint32_t* __restrict__ list, uint32_t n,
                                                    const uint32_t* __restrict__ slab_n, uint32_t maxn,
                                                    uint32_t* __restrict__ out) {
    __shared__ uint32_t cnt[256];
    const uint32_t tid = threadIdx.x;
    if (tid < 256) cnt[tid] = 0;
    __syncthreads();
    auto cls = [&](uint32_t s) { return 255u - (uint32_t)(((uint64_t)slab_n[s] * 256u) / ((uint64_t)maxn + 1u)); };
    for (uint32_t i = tid; i < n; i += 1024) atomicAdd(&cnt[cls(list[i])], 1u);
    __syncthreads();
    if (tid < 64) {   // exclusive prefix over the 256 classes, 4 per lane
        uint32_t c4[4], t = 0;
        for (int q = 0; q < 4; q++) { c4[q] = cnt[tid * 4 + q]; t += c4[q]; }
        uint32_t x = t;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (tid >= (uint32_t)d) x += y;
        }
        uint32_t a = x - t;
        for (int q = 0; q < 4; q++) { cnt[tid * 4 + q] = a; a += c4[q]; }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += 1024) {
        const uint32_t sl = list[i];
        out[atomicAdd(&cnt[cls(sl)], 1u)] = sl;
    }
}

__global__ void k_dense_desc(const uint32_t* list, uint32_t nlist, const uint32_t* slab_cell, const int32_t* slab_layer,
                             const uint32_t* slab_off, const uint32_t* slab_n, const int32_t* cell_idx,
                             const uint32_t* cell_sb, const uint32_t* dest_off, const uint32_t* dcap, SmallDesc* out,
                             const uint32_t* slab_prior, const PriorSlabRec* prec, uint64_t acap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlist) return;
    SmallDesc D = slab_desc(list[i], slab_cell, slab_layer, slab_off, slab_n, cell_idx, cell_sb, dest_off, dcap, acap);
    if (slab_prior) {   // merge, level >= 1: seeds read in place (pad0 = offset in the seed array, pad1 = count)
        const uint32_t pr = slab_prior[D.s];
        if (pr != kNoPriorSlab) { D.pad0 = prec[pr].seed_off; D.pad1 = prec[pr].nseed; D.ng = prec[pr].ngrid; }
    }
    out[i] = D;
}

__global__ void k_small_desc(const uint32_t* list, uint32_t nlist, const uint32_t* slab_cell, const int32_t* slab_layer,
                             const uint32_t* slab_off, const uint32_t* slab_n, const int32_t* cell_idx,
                             const uint32_t* cell_sb, const uint32_t* dest_off, const uint32_t* dcap, SmallDesc* wave_out,
                             SmallDesc* block_out, uint32_t* counts, const uint32_t* slab_prior,
                             const PriorSlabRec* prec, uint64_t acap) {
    __shared__ uint32_t wc[4][4], bpre[4][4];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < nlist;
    SmallDesc D = slab_desc(in ? list[i] : list[0], slab_cell, slab_layer, slab_off, slab_n, cell_idx, cell_sb,
                            dest_off, dcap, acap);
    if (slab_prior) {   // merge, level >= 1: the slab's seeds stay in the seed array (pad0 = offset, pad1 = count)
        const uint32_t pr = slab_prior[D.s];
        if (pr != kNoPriorSlab) { D.pad0 = prec[pr].seed_off; D.pad1 = prec[pr].nseed; D.ng = prec[pr].ngrid; }
    }
    // size class: 0..2 one wave (< 128, < 256, < 512 arrivals), 3 block; the
    // wave classes share wave_out, class c from offset c * nlist.  One global
    // atomic per block and class.  A destination span of 2^16 points or more
    // (a merge: child slabs with many seeds in front of their emissions) takes
    // the block kernel, whose displaced-payload positions are 32-bit (the wave
    // kernel's are 16-bit: WaveLds::fate)
    const uint32_t cls = !in ? 4u : (D.dlen > 0xFFFFu ? 3u : (D.n < kWaveMax / 4 ? 0u : (D.n < kWaveMax / 2 ? 1u : (D.n < kWaveMax ? 2u : 3u))));
    const uint64_t lt = lanemask_lt();
    const uint32_t w = threadIdx.x / 64;
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t c = 0; c < 4; c++) {
        const uint64_t m = __ballot(cls == c);
        if (cls == c) rank = (uint32_t)__popcll(m & lt);
        if (__lane_id() == 0) wc[w][c] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint32_t c = threadIdx.x;
        uint32_t acc = 0;
        for (int q = 0; q < 4; q++) { bpre[q][c] = acc; acc += wc[q][c]; }
        const uint32_t b = acc ? atomicAdd(&counts[c], acc) : 0u;
        for (int q = 0; q < 4; q++) bpre[q][c] += b;
    }
    __syncthreads();
    if (cls < 3) wave_out[(uint64_t)cls * nlist + bpre[w][cls] + rank] = D;
    else if (cls == 3) block_out[bpre[w][3] + rank] = D;
}

// Per-thread register copy of one small slab's inputs (loaded one slab ahead).
struct SmallPre {
    u32x4 pp[kSmallCh];
    uint32_t pk[kSmallCh];
    uint32_t rh[kSmallCh], rl[kSmallCh];   // merge: a grid seed's slot-table record (k_seed_rec), else rh = ~0
    uint32_t doff, dcap;
};

__device__ __forceinline__ void small_prefetch(const SlabParams& P, uint32_t li, SmallDesc& D, SmallPre& R,
                                               uint32_t tid) {
    if (li >= P.nlist) return;   // block-uniform
    D = P.sdesc[li];
    const uint64_t nb = (uint64_t)D.n * 4;
    const __amdgpu_buffer_rsrc_t rP = srd(P.in.p + D.off, nb * 4), rK = srd(P.in.k + D.off, nb);
    if (D.pad1) {   // merge: arrivals 0 .. pad1-1 are seeds, read from the seed array (no copy into the room)
        const uint32_t ns = D.pad1;
        const __amdgpu_buffer_rsrc_t rS = srd(P.inj + D.pad0, (uint64_t)ns * 16),
                                     rT = srd(P.inj_keys + D.pad0, (uint64_t)ns * 4);
#pragma unroll
        for (int c = 0; c < kSmallCh; c++) {
            const uint32_t j = c * kSmallBS + tid;
            const bool v = j < D.n, sd = j < ns;
            const u32x4 a = bld4(rS, sd ? j * 16 : 0xFFFFFFFFu), b = bld4(rP, (v && !sd) ? j * 16 : 0xFFFFFFFFu);
            R.pp[c] = u32x4{a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w};   // out-of-range loads return 0
            R.pk[c] = bld(rT, sd ? j * 4 : 0xFFFFFFFFu) | bld(rK, (v && !sd) ? j * 4 : 0xFFFFFFFFu);
        }
        // the grid seeds' records (out of range: 0xFFFFFFFF, i.e. flagged)
        const __amdgpu_buffer_rsrc_t rR = srd(P.inj_rec + D.pad0, (uint64_t)D.ng * 8);
#pragma unroll
        for (int c = 0; c < kSmallCh; c++) {
            const uint32_t j = c * kSmallBS + tid;
            R.rl[c] = bld(rR, j < D.ng ? j * 8 : 0xFFFFFFFFu);
            R.rh[c] = j < D.ng ? bld(rR, j * 8 + 4) : 0xFFFFFFFFu;
        }
    } else {
#pragma unroll
        for (int c = 0; c < kSmallCh; c++) {
            const uint32_t j = c * kSmallBS + tid;
            const bool v = j < D.n;
            R.pp[c] = bld4(rP, v ? j * 16 : 0xFFFFFFFFu);
            R.pk[c] = bld(rK, v ? j * 4 : 0xFFFFFFFFu);
            R.rl[c] = 0u;
            R.rh[c] = 0xFFFFFFFFu;
        }
    }
    const __amdgpu_buffer_rsrc_t rD = srd(P.dest_off + (uint64_t)D.s * kDests, kDests * 4);
    const __amdgpu_buffer_rsrc_t rC = srd(P.dcap + (uint64_t)D.s * kDests, kDests * 4);
    R.doff = bld(rD, tid < kDests ? tid * 4 : 0xFFFFFFFFu);
    R.dcap = bld(rC, tid < kDests ? tid * 4 : 0xFFFFFFFFu);
}

__device__ __forceinline__ void small_process(const SlabParams& P, SmallLds& S, const SmallDesc& D, SmallPre& R,
                                              uint32_t tid) {
    constexpr int BS = kSmallBS, NW = BS / 64, CH = kSmallCh;
    STAMP_DECL
    const uint32_t wv = tid / 64;
    const uint32_t s = D.s;
    const int32_t t = D.t;
    const uint32_t n = D.n;
    const uint32_t dbase = D.dbase;
    const uint64_t db = (uint64_t)D.dlen * 4;
    const int32_t cx = D.cx, cy = D.cy, cz = D.cz;
    const LevelGeo& G = P.G;
    const uint32_t nch = (n + BS - 1) / BS;
    uint32_t cap = 64;
    while (cap < 2 * n && cap < (uint32_t)kSmallTab) cap <<= 1;
    const uint32_t mask = cap - 1;
    const __amdgpu_buffer_rsrc_t oP = srd(P.nx.p + dbase, db * 4), oK = srd(P.nx.k + dbase, db);
    u32x4* pp = R.pp;
    uint32_t* pk = R.pk;
    for (uint32_t i = tid; i < cap; i += BS) { S.tab[i] = kEmpty64; S.tkey[i] = kEmpty32; }
    for (int i = tid; i < 2 * kSmallClaim; i += BS) (&S.claim[0][0])[i] = kEmpty32;
    for (int i = tid; i < kDests * kDests; i += BS) S.gcnt[i] = 0;
    if (tid < kDests) {
        S.dcur[tid] = 0;
        S.doff[tid] = R.doff - dbase;
        S.dcap[tid] = R.dcap;
    }
    if (tid < NW * kDests) (&S.wcnt[0][0])[tid] = 0;
    if (tid == 0) { S.npend[0] = 0; S.npend[1] = 0; S.nwin = 0; S.err = 0; }
    // reference slot: the one holding the cell centre (metadata.rs:104-106)
    const I3 c0 = hex_from_world(cell_pos1(cx, P.cs), cell_pos1(cy, P.cs), cell_pos1(cz, P.cs), G.cr);
    const int32_t rx = c0.x - P.tx / 2, ry = c0.y - P.ty / 2;
    const SlabCtx SC{cx, cy, cz, t};
    const float zt = (float)t * G.cr;   // slot centre z of the slab's layer (hex.rs:63)
    uint32_t err = 0;
    const uint64_t lt = lanemask_lt();
    __syncthreads();
    STAMP(0);

    int32_t rec_e[CH];    // table entry of an arrival that became a slot record, else -1
    int32_t own_d[CH], own_g[CH];
    // Merge: the whole chunks of grid seeds go straight into the table, from
    // their records (k_seed_rec): one per slot and below every other key, they
    // claim nothing and emit nothing (as in k_slab's merge mode); the chunk loop
    // starts after them.
    uint32_t ci0 = 0;
    if (D.ng >= (uint32_t)BS) {
        const uint32_t nfull = min(D.ng / (uint32_t)BS, (uint32_t)CH);
        bool flagged = false;
#pragma unroll
        for (int c = 0; c < CH; c++)
            if ((uint32_t)c < nfull) flagged |= (R.rh[c] >> 31) != 0u;
        if (!__syncthreads_or(flagged)) {
            ci0 = nfull;
#pragma unroll
            for (int c = 0; c < CH; c++) {
                if ((uint32_t)c >= nfull) break;
                const uint32_t j = c * BS + tid;
                const uint32_t local = R.rh[c] & 0x3FFFu, dn = (R.rh[c] >> 14) & 31u;
                own_d[c] = (int32_t)dn;
                own_g[c] = (int32_t)((R.rh[c] >> 19) & 31u) - 1;
                rec_e[c] = small_entry(S, local, mask);
                if (rec_e[c] < 0) {
                    err |= ERR_CLAIM;
                } else {
                    const unsigned long long mine =
                        ((unsigned long long)R.rl[c] << 33) | ((unsigned long long)dn << kJBits) | j;
                    // two grid points in one slot: not a cell a converter writes
                    if (atomicCAS(&S.tab[rec_e[c]], kEmpty64, mine) != kEmpty64) err |= ERR_CLAIM;
                }
            }
            __syncthreads();
        }
    }
    // emission of the previous chunk: kind (-1 none, 0 self, 1 displaced), occupant, child slab, grandchild
    int32_t em = -1, emg = -1;
    uint32_t emj = 0, emd = 0;
#pragma unroll
    for (int ci = 0; ci <= CH; ci++) {
        if ((uint32_t)ci > nch) break;   // block-uniform
        if ((uint32_t)ci < ci0) continue;   // whole chunks of grid seeds, installed above
        const uint32_t par = ci & 1;
        uint32_t* claim = S.claim[par];
        const bool have = ci < CH && (uint32_t)ci < nch;
        const uint32_t j = ci * BS + tid;
        const bool valid = have && j < n;
        bool pending = false, self_em = false;
        uint32_t local = 0;
        int e = 0, hc = -1;
        float d2 = 0.f;
        uint32_t dn = 0;
        if (ci < CH) {
            int d, g;
            if (!__ballot(valid && (R.rh[ci] >> 31))) {
                // merge: a wave of grid seeds with their records (k_seed_rec)
                d2 = __uint_as_float(R.rl[ci]);   // (no NaN in a merge)
                pending = valid;
                local = valid ? (R.rh[ci] & 0x3FFFu) : 0u;
                d = (int)((R.rh[ci] >> 14) & 31u);
                g = (int)((R.rh[ci] >> 19) & 31u) - 1;
            } else {
            const float x = __uint_as_float(pp[ci].x), y = __uint_as_float(pp[ci].y), z = __uint_as_float(pp[ci].z);
            const SlotDest sd = slot_dest(x, y, z, G, SC);
            const int32_t lx = sd.ox - rx, ly = sd.oy - ry;
            const bool layer_ok = sd.layer_ok;
            const bool range_ok = lx >= 0 && ly >= 0 && lx < P.tx && ly < P.ty;
            float X, Y, Z;
            slot_centre(sd, G.cr, zt, X, Y, Z);
            d2 = dist2(X, Y, Z, x, y, z);
            const bool foreign = !range_ok && d2 != d2;   // NaN x or y: slot (0, 0) outside the table (see k_slab)
            pending = valid && layer_ok && (range_ok || foreign);
            local = pending ? (range_ok ? (uint32_t)(ly * P.tx + lx) : kForeignSlot) : 0u;
            d = sd.d;
            g = sd.g;
            const bool bad = valid && (!layer_ok || (!range_ok && !foreign) || d < 0 || (P.check_gchild && g < 0));
            if (__ballot(bad)) {
                if (bad) err |= slot_route_errs(slot_route(x, y, z, G), layer_ok, range_ok, cx, cy, cz, t, P.check_gchild);
            }
            }
            if (pending && pk[ci] - P.kf_lo < P.kf_n) {   // merge mode: forced emission
                pending = false;
                self_em = true;
            }
            dn = d < 0 ? 0u : (uint32_t)d;
            own_d[ci] = (int32_t)dn;
            own_g[ci] = g;
            rec_e[ci] = -1;
            if (pending) {   // occupant pre-filter (see k_slab)
                e = small_entry(S, local, mask);
                if (e >= 0) {
                    const unsigned long long occ = S.tab[e];
                    if (occ != kEmpty64 && !(d2 < __uint_as_float((uint32_t)(occ >> 33)))) {
                        self_em = true;
                        pending = false;
                    } else {
                        hc = claim_insert<kSmallClaim>(claim, local, tid);
                    }
                }
                if (e < 0 || (pending && hc < 0)) { err |= ERR_CLAIM; pending = false; }
            }
        }
        {
            const uint32_t np = (uint32_t)__popcll(__ballot(pending));
            if ((tid & 63) == 0 && np) atomicAdd(&S.npend[par], np);
        }
        STAMP(1);
        STAMP_COUNT(10, 1);
        // wave ranks of chunk ci-1's emissions per child slab
        const bool vd = em >= 0;
        const int d = vd ? (int)emd : 0;
        uint64_t same = __ballot(vd);
#pragma unroll
        for (int b = 0; b < 5; b++) {
            const uint64_t bb = __ballot(vd && ((d >> b) & 1));
            same &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rw = __popcll(same & lt);
        if (vd && rw == 0) S.wcnt[wv][d] = (uint32_t)__popcll(same);
        {   // grandchild capacities of self emissions
            const bool vg = vd && em == 0 && emg >= 0;
            const int32_t gg = vg ? emg : 0;
            uint64_t sg = same & __ballot(vg);
#pragma unroll
            for (int b = 0; b < 5; b++) {
                const uint64_t bb = __ballot(vg && ((gg >> b) & 1));
                sg &= ((gg >> b) & 1) ? bb : ~bb;
            }
            if (vg && __popcll(sg & lt) == 0) atomicAdd(&S.gcnt[d * kDests + gg], (uint32_t)__popcll(sg));
        }
        STAMP(2);
        lds_barrier();
        STAMP(3);
        if (tid < kDests) {
            uint32_t acc = S.dcur[tid];
#pragma unroll
            for (int q = 0; q < NW; q++) { const uint32_t cc = S.wcnt[q][tid]; S.wpre[q][tid] = acc; acc += cc; S.wcnt[q][tid] = 0; }
            S.dcur[tid] = acc;
        }
        int32_t nem = self_em ? 0 : -1;
        uint32_t nemj = 0, nemd = self_em ? dn : 0u;
        bool first = true;
        for (;;) {
            bool won = false;
            if (pending && (claim[hc] & kClaimDone) == tid) {
                const unsigned long long occ = S.tab[e];
                const unsigned long long mine =
                    ((unsigned long long)dist_key(d2) << 33) | ((unsigned long long)dn << kJBits) | j;
                if (occ == kEmpty64) {
                    S.tab[e] = mine;
                    rec_e[ci] = e;
                } else if (d2 < __uint_as_float((uint32_t)(occ >> 33))) {   // strict: ties keep the old point
                    S.tab[e] = mine;
                    rec_e[ci] = e;
                    nem = 1;
                    nemj = (uint32_t)occ & kJMask;
                    nemd = (uint32_t)(occ >> kJBits) & 31u;
                } else {
                    nem = 0;
                    nemd = dn;
                }
                pending = false;
                won = true;
                claim[hc] = (local << 11) | kClaimDone;
            }
            {
                const uint64_t wm = __ballot(won);
                if ((tid & 63) == 0 && wm) atomicSub(&S.npend[par], (uint32_t)__popcll(wm));
            }
            STAMP(4);
            STAMP_COUNT(9, 1);
            lds_barrier();
            STAMP(5);
            if (first) {   // chunk ci-1: stores into its child slabs
                first = false;
                const uint32_t r = S.wpre[wv][d] + rw;
                const bool ok = vd && r < S.dcap[d];
                err |= (vd && !ok) ? (uint32_t)ERR_CAPACITY : 0u;
                const uint32_t pos = S.doff[d] + r;
                const uint32_t po = ok ? pos * 4 : 0xFFFFFFFFu;
                if (ci > 0) {
                    const int pc = ci - 1 < CH ? ci - 1 : 0;
                    bst4(oP, (ok && em == 0) ? pos * 16 : 0xFFFFFFFFu, pp[pc]);
                    bst(oK, po, pk[pc]);
                }
                if (ok && em == 1) S.fate[emj] = pos;
                STAMP(6);
            }
            if (S.npend[par] == 0) break;
            if (pending) atomicMin(&claim[hc], (local << 11) | tid);
            STAMP(4);
            lds_barrier();
            STAMP(5);
        }
        if (hc >= 0) claim[hc] = kEmpty32;
        em = nem; emj = nemj; emd = nemd;
        emg = ci < CH ? own_g[ci] : -1;
    }
    STAMP(7);
    __syncthreads();   // fate[] and the final table are complete
    STAMP(11);

    // pass 2 from registers: grid points and displaced payloads
    const __amdgpu_buffer_rsrc_t rG = srd(P.grid + P.grid_off[s], (uint64_t)n * 16);
#pragma unroll
    for (int ci = 0; ci < CH; ci++) {
        if ((uint32_t)ci >= nch) break;
        const uint32_t j = ci * BS + tid;
        bool win = false, dsp = false;
        if (rec_e[ci] >= 0) {
            const unsigned long long occ = S.tab[rec_e[ci]];
            win = ((uint32_t)occ & kJMask) == j;
            dsp = !win;
        }
        const uint64_t m = __ballot(win);
        uint32_t wb = 0;
        if ((tid & 63) == 0 && m) wb = atomicAdd(&S.nwin, (uint32_t)__popcll(m));
        wb = __shfl(wb, 0, 64);
        bst4(rG, win ? (wb + (uint32_t)__popcll(m & lt)) * 16 : 0xFFFFFFFFu, pp[ci]);
        if (dsp) {
            bst4(oP, S.fate[j] * 16, pp[ci]);
            if (own_g[ci] >= 0) atomicAdd(&S.gcnt[own_d[ci] * kDests + own_g[ci]], 1u);
        }
    }
    STAMP(8);
    if (err) atomicOr(&S.err, err);
    __syncthreads();
    if (tid == 0) {
        P.slab_grid_n[s] = S.nwin;
        if (S.err) set_err(P.ctr, S.err);
    }
    if (tid < kDests) P.dest_n[s * kDests + tid] = S.dcur[tid] < S.dcap[tid] ? S.dcur[tid] : S.dcap[tid];
    for (int i = tid; i < kDests * kDests; i += BS) {
        const int dd = i / kDests;
        if (S.dcur[dd]) P.gcap[(uint64_t)s * kDests * kDests + i] = S.gcnt[i];
    }
    STAMP_FLUSH(P.stamps);
}

// One workgroup per slab (launched with one per list entry; the grid stride
// keeps any smaller grid correct).
__global__ __launch_bounds__(kSmallBS) void k_slab_small(SlabParams P) {
    __shared__ SmallLds S;
    const uint32_t tid = threadIdx.x;
    SmallDesc D;
    SmallPre R;
    for (uint32_t li = blockIdx.x; li < P.nlist; li += gridDim.x) {
        small_prefetch(P, li, D, R, tid);
        small_process(P, S, D, R, tid);
        __syncthreads();   // the next slab re-initialises the LDS tables
    }
}

// ------------------------------------------------------------------ one wave per slab
// Slabs of < kWaveMax arrivals (most of the deepest levels): one 64-lane wave
// per slab, one workgroup per slab, ~13 KB of LDS each so a CU holds ~11
// slabs at once, and no s_barrier between waves.  The table entry holds the
// slot key beside the occupant, and same-slot arrivals of a 64-arrival chunk
// are applied in lane (= key) order, one ballot rank per round.  Grandchild
// capacities are counted in LDS (two 16-bit counters per word: a slab has < 512
// arrivals) and stored once per slab.  Instantiated per size class (CH chunks
// of 64: slabs of < 64 * CH arrivals, table 128 * CH entries), so the classes of
// small slabs hold less LDS and fewer registers and more of them fit on a CU.
template <int CH>
struct WaveLds {
    static constexpr int TAB = 128 * CH;
    unsigned long long tab[TAB];
    uint16_t fate[64 * CH];   // displaced occupants' positions in the destination span (< 2^16: k_small_desc)
    uint32_t doff[kDests], dcap[kDests], dcur[kDests];
    uint32_t gcnt[kDests * kDests / 2];   // (child, grandchild) counts, 16 bits each
};
template <class WL>
__device__ __forceinline__ void wave_gcount(WL& W, bool active, uint32_t key) {
    if (active) atomicAdd(&W.gcnt[key >> 1], (key & 1u) ? 0x10000u : 1u);
}

// Entry: (d2 bits << 33) | (dest << 28) | (slot << 14) | j, j < 2^14; a slot
// taken with no occupant yet has d2 bits 0x7FFFFFFF (kEmpty64: no slot).  The
// packed fields bound the geometry: slot indices of a dim-96 layer (< kDenseTab)
// fit 14 bits below the reserved 0x3FFF, dest 0..23 fits 5 bits, and the
// per-chunk register (entry + 1 in 11 bits, wave_peers<10> of the entry) needs
// TAB <= 1024 entries.
constexpr unsigned long long kW2None = 0x7FFFFFFFull << 33;
static_assert(kDenseTab < (1 << 14) - 1, "wave-kernel entry: slot in 14 bits");
static_assert(kDests < 31, "wave-kernel entry: dest in 5 bits");
static_assert(128 * (kWaveMax / 64) <= 1024, "wave-kernel entry index: 10-bit peers, 11-bit entry + 1");
static_assert(kWaveMax <= (1u << 14), "wave-kernel entry: j in 14 bits");
__device__ __forceinline__ unsigned long long w2_reserved(uint32_t local) {
    return kW2None | (31ull << 28) | ((unsigned long long)local << 14) | 0x3FFFull;
}
template <class WL>
__device__ __forceinline__ int wave_entry2(WL& W, uint32_t local, uint32_t mask) {
    uint32_t h = hash_slot(local) & mask;
    const unsigned long long res = w2_reserved(local);
    for (uint32_t probe = 0; probe <= mask; probe++) {
        const unsigned long long old = atomicCAS(&W.tab[h], kEmpty64, res);
        if (old == kEmpty64 || (((uint32_t)old >> 14) & 0x3FFFu) == local) return (int)h;
        h = (h + 1) & mask;
    }
    return -1;
}

#ifndef PCC_WAVE_OCC
#define PCC_WAVE_OCC 4   // k_slab_wave: minimum waves per SIMD asked of the compiler (<= 128 VGPRs, no spills)
#endif
// MRG: a merge level (seeds in place): whole chunks of grid seeds go into the
// table from their records (k_seed_rec)
template <int CH, bool MRG = false>
__global__ __launch_bounds__(64, PCC_WAVE_OCC) void k_slab_wave(SlabParams P) {
    using WL = WaveLds<CH>;
    __shared__ WL W;
    const uint32_t lane = threadIdx.x;
    const uint64_t lt = lanemask_lt();
    const LevelGeo& G = P.G;
    for (uint32_t li = blockIdx.x; li < P.nwave; li += gridDim.x) {
        const SmallDesc D = P.wdesc[li];
        const uint32_t s = D.s, n = D.n, off = D.off, dbase = D.dbase;
        const int32_t t = D.t, cx = D.cx, cy = D.cy, cz = D.cz;
        const uint32_t nch = (n + 63) / 64;
        uint32_t cap = 64;
        while (cap < 2 * n && cap < (uint32_t)WL::TAB) cap <<= 1;
        const uint32_t mask = cap - 1;
        const uint64_t nb = (uint64_t)n * 4, db = (uint64_t)D.dlen * 4;
        const __amdgpu_buffer_rsrc_t rP = srd(P.in.p + off, nb * 4), rK = srd(P.in.k + off, nb);
        const __amdgpu_buffer_rsrc_t oP = srd(P.nx.p + dbase, db * 4), oK = srd(P.nx.k + dbase, db);
        u32x4 pp[CH];
        uint32_t pk[CH];
        // merge: whole chunks of grid seeds (nfull) take their slot-table records
        // (k_seed_rec): beside the payloads when registers allow (KEEP), else in
        // pp.x / pp.y until pass 2 reloads the payloads
        constexpr bool KEEP = CH <= 4;
        uint32_t rlo[KEEP ? CH : 1], rhi[KEEP ? CH : 1];
        const uint32_t nfull = (MRG && D.pad1) ? min(D.ng / 64u, (uint32_t)CH) : 0u;
        const __amdgpu_buffer_rsrc_t rS = srd(P.inj + D.pad0, (uint64_t)D.pad1 * 16);
        if (D.pad1) {   // merge: the seeds (arrivals 0 .. pad1-1) in place in the seed array
            const uint32_t ns = D.pad1;
            const __amdgpu_buffer_rsrc_t rT = srd(P.inj_keys + D.pad0, (uint64_t)ns * 4),
                                         rR = srd(P.inj_rec + D.pad0, (uint64_t)D.ng * 8);
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const uint32_t j = c * 64 + lane;
                const bool v = j < n, sd = j < ns;
                if (MRG && !KEEP && (uint32_t)c < nfull) {   // wave-uniform
                    pp[c] = u32x4{bld(rR, j * 8), bld(rR, j * 8 + 4), 0u, 0u};
                } else {
                    if constexpr (MRG && KEEP) {
                        rlo[c] = (uint32_t)c < nfull ? bld(rR, j * 8) : 0u;
                        rhi[c] = (uint32_t)c < nfull ? bld(rR, j * 8 + 4) : 0xFFFFFFFFu;
                    }
                    const u32x4 a = bld4(rS, sd ? j * 16 : 0xFFFFFFFFu), b = bld4(rP, (v && !sd) ? j * 16 : 0xFFFFFFFFu);
                    pp[c] = u32x4{a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w};
                }
                pk[c] = bld(rT, sd ? j * 4 : 0xFFFFFFFFu) | bld(rK, (v && !sd) ? j * 4 : 0xFFFFFFFFu);
            }
        } else {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const uint32_t j = c * 64 + lane;
                const bool v = j < n;
                pp[c] = bld4(rP, v ? j * 16 : 0xFFFFFFFFu);
                pk[c] = bld(rK, v ? j * 4 : 0xFFFFFFFFu);
            }
        }
        for (uint32_t i = lane; i < cap; i += 64) W.tab[i] = kEmpty64;
        for (uint32_t i = lane; i < kDests * kDests / 2; i += 64) W.gcnt[i] = 0;
        if (lane < kDests) {
            W.dcur[lane] = 0;
            W.doff[lane] = P.dest_off[s * kDests + lane] - dbase;
            W.dcap[lane] = P.dcap[s * kDests + lane];
        }
        const I3 c0 = hex_from_world(cell_pos1(cx, P.cs), cell_pos1(cy, P.cs), cell_pos1(cz, P.cs), G.cr);
        const int32_t rx = c0.x - P.tx / 2, ry = c0.y - P.ty / 2;
        const SlabCtx SC{cx, cy, cz, t};
        const float zt = (float)t * G.cr;   // slot centre z of the slab's layer (hex.rs:63)
        uint32_t* gcap_s = P.gcap + (uint64_t)s * kDests * kDests;
        uint32_t err = 0;
        __syncthreads();   // one wave: orders the LDS initialisation

        // per chunk, one register: (entry + 1, 0 none) | own child slab << 11 | (own grandchild slab + 1) << 16
        uint32_t own[CH];
#pragma unroll
        for (int c = 0; c < CH; c++) {
            own[c] = 0u;
            if ((uint32_t)c >= nch) continue;   // wave-uniform
            const uint32_t j = c * 64 + lane;
            if (MRG && (uint32_t)c < nfull) {   // merge: a whole chunk of grid seeds
                const uint32_t rl = KEEP ? rlo[c] : pp[c].x, rh = KEEP ? rhi[c] : pp[c].y;
                if (!__ballot(rh >> 31)) {
                    // straight into the table from their records: one per slot and
                    // below every other key, they emit nothing (as k_slab's merge mode)
                    const uint32_t local = rh & 0x3FFFu, dn = (rh >> 14) & 31u;
                    own[c] = (dn << 11) | (((rh >> 19) & 31u) << 16);
                    const int e = wave_entry2(W, local, mask);
                    if (e < 0) {
                        err |= ERR_CLAIM;
                    } else {
                        const unsigned long long occ =
                            __hip_atomic_load(&W.tab[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        if ((occ >> 33) != 0x7FFFFFFFull) err |= ERR_CLAIM;   // two grid points in one slot
                        const unsigned long long mine = ((unsigned long long)rl << 33) |
                                                        ((unsigned long long)dn << 28) |
                                                        ((unsigned long long)local << 14) | j;
                        __hip_atomic_store(&W.tab[e], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        own[c] |= (uint32_t)(e + 1);
                    }
                    continue;
                }
                if constexpr (!KEEP) pp[c] = bld4(rS, j * 16);   // flagged records: the seeds' own arithmetic below
            }
            const bool valid = j < n;
            const float x = __uint_as_float(pp[c].x), y = __uint_as_float(pp[c].y), z = __uint_as_float(pp[c].z);
            const SlotDest sd = slot_dest(x, y, z, G, SC);
            const int32_t lx = sd.ox - rx, ly = sd.oy - ry;
            const bool layer_ok = sd.layer_ok;
            const bool range_ok = lx >= 0 && ly >= 0 && lx < P.tx && ly < P.ty;
            float X, Y, Z;
            slot_centre(sd, G.cr, zt, X, Y, Z);
            const float d2 = dist2(X, Y, Z, x, y, z);
            const bool foreign = !range_ok && d2 != d2;   // NaN x or y: slot (0, 0) outside the table (see k_slab)
            bool pending = valid && layer_ok && (range_ok || foreign);
            const uint32_t local = pending ? (range_ok ? (uint32_t)(ly * P.tx + lx) : kForeignSlot) : 0u;
            const int d = sd.d;
            int g = sd.g;
            const bool bad = valid && (!layer_ok || (!range_ok && !foreign) || d < 0 || (P.check_gchild && g < 0));
            if (__ballot(bad)) {
                if (bad) err |= slot_route_errs(slot_route(x, y, z, G), layer_ok, range_ok, cx, cy, cz, t, P.check_gchild);
            }
            const uint32_t dn = d < 0 ? 0u : (uint32_t)d;
            own[c] = (dn << 11) | ((uint32_t)(g + 1) << 16);
            int e = 0;
            int32_t em = -1;
            uint32_t emj = 0, emd = 0;
            if (pending && pk[c] - P.kf_lo < P.kf_n) {   // merge mode: forced emission
                pending = false;
                em = 0;
                emd = dn;
            }
            if (pending) {
                e = wave_entry2(W, local, mask);
                if (e < 0) {
                    err |= ERR_CLAIM;
                    pending = false;
                } else {   // occupant pre-filter (see k_slab)
                    const unsigned long long occ = W.tab[e];
                    if ((occ >> 33) != 0x7FFFFFFFull && !(d2 < __uint_as_float((uint32_t)(occ >> 33)))) {
                        pending = false;
                        em = 0;
                        emd = dn;
                    }
                }
            }
            {   // same-slot lanes applied in lane (= key) order: rank among the
                // pending lanes of the same entry, one rank per round.  One wave's
                // LDS operations execute in program order; the entry is read and
                // written as wavefront-scope atomics, so the compiler can neither
                // reuse the pre-filter's load nor reorder a round's store past the
                // next round's load (lane A writes in round r, lane B reads in r+1)
                const uint64_t same = wave_peers<10>((uint32_t)(pending ? e : 0), pending);
                const uint32_t rk = (uint32_t)__popcll(same & lt);
                for (uint32_t r = 0; __ballot(pending && rk >= r); r++) {
                    if (pending && rk == r) {
                        const unsigned long long occ =
                            __hip_atomic_load(&W.tab[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        const unsigned long long mine = ((unsigned long long)dist_key(d2) << 33) |
                                                        ((unsigned long long)dn << 28) |
                                                        ((unsigned long long)local << 14) | j;
                        if ((occ >> 33) == 0x7FFFFFFFull) {
                            __hip_atomic_store(&W.tab[e], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            own[c] |= (uint32_t)(e + 1);
                        } else if (d2 < __uint_as_float((uint32_t)(occ >> 33))) {   // strict: ties keep the old point
                            __hip_atomic_store(&W.tab[e], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            own[c] |= (uint32_t)(e + 1);
                            em = 1;
                            emj = (uint32_t)occ & 0x3FFFu;
                            emd = (uint32_t)(occ >> 28) & 31u;
                        } else {
                            em = 0;
                            emd = dn;
                        }
                        pending = false;
                    }
                }
            }
            // emissions of this chunk, in lane order per child slab
            const bool vd = em >= 0;
            const int dd = vd ? (int)emd : 0;
            const uint64_t same = wave_peers<5>((uint32_t)dd, vd);
            const uint32_t rw = mask_rank(same);
            uint32_t r0 = 0;
            if (vd && rw == 0) r0 = atomicAdd(&W.dcur[dd], (uint32_t)__popcll(same));
            const int leader = vd ? (int)(__ffsll((long long)same) - 1) : (int)lane;
            r0 = __shfl(r0, leader, 64);
            const uint32_t r = r0 + rw;
            const bool ok = vd && r < W.dcap[dd];
            err |= (vd && !ok) ? (uint32_t)ERR_CAPACITY : 0u;
            const uint32_t pos = W.doff[dd] + r;
            const uint32_t po = ok ? pos * 4 : 0xFFFFFFFFu;
            bst4(oP, (ok && em == 0) ? pos * 16 : 0xFFFFFFFFu, pp[c]);
            bst(oK, po, pk[c]);
            if (ok && em == 1) W.fate[emj] = (uint16_t)pos;
            wave_gcount(W, ok && em == 0 && g >= 0, (uint32_t)(dd * kDests + (g < 0 ? 0 : g)));
        }
        __syncthreads();
        // pass 2 from registers: grid points and displaced payloads (the
        // record-installed seed chunks' payloads loaded again first)
        if constexpr (MRG && !KEEP) {
#pragma unroll
            for (int c = 0; c < CH; c++)
                if ((uint32_t)c < nfull) pp[c] = bld4(rS, (c * 64 + lane) * 16);
        }
        const __amdgpu_buffer_rsrc_t rG = srd(P.grid + P.grid_off[s], (uint64_t)n * 16);
        uint32_t nwin = 0;
#pragma unroll
        for (int c = 0; c < CH; c++) {
            if ((uint32_t)c >= nch) break;
            const uint32_t j = c * 64 + lane;
            bool win = false, dsp = false;
            const int32_t rec = (int32_t)(own[c] & 0x7FFu) - 1;
            const int32_t od = (int32_t)((own[c] >> 11) & 31u), og = (int32_t)((own[c] >> 16) & 31u) - 1;
            if (rec >= 0) {
                const unsigned long long occ = W.tab[rec];
                win = ((uint32_t)occ & 0x3FFFu) == j;
                dsp = !win;
            }
            const uint64_t m = __ballot(win);
            bst4(rG, win ? (nwin + (uint32_t)__popcll(m & lt)) * 16 : 0xFFFFFFFFu, pp[c]);
            nwin += (uint32_t)__popcll(m);
            bst4(oP, dsp ? (uint32_t)W.fate[j] * 16 : 0xFFFFFFFFu, pp[c]);
            wave_gcount(W, dsp && og >= 0, (uint32_t)(od * kDests + (og < 0 ? 0 : og)));
        }
        if (lane == 0) {
            P.slab_grid_n[s] = nwin;
        }
        const uint32_t wer = __reduce_or_sync(~0ull, err);
        if (lane == 0 && wer) set_err(P.ctr, wer);
        if (lane < kDests) P.dest_n[s * kDests + lane] = W.dcur[lane] < W.dcap[lane] ? W.dcur[lane] : W.dcap[lane];
        // grandchild capacities of the child slabs that received emissions
        for (uint32_t i = lane; i < kDests * kDests; i += 64) {
            if (W.dcur[i / kDests]) gcap_s[i] = (W.gcnt[i >> 1] >> ((i & 1u) * 16)) & 0xFFFFu;
        }
        __syncthreads();   // the next slab re-initialises the LDS tables
    }
}

// Capacities of the level-0 slabs: arrivals per child slab (24 per slab), one
// streaming pass over the level's arena.  Grid (nslabs, Y): block (s, y) takes
// arrivals y*256 + tid, stride Y*256.
struct DcapParams {
    Arena A;
    const int32_t* cell_idx;
    const uint32_t* slab_cell;
    const int32_t* slab_layer;
    const uint32_t* slab_off;
    const uint32_t* slab_n;
    uint32_t* dcap;
    Counters* ctr;
    float csc, inv_csc, crc, inv_crc;   // child level cell size / hex radius
    uint32_t check;                     // routing errors only matter if the child level can exist
};
__global__ __launch_bounds__(256) void k_dcap(DcapParams P) {
    __shared__ uint32_t cnt[kDests];
    const uint32_t s = blockIdx.x;
    const uint32_t off = P.slab_off[s], n = P.slab_n[s];
    const uint32_t j0 = blockIdx.y * 256;
    if (j0 >= n) return;
    if (threadIdx.x < kDests) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t cr_ = P.slab_cell[s];
    const int32_t t = P.slab_layer[s];
    const int32_t cx = P.cell_idx[3 * cr_], cy = P.cell_idx[3 * cr_ + 1], cz = P.cell_idx[3 * cr_ + 2];
    uint32_t err = 0;
    uint32_t loc[kDests] = {};
    const uint32_t stride = gridDim.y * 256;
    for (uint32_t j = j0 + threadIdx.x; j < n; j += stride) {
        const float4 v = P.A.p[off + j];
        bool amb = false;
        RouteIdx R = route_idx_q(P.csc, P.inv_csc, P.inv_crc, v.x, v.y, v.z, amb);
        if (__ballot(amb)) {
            if (amb) R = route_idx_exact(P.csc, P.crc, v.x, v.y, v.z);
        }
        const int d = route_dest(R, cx, cy, cz, t, err);
#pragma unroll
        for (int q = 0; q < kDests; q++) loc[q] += (q == d);
    }
#pragma unroll
    for (int q = 0; q < kDests; q++) {
        uint32_t v = loc[q];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&cnt[q], v);
    }
    if (err && P.check) set_err(P.ctr, err);
    __syncthreads();
    if (threadIdx.x < kDests && cnt[threadIdx.x]) atomicAdd(&P.dcap[s * kDests + threadIdx.x], cnt[threadIdx.x]);
}

// ------------------------------------------------------------------ bucket resolution
struct BucketParams {
    Arena nx;          // arrivals of level h+1 (== emissions of level h)
    const uint32_t* files;    // event batches from keys (lib.rs:31-52)
    uint32_t nfiles;
    const uint32_t* cell_sb;  // running spill batch of the level-h cells
    const int32_t* cell_idx;  // merge mode: the existing cloud's bucket states of this level's cells
    const PriorCell* prior;   // sorted by (x, y, z)
    uint32_t nprior;
    Point* kept;
    uint64_t kept_cap;
    unsigned long long* ksort;   // kept lists above kKeptMax: global sort scratch at 2 x their kept offset
    const uint32_t* cell_slab0;
    const uint32_t* dest_off;
    const uint32_t* dest_n;
    uint32_t* bkt_state;
    uint32_t* bkt_off;
    uint32_t* bkt_n;
    uint32_t* bkt_sb;
    uint32_t* bkt_nd;
    const uint32_t* room;     // merge: seeds injected into each child slab (a child slab exists if it has any)
    Counters* ctr;
    uint32_t L;
    uint32_t* dlist;    // buckets deferred to the second launch (k_bucket), and their count
    uint32_t* dcount;
};

constexpr int kBktBS = 512;
#ifndef PCC_BKT_ABL
#define PCC_BKT_ABL 0   // diagnostic builds only: 1 no kept-list sort, 2 no spill-batch search
#endif

// event batch of an emission of a level-h cell: max(eb0(key), cell's running sb)
__device__ __forceinline__ uint32_t emission_eb(const BucketParams& B, uint32_t key, uint32_t csb) {
    return max(event_batch(B.files, B.nfiles, key), csb);
}
// Smallest key with event_batch(key) > e: the first key of batch e + 1, in the
// last file whose first batch is <= e + 1 (clamped to the next file's start:
// a short last batch, or batches of an empty reader).
__device__ __forceinline__ uint32_t first_key_after(const uint32_t* files, uint32_t nfiles, uint32_t e) {
    const uint32_t b = e + 1;
    uint32_t lo = 0, hi = nfiles - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (files[4 * mid + 2] <= b) lo = mid; else hi = mid - 1;
    }
    const uint64_t start = (uint64_t)files[4 * lo] | ((uint64_t)files[4 * lo + 1] << 32);
    uint64_t k = files[4 * lo + 2] <= b ? start + (uint64_t)(b - files[4 * lo + 2]) * files[4 * lo + 3] : start;
    if (lo + 1 < nfiles) k = min(k, (uint64_t)files[4 * lo + 4] | ((uint64_t)files[4 * lo + 5] << 32));
    return (uint32_t)min(k, (uint64_t)0xFFFFFFFFu);
}

// cell.rs:108-153 add_points_in_overflow, resolved for all batches at once
// (SURVEY.md Appendix C.3): bucket = (cell, child octant), emissions key-ordered
// inside each of its child slabs.
// Two launches per level: k_bucket<kBktSmallBS, kKeptSmall> resolves every
// bucket except a kept list longer than kKeptSmall, which it appends to a list
// of deferred buckets (state 4); k_bucket<kBktBS, kKeptMax, true>, a few
// resident workgroups per CU, then walks that list with the 64 KB sort array.
// The first launch's 8 KB sort array lets several workgroups share a CU (most
// kept lists are short: the last level's cells have few emissions).
constexpr int kBktSmallBS = 256;
constexpr int kKeptSmall = 1024;
constexpr uint32_t kBktSplitMin = 8192;
constexpr int kBktLists = 640;   // a bucket's child-slab lists: 3 per slab of its cell (<= 3 x (2 dim + 5))   // buckets per level from which the two launches pay
constexpr uint32_t kBktDeferred = 4;
// A kept list in key order by a stable LSD radix sort, 4 key bits per pass over
// the bucket's key range (kmax - kmin: config 3's 27 bits in 7 passes).  The
// child-slab lists are each key-ordered, but a bucket has hundreds of short ones,
// so merging them gains little; the bitonic network it replaces took 91
// barrier-separated stages for 8 192 words and was the level's critical path
// on skewed clouds.  LDS: the keys (u32) and the element indices ping-ponged
// (u16) in the 64 KB of the packed-word array, plus per-pass digit counts per
// (row, wave) and their block-scanned bases.  An element's index is its place
// in the concatenation of the lists in destination order, so its arena
// position follows from a binary search over the lists' first indices.
#ifndef PCC_BKT_RADIX
#define PCC_BKT_RADIX 1
#endif
constexpr uint32_t kBktRadixMin = 1024;   // kept lists at least this long: radix sort
template <int BS, int KMAX>
__device__ __forceinline__ void bucket_sort_radix(const BucketParams& B, uint32_t b, uint32_t s0, uint32_t oct, uint32_t nd,
                                                  uint32_t tot, uint32_t s_off, uint32_t* lds, unsigned long long* skp,
                                                  uint32_t* s_lo, uint32_t* s_ln, uint32_t* s_lp) {
    constexpr int W = BS / 64, ROWS = KMAX / BS, NRW = KMAX / 64, NC = 16 * NRW, EPT = NC / BS;
    static_assert(KMAX % BS == 0 && NC % BS == 0 && ROWS <= 32, "radix geometry");
    __shared__ alignas(16) uint8_t rcnt[NC];
    __shared__ uint16_t rpre[NC];
    __shared__ uint32_t r_min, r_max;
    uint32_t* skey = reinterpret_cast<uint32_t*>(skp);
    uint16_t* sidx[2] = {reinterpret_cast<uint16_t*>(skey + KMAX), reinterpret_cast<uint16_t*>(skey + KMAX) + KMAX};
    const uint32_t tid = threadIdx.x, w = tid / 64, lane = tid & 63;
    // the lists' first indices in destination order (one block scan)
    constexpr uint32_t LPT = (kBktLists + BS - 1) / BS;
    uint32_t ln_[LPT], acc = 0;
#pragma unroll
    for (uint32_t j = 0; j < LPT; j++) {
        const uint32_t i = tid * LPT + j;
        ln_[j] = 0;
        if (i < nd) {
            const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
            ln_[j] = B.dest_n[di];
            s_lo[i] = B.dest_off[di];
            s_ln[i] = ln_[j];
        }
        acc += ln_[j];
    }
    uint32_t t_;
    uint32_t base = block_excl_scan<BS>(acc, lds, &t_);
#pragma unroll
    for (uint32_t j = 0; j < LPT; j++) {
        const uint32_t i = tid * LPT + j;
        if (i < nd) s_lp[i] = base;
        base += ln_[j];
    }
    if (tid == 0) { r_min = 0xFFFFFFFFu; r_max = 0; }
    __syncthreads();
    // keys in (a wave per list), indices 0 .. tot-1
    for (uint32_t k = w; k < nd; k += W) {
        const uint32_t n = s_ln[k], o = s_lo[k], p = s_lp[k];
        for (uint32_t q = lane; q < n; q += 64) skey[p + q] = B.nx.k[o + q];
    }
    for (uint32_t i = tid; i < tot; i += BS) sidx[0][i] = (uint16_t)i;
    __syncthreads();
    uint32_t kmn = 0xFFFFFFFFu, kmx = 0;
    for (uint32_t i = tid; i < tot; i += BS) { kmn = min(kmn, skey[i]); kmx = max(kmx, skey[i]); }
    atomicMin(&r_min, kmn);
    atomicMax(&r_max, kmx);
    __syncthreads();
    const uint32_t kmin = r_min, span = r_max - r_min;
    const uint32_t bits = span ? 32u - (uint32_t)__clz(span) : 0u;
    const uint64_t lt = lanemask_lt();
    int cur = 0;
    for (uint32_t sh = 0; sh < bits; sh += 4, cur ^= 1) {
        for (uint32_t i = tid; i < NC / 4; i += BS) reinterpret_cast<uint32_t*>(rcnt)[i] = 0;
        __syncthreads();
        uint32_t reg[ROWS];   // per row: element index | rank << 13 | digit << 19 | valid << 23
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const uint32_t i = (uint32_t)r * BS + tid;
            const bool valid = i < tot;
            const uint32_t id = valid ? sidx[cur][i] : 0u;
            const uint32_t d = valid ? ((skey[id] - kmin) >> sh) & 15u : 0u;
            const uint64_t peers = wave_peers<4>(d, valid);
            const uint32_t rk = (uint32_t)__popcll(peers & lt);
            if (valid && rk == 0) rcnt[d * NRW + r * W + w] = (uint8_t)__popcll(peers);
            reg[r] = id | (rk << 13) | (d << 19) | (valid ? 1u << 23 : 0u);
        }
        __syncthreads();
        // bases: exclusive scan of the counts in (digit, row, wave) order
        uint32_t c[EPT], sum = 0;
#pragma unroll
        for (int e = 0; e < EPT; e++) { c[e] = rcnt[tid * EPT + e]; sum += c[e]; }
        uint32_t tt;
        uint32_t pb = block_excl_scan<BS>(sum, lds, &tt);
#pragma unroll
        for (int e = 0; e < EPT; e++) { rpre[tid * EPT + e] = (uint16_t)pb; pb += c[e]; }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const uint32_t v = reg[r];
            if (v >> 23) {
                const uint32_t d = (v >> 19) & 15u, rk = (v >> 13) & 63u;
                sidx[cur ^ 1][rpre[d * NRW + r * W + w] + rk] = (uint16_t)(v & 0x1FFFu);
            }
        }
        __syncthreads();
    }
    // the points in key order: element -> its list (last first index <= it) -> arena position
    for (uint32_t i = tid; i < tot; i += BS) {
        const uint32_t e = sidx[cur][i];
        uint32_t lo = 0, hi = nd;   // first list with s_lp > e, minus one
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (s_lp[m] <= e) lo = m + 1; else hi = m;
        }
        const uint32_t k = lo - 1;
        reinterpret_cast<float4*>(B.kept)[s_off + i] = B.nx.p[s_lo[k] + (e - s_lp[k])];
    }
    if (tid == 0) { B.bkt_state[b] = 1; B.bkt_off[b] = s_off; B.bkt_n[b] = tot; B.bkt_nd[b] = 0; B.bkt_sb[b] = 0; }
}

template <int BS, int KMAX, bool DEFERRED>
__device__ __forceinline__ void bucket_one(const BucketParams& B, const uint32_t b, uint32_t* lds,
                                           unsigned long long* skp) {
    __shared__ uint32_t s_cnt, s_off, s_nl;
    __shared__ uint32_t s_min, s_max;
    __shared__ uint32_t s_lo[kBktLists], s_ln[kBktLists], s_lp[kBktLists];   // a kept bucket's lists
    const uint32_t cell = b >> 3, oct = b & 7;
    const uint32_t s0 = B.cell_slab0[cell], s1 = B.cell_slab0[cell + 1];
    const uint32_t nd = (s1 - s0) * 3;
    const uint32_t L = B.L;
    const uint32_t csb = B.cell_sb[cell];
    uint32_t tot = 0, nne = 0, emin = 0xFFFFFFFFu, emax = 0;
    for (uint32_t i = threadIdx.x; i < nd; i += BS) {
        const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
        const uint32_t n = B.dest_n[di];
        nne += (n || (B.room && B.room[di])) ? 1u : 0u;   // slabs of the child cell, if it is built
        if (n) {
            const uint32_t o = B.dest_off[di];
            tot += n;
            emin = min(emin, emission_eb(B, B.nx.k[o], csb));
            emax = max(emax, emission_eb(B, B.nx.k[o + n - 1], csb));
        }
    }
    if (threadIdx.x == 0) { s_min = 0xFFFFFFFFu; s_max = 0; }
    __syncthreads();
    atomicMin(&s_min, emin);
    atomicMax(&s_max, emax);
    tot = block_sum<BS>(tot, lds);
    nne = block_sum<BS>(nne, lds);
    emin = s_min;
    emax = s_max;
    if (B.nprior) {   // merge mode: a bucket that is None on disk forwards everything at once (cell.rs:128-130)
        const int32_t x = B.cell_idx[3 * cell], y = B.cell_idx[3 * cell + 1], z = B.cell_idx[3 * cell + 2];
        uint32_t lo = 0, hi = B.nprior;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const PriorCell& q = B.prior[mid];
            const bool less = q.x != x ? q.x < x : (q.y != y ? q.y < y : q.z < z);
            if (less) lo = mid + 1; else hi = mid;
        }
        const bool found = lo < B.nprior && B.prior[lo].x == x && B.prior[lo].y == y && B.prior[lo].z == z;
        if (found && ((B.prior[lo].st >> (2 * oct)) & 3u) == 2u) {
            // state 3: None with nothing forwarded in this build (no child cell to build)
            if (threadIdx.x == 0) {
                B.bkt_state[b] = tot ? 2u : 3u; B.bkt_n[b] = tot; B.bkt_nd[b] = tot ? nne : 0u; B.bkt_sb[b] = 0; B.bkt_off[b] = 0;
            }
            return;
        }
    }
    if (tot == 0) {
        if (threadIdx.x == 0) { B.bkt_state[b] = 0; B.bkt_n[b] = 0; B.bkt_nd[b] = 0; B.bkt_off[b] = 0; B.bkt_sb[b] = 0; }
        return;
    }
    const bool spilled = tot > L || (tot == L && emin != emax);
    if (!spilled) {
        // Some(list): the bucket's points in key order, kept in this cell's file
        if (!DEFERRED && KMAX < kKeptMax && tot > (uint32_t)KMAX) {   // sorted by the second launch
            if (threadIdx.x == 0) {
                B.bkt_state[b] = kBktDeferred;
                B.dlist[atomicAdd(B.dcount, 1u)] = b;
            }
            return;
        }
        const bool big = tot > (uint32_t)KMAX;   // (limit > kKeptMax): sorted in global memory
        if (big && !B.ksort) {
            if (threadIdx.x == 0) { set_err(B.ctr, ERR_KEPT_CAP); B.bkt_state[b] = 0; }
            return;
        }
        if (threadIdx.x == 0) {
            s_cnt = 0;
            s_nl = 0;
            s_off = atomicAdd(&B.ctr->kept_cur, tot);
            if ((uint64_t)s_off + tot > B.kept_cap) set_err(B.ctr, ERR_KEPT_CAP);
        }
        __syncthreads();
        if ((uint64_t)s_off + tot > B.kept_cap) return;
        // long lists by the radix sort (a fixed number of passes), short ones by
        // the bitonic network (log^2 stages of a small power of two: config 4's
        // last level of 32 768 mostly short lists ran 0.33 ms slower all radix)
        if (!big && nd <= (uint32_t)kBktLists && PCC_BKT_RADIX && tot >= kBktRadixMin) {
            bucket_sort_radix<BS, KMAX>(B, b, s0, oct, nd, tot, s_off, lds, skp, s_lo, s_ln, s_lp);
            return;
        }
        // the packed words (key << 32 | arena position) in LDS, or for a list
        // above the LDS capacity in the scratch at twice its kept offset (a
        // power-of-two padding below twice the list never reaches the next list's)
        unsigned long long* sk = big ? B.ksort + 2ull * s_off : skp;
        if (nd <= (uint32_t)kBktLists) {
            // the non-empty child-slab lists into an LDS table (threads over
            // lists), then each list copied by one wave (lanes over its points):
            // a long list is not one thread's serial loop
            for (uint32_t i = threadIdx.x; i < nd; i += BS) {
                const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
                const uint32_t n = B.dest_n[di];
                if (n) {
                    const uint32_t k = atomicAdd(&s_nl, 1u);
                    s_lo[k] = B.dest_off[di];
                    s_ln[k] = n;
                    s_lp[k] = atomicAdd(&s_cnt, n);
                }
            }
            __syncthreads();
            const uint32_t wv = threadIdx.x / 64, ln = threadIdx.x & 63, nl = s_nl;
            for (uint32_t k = wv; k < nl; k += BS / 64) {
                const uint32_t o = s_lo[k], n = s_ln[k], p = s_lp[k];
                for (uint32_t q = ln; q < n; q += 64) sk[p + q] = ((unsigned long long)B.nx.k[o + q] << 32) | (o + q);
            }
        } else {
            for (uint32_t i = threadIdx.x; i < nd; i += BS) {
                const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
                const uint32_t n = B.dest_n[di];
                if (n) {
                    const uint32_t o = B.dest_off[di];
                    const uint32_t p = atomicAdd(&s_cnt, n);
                    for (uint32_t q = 0; q < n; q++) sk[p + q] = ((unsigned long long)B.nx.k[o + q] << 32) | (o + q);
                }
            }
        }
        uint32_t np2 = 1;
        while (np2 < tot) np2 <<= 1;
        __syncthreads();
        for (uint32_t i = tot + threadIdx.x; i < np2; i += BS) sk[i] = ~0ull;
        __syncthreads();
        // bitonic sort by key (keys are unique, so the packed words order by
        // key); one thread per compare-exchange pair (the workgroup barrier
        // orders the global scratch's accesses too: one workgroup owns it)
#if PCC_BKT_ABL == 1
        if (tot > 0xFFFFFFFEu)   // (diagnostic build: the sort skipped, timing only)
#endif
        for (uint32_t kk = 2; kk <= np2; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                for (uint32_t p = threadIdx.x; p < np2 / 2; p += BS) {
                    const uint32_t i = ((p & ~(jj - 1)) << 1) | (p & (jj - 1)), ix = i | jj;
                    const bool up = (i & kk) == 0;
                    const unsigned long long a = sk[i], c = sk[ix];
                    if ((a > c) == up) { sk[i] = c; sk[ix] = a; }
                }
                __syncthreads();
            }
        for (uint32_t i = threadIdx.x; i < tot; i += BS) {
            const uint32_t o = (uint32_t)sk[i];
            const float4 v = B.nx.p[o];
            reinterpret_cast<float4*>(B.kept)[s_off + i] = v;
        }
        if (threadIdx.x == 0) { B.bkt_state[b] = 1; B.bkt_off[b] = s_off; B.bkt_n[b] = tot; B.bkt_nd[b] = 0; B.bkt_sb[b] = 0; }
        return;
    }
    // None: spilled.  Spill batch sb = smallest e with c(e) >= L + [c(e0) == L],
    // c(e) = #bucket emissions with eb <= e (== Appendix C.3's rank rule).  eb is
    // monotone in the key inside a list, so a list's share of c(e) is the lower
    // bound of K(e) = the first key with eb0 > e (0 below the cell's sb).  Binary
    // search over e; each list keeps the window of its count that the search so
    // far allows (counts are monotone in e), so a step costs a few loads per list.
    constexpr int WL = 4;   // lists per thread with a window (nd <= WL * BS)
    __shared__ uint32_t s_k;
    const bool windowed = nd <= (uint32_t)(WL * BS);
    uint32_t wlo[WL], whi[WL], woff[WL], wr[WL];
#pragma unroll
    for (int w = 0; w < WL; w++) {
        wlo[w] = whi[w] = woff[w] = wr[w] = 0;
        const uint32_t i = threadIdx.x + (uint32_t)w * BS;
        if (windowed && i < nd) {
            const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
            const uint32_t n = B.dest_n[di];
            if (n) { woff[w] = B.dest_off[di]; whi[w] = n < L + 1 ? n : L + 1; }
        }
    }
    auto eval = [&](uint32_t e) -> uint32_t {   // c(e) (first L + 1 of each list); wr = per-list shares
        __syncthreads();
        if (threadIdx.x == 0) s_k = e < csb ? 0u : first_key_after(B.files, B.nfiles, e);
        __syncthreads();
        const uint32_t K = s_k;
        uint32_t c = 0;
        if (windowed) {
#pragma unroll
            for (int w = 0; w < WL; w++) {
                uint32_t lo2 = wlo[w], hi2 = whi[w];
                while (lo2 < hi2) {
                    const uint32_t mid = (lo2 + hi2) >> 1;
                    if (B.nx.k[woff[w] + mid] < K) lo2 = mid + 1; else hi2 = mid;
                }
                wr[w] = lo2;
                c += lo2;
            }
        } else {
            for (uint32_t i = threadIdx.x; i < nd; i += BS) {
                const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
                const uint32_t n = B.dest_n[di];
                if (!n) continue;
                const uint32_t o = B.dest_off[di];
                uint32_t lo2 = 0, hi2 = n < L + 1 ? n : L + 1;
                while (lo2 < hi2) {
                    const uint32_t mid = (lo2 + hi2) >> 1;
                    if (B.nx.k[o + mid] < K) lo2 = mid + 1; else hi2 = mid;
                }
                c += lo2;
            }
        }
        return block_sum<BS>(c, lds);
    };
    const uint32_t c0 = eval(emin);
#pragma unroll
    for (int w = 0; w < WL; w++) wlo[w] = wr[w];   // every later e is >= emin
    const uint32_t target = L + (c0 == L ? 1u : 0u);
    uint32_t lo = emin, hi = emax;   // c(emax) = tot >= target
#if PCC_BKT_ABL == 2
    hi = lo;   // (diagnostic build: the spill-batch search skipped, timing only)
#endif
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (eval(mid) >= target) {
            hi = mid;
#pragma unroll
            for (int w = 0; w < WL; w++) whi[w] = wr[w];
        } else {
            lo = mid + 1;
#pragma unroll
            for (int w = 0; w < WL; w++) wlo[w] = wr[w];
        }
    }
    if (threadIdx.x == 0) { B.bkt_state[b] = 2; B.bkt_n[b] = tot; B.bkt_nd[b] = nne; B.bkt_sb[b] = lo; B.bkt_off[b] = 0; }
}
template <int BS, int KMAX, bool DEFERRED = false>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_bucket(BucketParams B) {   // (two 512-thread workgroups per CU)
    __shared__ uint32_t lds[BS / 64 + 1];
    __shared__ unsigned long long skp[KMAX];   // (key << 32) | arena position
    if constexpr (!DEFERRED) {
        bucket_one<BS, KMAX, false>(B, blockIdx.x, lds, skp);
    } else {
        // the deferred buckets by ticket (their sizes vary)
        __shared__ uint32_t s_next;
        const uint32_t nl = *B.dcount;
        uint32_t i = blockIdx.x;
        while (i < nl) {
            bucket_one<BS, KMAX, true>(B, B.dlist[i], lds, skp);
            if (threadIdx.x == 0) s_next = atomicAdd(B.dcount + 1, 1u) + gridDim.x;
            __syncthreads();   // (also: the next bucket reuses the LDS)
            i = s_next;
            __syncthreads();
        }
    }
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
    const uint32_t* gcap;
    int32_t* ncell_idx;
    uint32_t* ncell_sb;
    uint32_t* ncell_slab0;
    uint32_t* nslab_cell;
    int32_t* nslab_layer;
    uint32_t* nslab_off;
    uint32_t* nslab_n;
    uint32_t* ndcap;
    uint32_t* nbig_list;
    uint32_t* nsmall_list;
    // merge (nullptr otherwise): records of this level's slabs, the reserved seed
    // room per child slab, the existing cloud's slab records at this level and the next
    const uint32_t* slab_prior;
    const uint32_t* room;
    const PriorSlabRec* prec;
    const PriorSlabRec* prec_next;
    uint32_t* nslab_prior;
    Counters* ctr;
};

__global__ __launch_bounds__(256) void k_next_emit(NextParams Q) {
    __shared__ uint32_t lds[256 / 64 + 1];
    __shared__ uint32_t carry, s_big, s_small, s_bigbase, s_smallbase, s_max;
    __shared__ unsigned long long s_arr, s_arr_big;
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
        s_big = 0;
        s_small = 0;
        s_arr = 0;
        s_arr_big = 0;
        s_max = 0;
    }
    __syncthreads();
    const uint32_t s0 = Q.cell_slab0[cell], s1 = Q.cell_slab0[cell + 1];
    const uint32_t nd = (s1 - s0) * 3;
    // pass 1: count big / small slabs of this cell (one global atomic per block)
    for (uint32_t i = threadIdx.x; i < nd; i += 256) {
        const uint32_t di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
        const uint32_t n = Q.dest_n[di] + (Q.room ? Q.room[di] : 0u);   // + injected seeds
        if (n) {
            atomicAdd(n >= kSmallMax ? &s_big : &s_small, 1u);
            atomicAdd(&s_arr, (unsigned long long)n);
            if (n >= kSmallMax) atomicAdd(&s_arr_big, (unsigned long long)n);
            atomicMax(&s_max, n);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_max) atomicMax(&Q.ctr->max_slab, s_max);
        s_bigbase = s_big ? atomicAdd(&Q.ctr->nbig, s_big) : 0;
        s_smallbase = s_small ? atomicAdd(&Q.ctr->nsmall, s_small) : 0;
        if (s_arr) atomicAdd(&Q.ctr->arrivals_next, s_arr);
        if (s_arr_big) atomicAdd(&Q.ctr->dense_arrivals, s_arr_big);
        if (s_arr > s_arr_big) atomicAdd(&Q.ctr->small_arrivals, s_arr - s_arr_big);
        s_big = 0;
        s_small = 0;
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < nd; i0 += 256) {
        const uint32_t i = i0 + threadIdx.x;
        uint32_t n = 0, di = 0, rm = 0;
        if (i < nd) {
            di = (s0 + i / 3) * kDests + oct * 3 + i % 3;
            rm = Q.room ? Q.room[di] : 0u;
            n = Q.dest_n[di] + rm;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<256>(n ? 1u : 0u, lds, &tot);
        if (n) {
            const uint32_t sid = base + carry + ex;
            const int32_t t = Q.slab_layer[s0 + i / 3];
            Q.nslab_cell[sid] = r;
            Q.nslab_layer[sid] = 2 * t + (int32_t)(i % 3) - 1;
            Q.nslab_off[sid] = Q.dest_off[di] - rm;   // the seeds are copied in front of the emissions
            Q.nslab_n[sid] = n;
            const uint32_t* g = Q.gcap + (uint64_t)di * kDests;
            uint32_t pr = kNoPriorSlab;
            if (Q.nslab_prior) {
                const uint32_t ps = Q.slab_prior[s0 + i / 3];
                pr = (rm && ps != kNoPriorSlab) ? Q.prec[ps].child[oct * 3 + i % 3] : kNoPriorSlab;
                Q.nslab_prior[sid] = pr;
            }
            const uint32_t* sd = pr != kNoPriorSlab ? Q.prec_next[pr].dcap : nullptr;
            // the slab kernels write a gcap row only for a child slab that received
            // emissions (dest_n > 0); a child slab of seeds alone has none
            const bool ge = Q.dest_n[di] != 0;
            {   // the 24-word rows as six 16-byte loads, all issued before the stores
                u32x4 v[kDests / 4];
#pragma unroll
                for (int k = 0; k < kDests / 4; k++)
                    v[k] = ge ? reinterpret_cast<const u32x4*>(g)[k] : u32x4{0u, 0u, 0u, 0u};
                if (sd) {
#pragma unroll
                    for (int k = 0; k < kDests / 4; k++) v[k] += reinterpret_cast<const u32x4*>(sd)[k];
                }
#pragma unroll
                for (int k = 0; k < kDests / 4; k++) reinterpret_cast<u32x4*>(Q.ndcap + (uint64_t)sid * kDests)[k] = v[k];
            }
            if (n >= kSmallMax) Q.nbig_list[s_bigbase + atomicAdd(&s_big, 1u)] = sid;
            else Q.nsmall_list[s_smallbase + atomicAdd(&s_small, 1u)] = sid;
        }
        __syncthreads();
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
}

// big / small slab lists at level 0 (block-aggregated atomics)
// (dn: the slab count on the device, else nslabs)
__global__ __launch_bounds__(256) void k_l0_lists(const uint32_t* slab_n, uint32_t nslabs, uint32_t* big,
                                                  uint32_t* small, Counters* ctr, const uint32_t* dn) {
    if (dn) nslabs = *dn;
    __shared__ uint32_t nb, ns, bb, bs;
    __shared__ unsigned long long ab, as;
    if (threadIdx.x == 0) { nb = 0; ns = 0; ab = 0; as = 0; }
    __syncthreads();
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    uint32_t rb = 0, rs = 0;
    const bool v = s < nslabs;
    const bool isbig = v && slab_n[s] >= kSmallMax;
    if (v) {
        if (isbig) { rb = atomicAdd(&nb, 1u); atomicAdd(&ab, (unsigned long long)slab_n[s]); }
        else { rs = atomicAdd(&ns, 1u); atomicAdd(&as, (unsigned long long)slab_n[s]); }
    }
    uint32_t mx = v ? slab_n[s] : 0;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&ctr->max_slab, mx);
    __syncthreads();
    if (threadIdx.x == 0) {
        bb = nb ? atomicAdd(&ctr->nbig, nb) : 0;
        bs = ns ? atomicAdd(&ctr->nsmall, ns) : 0;
        if (ab) atomicAdd(&ctr->dense_arrivals, ab);
        if (as) atomicAdd(&ctr->small_arrivals, as);
    }
    __syncthreads();
    if (v) { if (isbig) big[bb + rb] = s; else small[bs + rs] = s; }
}

__global__ void k_set_u32(uint32_t* p, uint32_t v) { *p = v; }
__global__ __launch_bounds__(256) void k_readback(RbSrc r, uint32_t* __restrict__ out) {
    uint32_t o = 0;
    for (int k = 0; k < 4; k++) {
        for (uint32_t i = threadIdx.x; i < r.n[k]; i += 256) out[o + i] = r.p[k][i];
        o += r.n[k];
    }
}
// A level's counters back to zero, and the sum of its child-slab capacities
// checked against the next arena (the slab descriptors clamp every region to it)
__global__ void k_level_begin(Counters* ctr, const uint32_t* cap_total, uint64_t cap) {
    ctr->kept_cur = 0;
    ctr->nbig = ctr->nsmall = 0;
    ctr->max_slab = 0;
    ctr->arrivals_next = 0;
    if (*cap_total > cap) ctr->err |= ERR_ARENA;
}

// merge: the existing cloud's record of each level-0 slab (cell by binary search
// over the sorted prior cells, then the layer inside the cell's records)
__global__ void k_prior_lookup0(const int32_t* cell_idx, const uint32_t* slab_cell, const int32_t* slab_layer,
                                uint32_t nslabs, const PriorCell* pc, const uint32_t* pc_slab0, const int32_t* p_layer,
                                uint32_t npc, uint32_t* slab_prior) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslabs) return;
    const uint32_t c = slab_cell[s];
    const int32_t x = cell_idx[3 * c], y = cell_idx[3 * c + 1], z = cell_idx[3 * c + 2], t = slab_layer[s];
    uint32_t lo = 0, hi = npc;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const PriorCell& q = pc[mid];
        const bool less = q.x != x ? q.x < x : (q.y != y ? q.y < y : q.z < z);
        if (less) lo = mid + 1; else hi = mid;
    }
    uint32_t r = kNoPriorSlab;
    if (lo < npc && pc[lo].x == x && pc[lo].y == y && pc[lo].z == z) {
        uint32_t a = pc_slab0[lo], b = pc_slab0[lo + 1];
        while (a < b) {
            const uint32_t mid = (a + b) >> 1;
            if (p_layer[mid] < t) a = mid + 1; else b = mid;
        }
        if (a < pc_slab0[lo + 1] && p_layer[a] == t) r = a;
    }
    slab_prior[s] = r;
}

// merge: seeds reserved in front of each child slab (room) and the scan input
// (capacity + room) of the emission regions
__global__ void k_room(const uint32_t* slab_prior, uint32_t nslabs, const PriorSlabRec* prec,
                       const PriorSlabRec* prec_next, const uint32_t* dcap, uint32_t* room, uint32_t* cap_room) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= (uint64_t)nslabs * kDests) return;
    const uint32_t ps = slab_prior[i / kDests];
    const uint32_t ch = ps != kNoPriorSlab ? prec[ps].child[i % kDests] : kNoPriorSlab;
    const uint32_t r = ch != kNoPriorSlab ? prec_next[ch].nseed : 0u;
    room[i] = r;
    cap_room[i] = dcap[i] + r;
}
// dest_off = (exclusive scan of capacity + room) + room: the emissions follow the seeds
__global__ void k_add_room(uint32_t* dest_off, const uint32_t* room, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) dest_off[i] += room[i];
}
// merge: copy each new slab's seeds (points and keys) in front of its emissions
__global__ __launch_bounds__(256) void k_inject_seeds(const uint32_t* slab_prior, const uint32_t* slab_off, uint32_t nslabs,
                                                      const PriorSlabRec* prec, const float4* __restrict__ inj,
                                                      const uint32_t* __restrict__ inj_keys, Arena A,
                                                      const uint32_t* __restrict__ slab_n) {
    for (uint32_t s = blockIdx.x; s < nslabs; s += gridDim.x) {
        const uint32_t pr = slab_prior[s];
        if (pr == kNoPriorSlab || slab_n[s] < kSmallMax) continue;   // small slabs read their seeds in place
        const uint32_t so = prec[pr].seed_off, n = prec[pr].nseed, o = slab_off[s];
        for (uint32_t j = threadIdx.x; j < n; j += 256) {
            A.p[(uint64_t)o + j] = inj[(uint64_t)so + j];
            A.k[(uint64_t)o + j] = inj_keys[(uint64_t)so + j];
        }
    }
}

// keys of a merge's level-0 input: the level-0 seeds 0 .. n0-1, then S + each new
// point's key (its index, or its global key for sharded input)
__global__ void k_comb_keys(uint32_t* out, const uint32_t* keys, uint64_t n0, uint64_t S, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n0 + n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = i < n0 ? (uint32_t)i : (uint32_t)(S + (keys ? (uint64_t)keys[i - n0] : i - n0));
}

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
    HIP_CHECK(hipMalloc(&dev_->rb_dev, kReadbackWords * 4));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&dev_->rb_host), kReadbackWords * 4, hipHostMallocDefault));
}

// Small device values for the host (counters, totals, boxes) in one round trip:
// a one-block kernel packs up to four word ranges into one device block, one
// copy moves it to pinned memory, one stream sync, then the host unpacks.
// (Separate copies into pageable stack variables cost 20-60 us each between
// kernels, a few per level.)
void Engine::readback(std::initializer_list<RbPart> parts) {
    readback_begin(parts);
    readback_end();
}
// begin: queue the pack and the copy, then record an event; end: wait for that
// event only (work queued after begin keeps running) and unpack
void Engine::readback_begin(std::initializer_list<RbPart> parts) {
    RbSrc r{};
    uint32_t k = 0, words = 0;
    rb_parts_.assign(parts.begin(), parts.end());
    for (const RbPart& q : parts) {
        r.p[k] = static_cast<const uint32_t*>(q.dev);
        r.n[k] = (uint32_t)(q.bytes / 4);
        words += r.n[k++];
    }
    if (words > kReadbackWords) throw std::runtime_error("readback: too many words");
    k_readback<<<1, 256, 0, stream_>>>(r, dev_->rb_dev);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(dev_->rb_host, dev_->rb_dev, (uint64_t)words * 4, hipMemcpyDeviceToHost, stream_));
    if (!rb_ev_) HIP_CHECK(hipEventCreateWithFlags(&rb_ev_, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(rb_ev_, stream_));
}
void Engine::readback_end() {
    HIP_CHECK(hipEventSynchronize(rb_ev_));
    uint32_t o = 0;
    for (const RbPart& q : rb_parts_) {
        std::memcpy(q.host, dev_->rb_host + o, q.bytes);
        o += (uint32_t)(q.bytes / 4);
    }
    rb_parts_.clear();
}

Engine::~Engine() {
    try {
        free_all();
    } catch (...) {
    }
    if (own_stream_) (void)hipStreamDestroy(stream_);
    for (Staging& b : stage_) {
        if (b.host) (void)hipHostFree(b.host);
        if (b.done) (void)hipEventDestroy(b.done);
    }
    if (copy_) (void)hipStreamDestroy(copy_);
    if (pre_ev_) (void)hipEventDestroy(pre_ev_);
    (void)hipFree(d_tile6_);
    (void)hipFree(d_prepart_);
    (void)hipFree(d_preflag_);
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

// Blocks go back to the process-wide cache, where another converter (any
// stream) can take them at once: nothing queued on this engine's streams may
// still touch them (hipFree synchronised implicitly, the cache does not).
void Engine::quiesce() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (copy_) (void)hipStreamSynchronize(copy_);
}

void Engine::free_all() {
    quiesce();
    for (auto& u : ev_used_) { ev_pool_.push_back(u.second.first); ev_pool_.push_back(u.second.second); }
    ev_used_.clear();
    for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
    ev_pool_.clear();
    for (Level* l : levels_) delete l;
    delete pending_;
    pending_ = nullptr;
    levels_.clear();
    if (dev_) {
        for (int a = 0; a < 2; a++) {
            dev_release(dev_->ar[a].p); dev_release(dev_->ar[a].k);
        }
        (void)hipFree(dev_->ctr);
        (void)hipFree(dev_->bbox_part);
        (void)hipFree(dev_->bbox_flag);
        (void)hipFree(dev_->rb_dev);
        if (rb_ev_) (void)hipEventDestroy(rb_ev_);
        rb_ev_ = nullptr;
        if (dev_->rb_host) (void)hipHostFree(dev_->rb_host);
        if (dev_->hst) (void)hipHostFree(dev_->hst);
        (void)hipFree(dev_->scan.bsums);
        for (auto& c : dev_->chunks) dev_release(c.first);
        delete dev_;
        dev_ = nullptr;
    }
    dev_release(d_in_);
    d_in_ = nullptr;
    dev_release(d_keys_);
    d_keys_ = nullptr;
    keys_cap_ = 0;
    dev_release(d_comb_);
    d_comb_ = nullptr;
    dev_release(d_ckeys_);
    d_ckeys_ = nullptr;
    ckeys_cap_ = 0;
    // non-finite inputs' split copies, the upload-time pass-1 records
    dev_release(d_nf_pts_); dev_release(d_nf_keys_);
    d_nf_pts_ = nullptr; d_nf_keys_ = nullptr; nf_cap_ = 0;
    dev_release(d_inf_pts_); dev_release(d_inf_keys_);
    d_inf_pts_ = nullptr; d_inf_keys_ = nullptr; inf_cap_ = 0;
    dev_release(d_pre6_cnt_); dev_release(d_pre6_ph_); dev_release(d_pre6_gpar_); dev_release(d_pre6_dummy_);
    dev_release(d_pre6_glist_);
    d_pre6_glist_ = nullptr;
    pre6_glist_cap_ = 0;
    if (land_ev_) (void)hipEventDestroy(land_ev_);
    land_ev_ = nullptr;
    d_pre6_cnt_ = d_pre6_ph_ = d_pre6_gpar_ = nullptr;
    d_pre6_dummy_ = nullptr;
    pre6_alloc_tiles_ = pre6_alloc_groups_ = 0;
    pre6_ = false;
    free_prior();
}

void Engine::free_prior() {
    quiesce();
    dev_release(d_seeds_);
    d_seeds_ = nullptr;
    dev_release(d_inj_);
    d_inj_ = nullptr;
    dev_release(d_inj_keys_);
    d_inj_keys_ = nullptr;
    dev_release(d_inj_rec_);
    d_inj_rec_ = nullptr;
    for (PriorDev& d : pdev_) {
        dev_release(d.cells); dev_release(d.cell_slab0); dev_release(d.slab_layer); dev_release(d.slabs);
    }
    pdev_.clear();
}

int Engine::fail(int code, const std::string& msg) {
    err_ = msg;
    return code;
}
// A point whose level-0 cell, layer or child route disagrees with the grid the
// parallel binning laid out: at coordinates far from the origin (f32 spacing
// near the sub-cell size) the separately rounded quotients x / cs and z / r
// need not nest as they do nearer the origin.  build() replays such an input
// sequentially (the reference's own per-point arithmetic) when it can.
int Engine::geom_fail(const char* msg) {
    geom_fault_ = true;
    return fail(-34, std::string(msg) + " (coordinates far from the origin: the sequential replay takes inputs of "
                                        "at most 2^24 points without merge or level range)");
}

void Engine::reserve(uint64_t n) {
    if (ext_in_) throw std::runtime_error("input added after borrowed keyed input");
    if (n <= cap_) return;
    if (n >= 0xFFFFFFFFull) throw std::runtime_error("more than 2^32-1 points per build are not supported");
    Point* p = nullptr;
    dev_alloc_t(p, std::max<uint64_t>(n, 1) * sizeof(Point));
    // the points of the files so far and of the one being streamed in
    const uint64_t live = n_ + stream_n_;
    if (live) HIP_CHECK(hipMemcpyAsync(p, d_in_, live * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    dev_release(d_in_);
    d_in_ = p;
    cap_ = n;
}

static uint32_t batches_of(uint64_t n, uint32_t batch) {
    const uint64_t b = std::max<uint32_t>(batch, 1);
    return (uint32_t)std::max<uint64_t>(1, (n + b - 1) / b);
}

void Engine::add_file_host(const Point* pts, uint64_t n, uint32_t batch) {
    comb_ok_ = false;
    reserve(n_ + n);
    // the copy in pieces on the copy stream; behind each piece, on the engine
    // stream, level-0 pass 0 of the tiles it completes (the host thread blocks
    // in each copy of pageable memory while the device counts the last piece)
    if (!copy_) HIP_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
    if (!pre_ev_) HIP_CHECK(hipEventCreateWithFlags(&pre_ev_, hipEventDisableTiming));
    const char* pp = getenv("PCC_PRE_PIECE");   // (tests: smaller pieces)
    const uint64_t piece = pp ? std::max<uint64_t>(1, strtoull(pp, nullptr, 10)) : kPrePiece;
    for (uint64_t off = 0; off < n; off += piece) {
        const uint64_t m = std::min<uint64_t>(piece, n - off);
        HIP_CHECK(hipMemcpyAsync(d_in_ + n_ + off, pts + off, m * sizeof(Point), hipMemcpyHostToDevice, copy_));
        HIP_CHECK(hipEventRecord(pre_ev_, copy_));
        pre0_count(n_ + off + m, pre_ev_, false);
    }
    HIP_CHECK(hipStreamSynchronize(copy_));
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += n;
    nbatches_ += batches_of(n, batch);
    // (the level-0 work behind the copies may still run on the engine stream:
    // the build is ordered behind it)
}

void Engine::stream_begin(uint64_t expected) {
    if (!copy_) HIP_CHECK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));   // (add_file_host makes it too)
    if (!stage_[0].host) {
        for (Staging& b : stage_) {
            HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.host), kStagePts * sizeof(Point), hipHostMallocDefault));
            HIP_CHECK(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
        }
    }
    comb_ok_ = false;
    reserve(n_ + expected);
    stream_n_ = 0;
}

void Engine::stream_push(const Point* pts, uint64_t n) {
    while (n) {
        Staging& b = stage_[stage_i_];
        if (b.busy) HIP_CHECK(hipEventSynchronize(b.done));   // its previous copy has landed
        const uint64_t m = std::min(n, kStagePts);
        if (n_ + stream_n_ + m > cap_) {   // grow: the copies in flight must land in the old buffer first
            HIP_CHECK(hipStreamSynchronize(copy_));
            reserve(std::max<uint64_t>(n_ + stream_n_ + m, cap_ + cap_ / 2));
        }
        std::memcpy(b.host, pts, m * sizeof(Point));
        HIP_CHECK(hipMemcpyAsync(d_in_ + n_ + stream_n_, b.host, m * sizeof(Point), hipMemcpyHostToDevice, copy_));
        HIP_CHECK(hipEventRecord(b.done, copy_));
        b.busy = true;
        stream_n_ += m;
        pre0_count(n_ + stream_n_, b.done, false);
        pts += m;
        n -= m;
        stage_i_ = (stage_i_ + 1) % kStages;
    }
}

uint64_t Engine::stream_end(uint64_t keep, uint32_t batch) {
    if (copy_) HIP_CHECK(hipStreamSynchronize(copy_));
    for (Staging& b : stage_) b.busy = false;
    keep = std::min(keep, stream_n_);
    if (keep < stream_n_) pre0_reset();   // counted points that are not kept
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += keep;
    nbatches_ += batches_of(keep, batch);
    stream_n_ = 0;
    return keep;
}

void Engine::stream_cancel() {
    if (copy_) HIP_CHECK(hipStreamSynchronize(copy_));
    for (Staging& b : stage_) b.busy = false;
    if (stream_n_) pre0_reset();
    stream_n_ = 0;
}

void Engine::add_file_device(const Point* dpts, uint64_t n, uint32_t batch) {
    comb_ok_ = false;
    reserve(n_ + n);
    if (n) HIP_CHECK(hipMemcpyAsync(d_in_ + n_, dpts, n * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += n;
    nbatches_ += batches_of(n, batch);
}

void Engine::add_file_synth(uint64_t seed, int kind, uint64_t n, uint32_t batch, float lo, float ext) {
    comb_ok_ = false;
    reserve(n_ + n);
    if (n) k_synth<<<grid_for(n, 256, 1 << 20), 256, 0, stream_>>>(d_in_, n_, n, seed, kind, lo, ext);
    HIP_CHECK(hipGetLastError());
    file_start_.push_back(n_);
    file_eb0_.push_back(nbatches_);
    file_batch_.push_back(std::max<uint32_t>(batch, 1));
    n_ += n;
    nbatches_ += batches_of(n, batch);
}

void Engine::declare_files(const uint64_t* file_points, uint64_t nfiles, uint32_t batch) {
    uint64_t g = 0;
    for (uint64_t f = 0; f < nfiles; f++) {
        file_start_.push_back(g);
        file_eb0_.push_back(nbatches_);
        file_batch_.push_back(std::max<uint32_t>(batch, 1));
        g += file_points[f];
        nbatches_ += batches_of(file_points[f], batch);
    }
    declared_total_ += g;
    keyed_ = true;
}

void Engine::set_event_table(const uint64_t* starts, const uint32_t* eb, uint64_t n, uint64_t total_batches) {
    if (!file_start_.empty()) throw std::runtime_error("event table after declared files or input");
    for (uint64_t k = 0; k < n; k++) {
        if (k && !(starts[k] > starts[k - 1] && eb[k] > eb[k - 1]))
            throw std::runtime_error("event table: starts and batches must ascend");
        if (eb[k] >= total_batches) throw std::runtime_error("event table: batch beyond the batch count");
        file_start_.push_back(starts[k]);
        file_eb0_.push_back(eb[k]);
        file_batch_.push_back(0x7FFFFFFFu);   // (i - start) / batch = 0: one batch per entry
    }
    if (n && starts[0] != 0) throw std::runtime_error("event table: the first entry must start at point 0");
    nbatches_ = total_batches;
    event_table_ = true;
    keyed_ = true;
}

void Engine::set_keyed_external(const Point* dpts, const uint32_t* dkeys, uint64_t n) {
    if (n_ || !keyed_) throw std::runtime_error("borrowed keyed input needs declared files and no other input");
    if (n >= 0xFFFFFFFFull) throw std::runtime_error("more than 2^32-1 points per build are not supported");
    ext_in_ = dpts;
    ext_keys_ = dkeys;
    n_ = n;
    comb_ok_ = false;
}

void Engine::add_keyed_device(const Point* dpts, const uint32_t* dkeys, uint64_t n) {
    if (event_table_) throw std::runtime_error("keyed points after an event table (keys are the indices there)");
    reserve(n_ + n);
    if (keys_cap_ < n_ + n) {
        uint32_t* k = nullptr;
        dev_alloc_t(k, std::max<uint64_t>(cap_, 1) * 4);
        if (n_) HIP_CHECK(hipMemcpyAsync(k, d_keys_, n_ * 4, hipMemcpyDeviceToDevice, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        dev_release(d_keys_);
        d_keys_ = k;
        keys_cap_ = cap_;
    }
    if (n) {
        HIP_CHECK(hipMemcpyAsync(d_in_ + n_, dpts, n * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
        HIP_CHECK(hipMemcpyAsync(d_keys_ + n_, dkeys, n * 4, hipMemcpyDeviceToDevice, stream_));
    }
    n_ += n;
    keyed_ = true;
    comb_ok_ = false;
}

template <class T, class A>
static T* upload(const std::vector<T, A>& v) {
    T* d = nullptr;
    dev_alloc_t(d, std::max<size_t>(v.size(), 1) * sizeof(T));
    if (!v.empty()) HIP_CHECK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

// Slot-table geometry of level h (the slab kernels' quotients, hex.rs:67-85,
// metadata.rs:91-102)
static LevelGeo level_geo(const Config& cfg, uint32_t h) {
    const uint32_t dim = cfg.sub_grid_dimension;
    const float cs = cell_size(cfg.max_cell_size, h), csc = cell_size(cfg.max_cell_size, h + 1),
                csg = cell_size(cfg.max_cell_size, h + 2);
    LevelGeo G;
    G.cr = hex_radius(sub_cell_size(cs, dim));
    G.crx = G.cr * kSqrt3;
    G.cry = (-G.cr) * kSqrt3;
    G.inv_crx = 1.0f / G.crx;
    G.inv_cry = 1.0f / G.cry;
    G.inv_cr = 1.0f / G.cr;
    G.csc = csc;
    G.inv_csc = 1.0f / csc;
    G.crc = hex_radius(sub_cell_size(csc, dim));
    G.inv_crc = 1.0f / G.crc;
    G.csg = csg;
    G.inv_csg = 1.0f / csg;
    G.crg = hex_radius(sub_cell_size(csg, dim));
    G.inv_crg = 1.0f / G.crg;
    G.exact = 0;
    for (float v : {G.cr, G.crx, G.cry, G.csg, G.crg})   // div_rc's divisor range
        if (!(std::fabs(v) >= 0x1p-60f && std::fabs(v) <= 0x1p60f)) G.exact = 1;
    return G;
}

// The slot-table record of every grid seed of the existing cloud's levels >= 1,
// made once when the cloud is adopted (the reference recomputes each stored
// point's slot when it reads a cell, cell.rs:183-229): the slab kernel's merge
// mode then installs a seed with one load and one LDS CAS instead of its slot
// and route arithmetic.  Record: d2 key (bits 0-31), slot index in the slab's
// table (32-45), child slab (46-50), grandchild slab + 1 (51-55); bit 63: the
// seed's slot or route failed (the kernel recomputes it and reports the error).
__global__ __launch_bounds__(256) void k_seed_rec(const PriorCell* __restrict__ cells, const uint32_t* __restrict__ cell_slab0,
                                                  const int32_t* __restrict__ slab_layer,
                                                  const PriorSlabRec* __restrict__ slabs, uint32_t ncells,
                                                  const float4* __restrict__ inj, LevelGeo G, float cs, int32_t tx, int32_t ty,
                                                  int32_t check_gchild, uint32_t flag_all,
                                                  unsigned long long* __restrict__ rec) {
    for (uint32_t c = blockIdx.x; c < ncells; c += gridDim.x) {
        const int32_t cx = cells[c].x, cy = cells[c].y, cz = cells[c].z;
        const I3 c0 = hex_from_world(cell_pos1(cx, cs), cell_pos1(cy, cs), cell_pos1(cz, cs), G.cr);
        const int32_t rx = c0.x - tx / 2, ry = c0.y - ty / 2;
        for (uint32_t s = cell_slab0[c]; s < cell_slab0[c + 1]; s++) {
            const int32_t t = slab_layer[s];
            const SlabCtx SC{cx, cy, cz, t};
            const float zt = (float)t * G.cr;
            const uint32_t off = slabs[s].seed_off, ng = slabs[s].ngrid;
            for (uint32_t j = threadIdx.x; j < ng; j += 256) {
                const float4 q = inj[off + j];
                const SlotDest sd = slot_dest(q.x, q.y, q.z, G, SC);
                const int32_t lx = sd.ox - rx, ly = sd.oy - ry;
                const bool range_ok = lx >= 0 && ly >= 0 && lx < tx && ly < ty;
                float X, Y, Z;
                slot_centre(sd, G.cr, zt, X, Y, Z);
                const float d2 = dist2(X, Y, Z, q.x, q.y, q.z);
                const bool bad = flag_all || !sd.layer_ok || !range_ok || sd.d < 0 || (check_gchild && sd.g < 0) ||
                                 (uint32_t)(ly * tx + lx) >= (1u << 14);
                rec[off + j] = bad ? (1ull << 63)
                                   : ((unsigned long long)dist_key(d2) | ((unsigned long long)(ly * tx + lx) << 32) |
                                      ((unsigned long long)sd.d << 46) | ((unsigned long long)(sd.g + 1) << 51));
            }
        }
    }
}

void Engine::set_prior(const PriorState& p) {
    HIP_CHECK(hipStreamSynchronize(stream_));
    free_prior();
    nseeds_ = p.nseeds;
    nseeds0_ = p.seeds0.size();
    prior_nan_ = p.has_nan;
    prior_max_abs_ = p.max_abs;
    d_seeds_ = upload(p.seeds0);
    d_inj_ = upload(p.inj);
    d_inj_keys_ = upload(p.inj_keys);
    forced_lo_ = p.forced_lo;
    for (const PriorLevel& lv : p.levels) {
        PriorDev d;
        d.cells = upload(lv.cells);
        d.cell_slab0 = upload(lv.cell_slab0);
        d.slab_layer = upload(lv.slab_layer);
        d.slabs = upload(lv.slabs);
        d.ncells = (uint32_t)lv.cells.size();
        d.nslabs = (uint32_t)lv.slabs.size();
        pdev_.push_back(d);
    }
    // the grid seeds' slot-table records (levels >= 1; level h of the build is
    // level h of the existing cloud: the config governs both)
    dev_alloc_t(d_inj_rec_, std::max<size_t>(p.inj.size(), 1) * 8);
    {
        const SlabGeom g = slab_geom(cfg_.sub_grid_dimension);
        for (size_t h = 1; h < pdev_.size(); h++) {
            const PriorDev& d = pdev_[h];
            if (!d.ncells) continue;
            k_seed_rec<<<std::min<uint32_t>(d.ncells, 65536), 256, 0, stream_>>>(
                d.cells, d.cell_slab0, d.slab_layer, d.slabs, d.ncells, reinterpret_cast<const float4*>(d_inj_),
                level_geo(cfg_, (uint32_t)h), cell_size(cfg_.max_cell_size, (uint32_t)h), g.tx, g.ty,
                (h + 2 < kMaxDepth) ? 1 : 0, getenv("PCC_NO_SEED_REC") ? 1u : 0u,   // (tests: every seed flagged)
                d_inj_rec_);
        }
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(stream_));
    }
    prior_ = true;
    comb_ok_ = false;
}

void Engine::clear_input() {
    HIP_CHECK(hipStreamSynchronize(stream_));
    comb_ok_ = false;
    n_ = 0;
    nbatches_ = 0;
    file_start_.clear();
    file_eb0_.clear();
    file_batch_.clear();
    keyed_ = false;
    ext_in_ = nullptr;
    ext_keys_ = nullptr;
    declared_total_ = 0;
    event_table_ = false;
    built_ = false;
    pre0_reset();
}

int Engine::build() {
    // a repeated build() re-runs everything from the resident input (bench steps)
    for (Level* l : levels_) delete l;
    levels_.clear();
    delete pending_;
    pending_ = nullptr;
    dev_->reset_pool();
    built_ = true;
    prof_ = StageProfile();
    const auto t0 = std::chrono::steady_clock::now();
    if (cfg_.sub_grid_dimension == 0) return fail(-22, "sub_grid_dimension must be > 0");
    if (cfg_.cell_point_overflow_limit > (1u << 24))
        return fail(-22, "cell_point_overflow_limit > 2^24 is not supported by the GPU build");
    const SlabGeom g = slab_geom(cfg_.sub_grid_dimension);
    // sub-grids beyond the LDS slot table or the level-0 layer field (dimension
    // > 96): the sequential replay (build_wide)
    const bool wide = g.tx * g.ty > kDenseTab || g.nl > (int32_t)kL0Layers || getenv("PCC_TEST_WIDE") != nullptr;
    if (wide && (prior_ || h0_ || max_levels_))
        return fail(-22, "sub_grid_dimension > 96: merges and level ranges are not supported");
    if (prior_ && (h0_ || max_levels_)) return fail(-22, "a merge cannot be split into level ranges");
    hierarchies_ = nbatches_ > 0 ? 1u : 0u;   // converter.rs:141-158 runs for every batch, even empty
    stats_ = BuildStats();
    side_.clear();
    if (n_ == 0) return 0;

    // Input of the build.  Merge mode: the existing
    // cloud's points come first as "seeds" with keys 0 .. S-1, so every one of
    // them precedes every new point in key order, then the new points with keys
    // S + i.  All seeds belong to a pseudo batch 0 before the new batches.
    if (event_table_) {   // rank-local keys: a borrowed input whose keys are its indices
        if (n_ && (!ext_in_ || ext_keys_)) return fail(-22, "event table: the input must be borrowed without keys");
        if (n_ && (file_start_.empty() || file_start_.back() >= n_))
            return fail(-22, "event table: an entry starts past the input");
    }
    if (prior_ && keyed_ && nseeds_ + declared_total_ >= 0xFFFFFFFFull)   // keys S + global key (k_comb_keys)
        return fail(-75, "sharded merge: this rank's existing points plus the global new points exceed 2^32-1 keys");
    if (prior_) {   // level-0 input: the level-0 seeds (keys 0 .. n0-1), then the new points (S + key)
        const uint64_t n0 = nseeds0_;
        if (!comb_ok_) {
            if (comb_cap_ < n0 + n_) {
                dev_release(d_comb_);
                dev_alloc_t(d_comb_, std::max<uint64_t>(n0 + n_, 1) * sizeof(Point));
                comb_cap_ = n0 + n_;
            }
            if (n0) HIP_CHECK(hipMemcpyAsync(d_comb_, d_seeds_, n0 * sizeof(Point), hipMemcpyDeviceToDevice, stream_));
            HIP_CHECK(hipMemcpyAsync(d_comb_ + n0, ext_in_ ? ext_in_ : d_in_, n_ * sizeof(Point),
                                     hipMemcpyDeviceToDevice, stream_));
            if (ckeys_cap_ < n0 + n_) {
                dev_release(d_ckeys_);
                dev_alloc_t(d_ckeys_, std::max<uint64_t>(n0 + n_, 1) * 4);
                ckeys_cap_ = n0 + n_;
            }
            k_comb_keys<<<grid_for(n0 + n_, 256), 256, 0, stream_>>>(d_ckeys_, ext_in_ ? ext_keys_ : keyed_ ? d_keys_ : nullptr,
                                                                    n0, nseeds_, n_);
            HIP_CHECK(hipGetLastError());
            comb_ok_ = true;
        }
        src_ = d_comb_;
        src_keys_ = d_ckeys_;
        nsrc_ = n0 + n_;
    } else {
        src_ = ext_in_ ? ext_in_ : d_in_;
        src_keys_ = ext_in_ ? ext_keys_ : keyed_ ? d_keys_ : nullptr;
        nsrc_ = n_;
    }
    if ((prior_ ? nseeds_ : 0) + n_ >= 0xFFFFFFFFull)
        return fail(-75, "more than 2^32-1 points (existing + new) per build are not supported");

    // arenas: SoA, ping-pong between levels.  A merge's levels also hold the
    // injected seeds of the touched cells (at most every existing point).
    const uint64_t acap = prior_ ? nseeds_ + n_ : nsrc_;
    if (dev_->cap < acap) {
        for (int a = 0; a < 2; a++) {
            Arena& A = dev_->ar[a];
            dev_release(A.p); dev_release(A.k);
            dev_alloc_t(A.p, acap * 16); dev_alloc_t(A.k, acap * 4);
        }
        dev_->cap = acap;
    }
    // file table for event batches
    {
        std::vector<uint32_t> ft;
        const uint64_t s0 = prior_ ? nseeds_ : 0;
        const uint32_t e0 = prior_ ? 1u : 0u;
        if (prior_) {   // pseudo file of the seeds: one batch, index 0
            ft.push_back(0);
            ft.push_back(0);
            ft.push_back(0);
            ft.push_back((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nseeds_, 0xFFFFFFFFull)));
        }
        for (size_t f = 0; f < file_start_.size(); f++) {
            const uint64_t st = file_start_[f] + s0;
            ft.push_back((uint32_t)st);
            ft.push_back((uint32_t)(st >> 32));
            ft.push_back(file_eb0_[f] + e0);
            ft.push_back(file_batch_[f]);
        }
        nfiles_dev_ = (uint32_t)(ft.size() / 4);
        dev_->files = static_cast<uint32_t*>(dev_->get(std::max<size_t>(ft.size(), 4) * 4));
        if (!ft.empty()) HIP_CHECK(hipMemcpyAsync(dev_->files, ft.data(), ft.size() * 4, hipMemcpyHostToDevice, stream_));
    }
    HIP_CHECK(hipMemsetAsync(dev_->ctr, 0, sizeof(Counters), stream_));

    nf_mode_ = false;
    ninf_ = 0;
    geom_fault_ = false;
    if (wide) {
        const int rcw = build_wide();
        stats_.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return rcw;
    }
    // the input as it stands (enter_nonfinite moves the infinite points apart):
    // what the sequential replay takes if the levels cannot be built in parallel
    const Point* src0 = src_;
    const uint32_t* keys0 = src_keys_;
    const uint64_t n0 = nsrc_;
    const bool can_replay = !prior_ && !h0_ && !max_levels_ && n0 <= kWideMax && getenv("PCC_NO_REPLAY") == nullptr;
    ev_begin(ST_L0);
    int rc = level0_bin();   // also computes the bounding box (converter.rs:96-104)
    if (rc && geom_fault_ && can_replay) {   // (see below: a level's geometry fault)
        rc = replay_whole(src0, keys0, n0, "level-0 cells and layers inconsistent at this magnitude");
        stats_.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return rc;
    }
    if (rc) return rc;
    stats_.ms_level0_bin = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t i = 0; !levels_.empty(); i++) {
        if (h0_ + i >= kMaxDepth) return fail(-75, "hierarchy depth limit (31) reached: more than cell_point_overflow_limit duplicate points?");
        const auto tl = std::chrono::steady_clock::now();
        rc = run_level(i);
        if (rc && geom_fault_ && can_replay) {
            // hexagon or slot indices saturated at a deep level (coordinates far
            // beyond the cell size, reachable through NaN-collapsed points): the
            // parallel slot geometry does not hold there, the reference's saturating
            // casts (hex.rs:67-85) do, so the whole build is replayed sequentially
            rc = replay_whole(src0, keys0, n0, "saturated hexagon indices");
            stats_.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            return rc;
        }
        if (rc) return rc;
        stats_.ms_level.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count());
        if (levels_.size() == i + 1) break;   // no next level
        if (max_levels_ && levels_.size() > max_levels_) {   // stop: the next level is exported, not built
            pending_ = levels_.back();
            levels_.pop_back();
            stats_.arrivals -= pending_->arrivals;
            stats_.cells -= pending_->ncells;
            stats_.slabs -= pending_->nslabs;
            break;
        }
    }
    hierarchies_ = std::max<uint32_t>(hierarchies_, h0_ + (uint32_t)levels_.size());
    stats_.levels = (uint32_t)levels_.size();
    rc = build_infinite();
    if (rc == kInfSaturated && can_replay) {   // finite cells that could meet the infinite points' ones
        rc = replay_whole(src0, keys0, n0, "finite coordinates saturating a cell index beside infinite ones");
        stats_.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return rc;
    }
    if (rc) return rc == kInfSaturated ? -22 : rc;
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

// H1: the level-1 histogram of the fused capacities (nullptr: plain level-0 histogram)
template <int BITS>
static void l0_pass(int p, int passes, Arena src, Arena dst, uint64_t n, const L0Params& P, int shift,
                    uint32_t* counts, uint32_t ntiles, uint32_t* hist, uint32_t D, Counters* ctr, const L1Grid& Q,
                    uint32_t* H1, uint32_t D1, ScanTemp& scan, hipStream_t st) {
    const uint64_t nc = (uint64_t)ntiles << BITS;
    if (p == 0 && H1) {
        k_l0_up_hist1<BITS><<<std::min<uint32_t>(ntiles, kL0DownGrid), kL0BS, 0, st>>>(src, n, P, Q, shift, counts, ntiles, H1, D1, ctr);
        k_l0_hist_from1<<<grid_for(D1, 256, 1u << 30), 256, 0, st>>>(H1, D1, P, Q, hist);
    } else if (p == 0) {
        k_l0_up_hist<BITS><<<std::min<uint32_t>(ntiles, 2048), kL0BS, 0, st>>>(src, n, P, shift, counts, ntiles, hist, D, ctr);
    } else {
        k_l0_up<BITS><<<ntiles, kL0BS, 0, st>>>(src, n, P, shift, counts, ntiles);
    }
    scan_excl_u32(counts, counts, (uint32_t)nc, nullptr, scan, st);
    k_l0_down<BITS, false, false><<<ntiles, kL0BS, 0, st>>>(nullptr, nullptr, src, dst, n, P, shift, counts, ntiles, nullptr, 0);
    HIP_CHECK(hipGetLastError());
}

// The level-0 parameters that do not depend on the bounding box.
static L0Params l0_base_params(const Config& cfg, uint32_t h0) {
    const uint32_t dim = cfg.sub_grid_dimension;
    const float cs = cell_size(cfg.max_cell_size, h0), csc = cell_size(cfg.max_cell_size, h0 + 1);
    L0Params P{};
    P.cs = cs;
    P.cr = hex_radius(sub_cell_size(cs, dim));
    P.csc = csc;
    P.crc = hex_radius(sub_cell_size(csc, dim));
    P.inv_cs = 1.0f / P.cs;
    P.inv_cr = 1.0f / P.cr;
    P.inv_csc = 1.0f / P.csc;
    P.inv_crc = 1.0f / P.crc;
    P.exact = 0;
    for (float v : {P.cs, P.cr, P.csc, P.crc})   // div_rc's divisor range
        if (!(std::fabs(v) >= 0x1p-60f && std::fabs(v) <= 0x1p60f)) P.exact = 1;
    P.nl = slab_geom(dim).nl;
    P.dim2 = 2 * (int32_t)dim;
    return P;
}

// Bounding box of one tile out of every ntiles / nb (block b: tile b * ntiles / nb).
__global__ __launch_bounds__(256) void k_bbox_sample(const Point* __restrict__ in, uint64_t n, uint64_t ntiles,
                                                     uint32_t nb, float* part) {
    const uint64_t t = (uint64_t)blockIdx.x * ntiles / nb;
    const float4* p4 = reinterpret_cast<const float4*>(in);
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint64_t i = t * kL0Tile + threadIdx.x; i < min((t + 1) * kL0Tile, n); i += 256) {
        const float4 v = p4[i];
        mn[0] = fminf(mn[0], v.x); mn[1] = fminf(mn[1], v.y); mn[2] = fminf(mn[2], v.z);
        mx[0] = fmaxf(mx[0], v.x); mx[1] = fmaxf(mx[1], v.y); mx[2] = fmaxf(mx[2], v.z);
    }
    __shared__ float s[4][6];
    for (int d = 32; d > 0; d >>= 1)
        for (int a = 0; a < 3; a++) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
        }
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; a++) { s[threadIdx.x / 64][a] = mn[a]; s[threadIdx.x / 64][3 + a] = mx[a]; }
    __syncthreads();
    if (threadIdx.x < 6) {
        float r = s[0][threadIdx.x];
        for (int q = 1; q < 4; q++) r = threadIdx.x < 3 ? fminf(r, s[q][threadIdx.x]) : fmaxf(r, s[q][threadIdx.x]);
        part[blockIdx.x * 6 + threadIdx.x] = r;
    }
}

// Level-0 pass 0 of the input uploaded so far (the complete tiles of its first
// `upto` points, or every tile when `all`), on the engine stream after `after`
// (the copy that brought them).  Only for a build whose source is the plain
// input (no merge seeds in front, no keyed input).
void Engine::pre0_count(uint64_t upto, hipEvent_t after, bool all) {
    if (prior_ || keyed_ || ext_in_ || h0_ != 0) return;
    if (pre6_run(upto, after, all)) return;
    const uint64_t t1 = all ? (upto + kL0Tile - 1) / kL0Tile : upto / kL0Tile;
    if (t1 <= pre_tiles_) return;
    if (!d_prepart_) {
        HIP_CHECK(hipMalloc(&d_prepart_, (1 + kPreBlocks) * 6 * sizeof(float)));
        HIP_CHECK(hipMalloc(&d_preflag_, 4));
    }
    if (pre_tiles_ == 0) {   // a fresh running box and flag
        static const float init[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
        HIP_CHECK(hipMemcpyAsync(d_prepart_, init, sizeof init, hipMemcpyHostToDevice, stream_));
        HIP_CHECK(hipMemsetAsync(d_preflag_, 0, 4, stream_));
    }
    if (t1 > tile6_cap_) {   // room for every tile of the reserved input
        const uint64_t cap = std::max<uint64_t>(t1, (cap_ + kL0Tile - 1) / kL0Tile);
        uint16_t* p = nullptr;
        HIP_CHECK(hipMalloc(&p, cap * 64 * sizeof(uint16_t)));
        if (pre_tiles_) HIP_CHECK(hipMemcpyAsync(p, d_tile6_, pre_tiles_ * 64 * sizeof(uint16_t), hipMemcpyDeviceToDevice, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        (void)hipFree(d_tile6_);
        d_tile6_ = p;
        tile6_cap_ = cap;
    }
    if (after) HIP_CHECK(hipStreamWaitEvent(stream_, after, 0));
    const uint32_t nb = (uint32_t)std::min<uint64_t>(t1 - pre_tiles_, kPreBlocks);
    k_l0_tiles0<<<nb, kL0BS, 0, stream_>>>(d_in_, upto, l0_base_params(cfg_, 0), pre_tiles_, t1, d_tile6_, d_prepart_,
                                           d_preflag_);
    k_bbox_final<<<1, 256, 0, stream_>>>(d_prepart_, nb + 1);
    HIP_CHECK(hipGetLastError());
    pre_tiles_ = t1;
}

void Engine::pre0_reset() {
    pre_tiles_ = 0;
    pre_decided_ = false;
    pre6_ = false;
    pre6_gdone_ = 0;
    landed_.clear();
    pre6_done_.clear();
    pre6_ndone_ = 0;
}

// pre0_count in its folded form: decides on the first landed piece (sample box
// of at most two level-0 cells per axis), then runs k_l0_tile6 over every group
// of tiles whose copy has landed.  Returns false when pass 0 runs instead.
bool Engine::pre6_run(uint64_t upto, hipEvent_t after, bool all) {
    if (!pre_decided_ && pre_tiles_ == 0) {
        const uint64_t landed = upto / kL0Tile;
        if (landed == 0 && !all) return true;   // decide once a tile has landed
        pre_decided_ = true;
        pre6_ = false;
        if (getenv("PCC_NO_PRE6") || getenv("PCC_NO_FOLD") || landed == 0) return false;
        if (after) HIP_CHECK(hipStreamWaitEvent(stream_, after, 0));
        const uint32_t nb = (uint32_t)std::min<uint64_t>(landed, 512);
        k_bbox_sample<<<nb, 256, 0, stream_>>>(d_in_, landed * kL0Tile, landed, nb, dev_->bbox_part);
        k_bbox_final<<<1, 256, 0, stream_>>>(dev_->bbox_part, nb);
        HIP_CHECK(hipGetLastError());
        float bb[6];
        HIP_CHECK(hipMemcpyAsync(bb, dev_->bbox_part, sizeof bb, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        const float cs = cell_size(cfg_.max_cell_size, 0);
        for (int a = 0; a < 3; a++) {
            if (!(std::isfinite(bb[a]) && std::isfinite(bb[3 + a]))) return false;
            if ((int64_t)cell_index1(bb[3 + a], cs) - (int64_t)cell_index1(bb[a], cs) >= 2) return false;
        }
        // room for the reserved input: run records, pair counts, the arenas
        pre6_tcap_ = (cap_ + kL0Tile - 1) / kL0Tile;
        pre6_tpg_ = (uint32_t)std::max<uint64_t>(1, (pre6_tcap_ + kL0Groups - 1) / kL0Groups);
        pre6_gcap_ = (uint32_t)((pre6_tcap_ + pre6_tpg_ - 1) / pre6_tpg_);
        if (pre6_alloc_tiles_ < pre6_tcap_) {
            dev_release(d_pre6_cnt_); dev_release(d_pre6_ph_);
            dev_alloc_t(d_pre6_cnt_, 64 * pre6_tcap_ * 4);
            dev_alloc_t(d_pre6_ph_, 64 * pre6_tcap_ * 4);
            pre6_alloc_tiles_ = pre6_tcap_;
        }
        if (pre6_alloc_groups_ < pre6_gcap_) {
            dev_release(d_pre6_gpar_);
            dev_alloc_t(d_pre6_gpar_, 64ull * pre6_gcap_ * 32 * 4);
            pre6_alloc_groups_ = pre6_gcap_;
        }
        if (dev_->cap < cap_) {
            for (int a = 0; a < 2; a++) {
                Arena& A = dev_->ar[a];
                dev_release(A.p); dev_release(A.k);
                dev_alloc_t(A.p, cap_ * 16); dev_alloc_t(A.k, cap_ * 4);
            }
            dev_->cap = cap_;
        }
        pre6_ar1_ = dev_->ar[1].p;
        if (!d_pre6_dummy_) dev_alloc_t(d_pre6_dummy_, 256ull * kL0BS * kL0IPT * 20);
        HIP_CHECK(hipMemsetAsync(dev_->bbox_flag, 0, 4, stream_));
        pre6_gdone_ = 0;
        pre6_src_ = d_in_;
        pre6_done_.clear();
        pre6_ = true;
    }
    if (!pre6_) return false;
    const uint64_t tl = all ? (upto + kL0Tile - 1) / kL0Tile : upto / kL0Tile;
    if (tl > pre6_tcap_) { pre6_ = false; return true; }   // beyond the reserved input: the build runs pass 1
    const uint32_t gend = (uint32_t)(all ? (tl + pre6_tpg_ - 1) / pre6_tpg_ : tl / pre6_tpg_);
    if (gend <= pre6_gdone_) return true;
    if (after) HIP_CHECK(hipStreamWaitEvent(stream_, after, 0));
    const uint32_t ntl = all ? (uint32_t)tl : gend * pre6_tpg_;
    const uint64_t n = all ? upto : (uint64_t)ntl * kL0Tile;
    // the arenas were sized for the input reserved when pass 1 was decided; a
    // later file grew the input (reserve) past them: the build runs pass 1
    if (n > dev_->cap || dev_->ar[1].p != pre6_ar1_) {
        pre6_ = false;
        return true;
    }
    Arena dummy{static_cast<float4*>(d_pre6_dummy_),
                reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_pre6_dummy_) + 256ull * kL0BS * kL0IPT * 16)};
    k_l0_tile6<false><<<gend - pre6_gdone_, kL0BS, 0, stream_>>>(d_in_, nullptr, dev_->ar[1], n, l0_base_params(cfg_, 0),
                                                                ntl, pre6_tpg_, pre6_gcap_, d_pre6_cnt_, d_pre6_ph_,
                                                                d_pre6_gpar_, dev_->bbox_part, dev_->bbox_flag, dummy,
                                                                pre6_gdone_, (uint32_t)pre6_tcap_);
    HIP_CHECK(hipGetLastError());
    pre6_gdone_ = gend;
    return true;
}

// Borrowed device input landing in pieces (a sharded rank's exchange, SURVEY
// §8e): the same level-0 pass 1 as behind a host upload (pre6_run), on every
// group of tiles whose points have all landed, in any order (a group's output,
// run records and pair counts depend on its own tiles only).  The fold is
// decided once, from the sample box of the first landed range.
int Engine::input_landed(uint64_t first, uint64_t last, hipStream_t after) {
    if (!ext_in_ || ext_keys_ || !event_table_ || prior_)   // (keyed input reads keys in pass 1: not this path)
        return fail(-22, "input_landed: the input must be borrowed with keys NULL and an event table, no merge");
    last = std::min<uint64_t>(last, n_);
    if (first >= last) return 0;
    if (after) {   // the engine's stream waits for the landing stream, the host does not
        if (!land_ev_) HIP_CHECK(hipEventCreateWithFlags(&land_ev_, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(land_ev_, after));
        HIP_CHECK(hipStreamWaitEvent(stream_, land_ev_, 0));
    }
    {   // merge [first, last) into the landed ranges
        auto& L = landed_;
        L.push_back({first, last});
        std::sort(L.begin(), L.end());
        std::vector<std::pair<uint64_t, uint64_t>> m;
        for (const auto& r : L) {
            if (!m.empty() && r.first <= m.back().second) m.back().second = std::max(m.back().second, r.second);
            else m.push_back(r);
        }
        L.swap(m);
    }
    const uint64_t ntiles = (n_ + kL0Tile - 1) / kL0Tile;
    if (!pre_decided_) {
        // the first range's whole tiles decide the fold (at most two level-0 cells per axis)
        const uint64_t t0 = (first + kL0Tile - 1) / kL0Tile, t1 = std::min<uint64_t>(last / kL0Tile, ntiles);
        if (t1 <= t0 && last < n_) return 0;   // decide once a whole tile has landed
        pre_decided_ = true;
        pre6_ = false;
        if (getenv("PCC_NO_PRE6") || getenv("PCC_NO_FOLD") || t1 <= t0) return 0;
        const uint64_t nt = t1 - t0;
        const uint32_t nb = (uint32_t)std::min<uint64_t>(nt, 512);
        k_bbox_sample<<<nb, 256, 0, stream_>>>(ext_in_ + t0 * kL0Tile, nt * kL0Tile, nt, nb, dev_->bbox_part);
        k_bbox_final<<<1, 256, 0, stream_>>>(dev_->bbox_part, nb);
        HIP_CHECK(hipGetLastError());
        float bb[6];
        HIP_CHECK(hipMemcpyAsync(bb, dev_->bbox_part, sizeof bb, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        const float cs = cell_size(cfg_.max_cell_size, 0);
        for (int a = 0; a < 3; a++) {
            if (!(std::isfinite(bb[a]) && std::isfinite(bb[3 + a]))) return 0;
            if ((int64_t)cell_index1(bb[3 + a], cs) - (int64_t)cell_index1(bb[a], cs) >= 2) return 0;
        }
        pre6_tcap_ = ntiles;
        pre6_tpg_ = (uint32_t)std::max<uint64_t>(1, (ntiles + kL0Groups - 1) / kL0Groups);
        pre6_gcap_ = (uint32_t)((ntiles + pre6_tpg_ - 1) / pre6_tpg_);
        if (pre6_alloc_tiles_ < pre6_tcap_) {
            dev_release(d_pre6_cnt_); dev_release(d_pre6_ph_);
            dev_alloc_t(d_pre6_cnt_, 64 * pre6_tcap_ * 4);
            dev_alloc_t(d_pre6_ph_, 64 * pre6_tcap_ * 4);
            pre6_alloc_tiles_ = pre6_tcap_;
        }
        if (pre6_alloc_groups_ < pre6_gcap_) {
            dev_release(d_pre6_gpar_);
            dev_alloc_t(d_pre6_gpar_, 64ull * pre6_gcap_ * 32 * 4);
            pre6_alloc_groups_ = pre6_gcap_;
        }
        if (pre6_glist_cap_ < pre6_gcap_) {
            dev_release(d_pre6_glist_);
            dev_alloc_t(d_pre6_glist_, (uint64_t)pre6_gcap_ * 4);
            pre6_glist_cap_ = pre6_gcap_;
        }
        if (dev_->cap < n_) {
            for (int a = 0; a < 2; a++) {
                Arena& A = dev_->ar[a];
                dev_release(A.p); dev_release(A.k);
                dev_alloc_t(A.p, n_ * 16); dev_alloc_t(A.k, n_ * 4);
            }
            dev_->cap = n_;
        }
        pre6_ar1_ = dev_->ar[1].p;
        if (!d_pre6_dummy_) dev_alloc_t(d_pre6_dummy_, 256ull * kL0BS * kL0IPT * 20);
        HIP_CHECK(hipMemsetAsync(dev_->bbox_flag, 0, 4, stream_));
        pre6_src_ = ext_in_;
        pre6_done_.assign(pre6_gcap_, 0);
        pre6_glist_.assign(pre6_gcap_, 0);
        pre6_ndone_ = 0;
        pre6_gdone_ = 0;
        pre6_ = true;
    }
    if (!pre6_ || pre6_src_ != ext_in_) return 0;
    // groups whose points have all landed and have not run
    std::vector<uint32_t> run;
    for (uint32_t g = 0; g < pre6_gcap_; g++) {
        if (pre6_done_[g]) continue;
        const uint64_t a = (uint64_t)g * pre6_tpg_ * kL0Tile;
        const uint64_t b = std::min<uint64_t>((uint64_t)(g + 1) * pre6_tpg_ * kL0Tile, n_);
        auto it = std::upper_bound(landed_.begin(), landed_.end(), std::make_pair(a, ~(uint64_t)0));
        if (it == landed_.begin()) continue;
        --it;
        if (it->first <= a && b <= it->second) run.push_back(g);
    }
    if (run.empty()) return 0;
    // every group runs once: the lists go one after another (no reuse, no wait)
    uint32_t* gl = d_pre6_glist_ + pre6_ndone_;
    std::copy(run.begin(), run.end(), pre6_glist_.begin() + pre6_ndone_);
    HIP_CHECK(hipMemcpyAsync(gl, pre6_glist_.data() + pre6_ndone_, run.size() * 4, hipMemcpyHostToDevice, stream_));
    Arena dummy{static_cast<float4*>(d_pre6_dummy_),
                reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_pre6_dummy_) + 256ull * kL0BS * kL0IPT * 16)};
    k_l0_tile6<false><<<(uint32_t)run.size(), kL0BS, 0, stream_>>>(ext_in_, nullptr, dev_->ar[1], n_,
                                                                  l0_base_params(cfg_, 0), (uint32_t)ntiles, pre6_tpg_,
                                                                  pre6_gcap_, d_pre6_cnt_, d_pre6_ph_, d_pre6_gpar_,
                                                                  dev_->bbox_part, dev_->bbox_flag, dummy, 0,
                                                                  (uint32_t)pre6_tcap_, gl);
    HIP_CHECK(hipGetLastError());
    for (uint32_t g : run) pre6_done_[g] = 1;
    pre6_ndone_ += run.size();
    return 0;
}

// ---- inputs with non-finite coordinates (kNfNan / kNfInf, see nf_class)
// Per block 15 floats: [0..5] min / max xyz over the non-NaN values of every
// point (f32::min/max skip NaN and keep infinities: bounding-volume/src/
// lib.rs:23-31); [6..8] 1 where the axis has a non-NaN value (otherwise the
// reference's box stays NaN there); [9..14] min / max over the points with no
// infinite coordinate, NaN taken as 0: the extent of the cells those points
// enter (cell index 0 on a NaN axis, metadata.rs:100-102).
constexpr int kNfParts = 15;
__global__ __launch_bounds__(256) void k_bbox_nf(const Point* __restrict__ in, uint64_t n, float* part) {
    float r[kNfParts];
    for (int a = 0; a < 3; a++) {
        r[a] = INFINITY; r[3 + a] = -INFINITY; r[6 + a] = 0.f; r[9 + a] = INFINITY; r[12 + a] = -INFINITY;
    }
    const float4* p4 = reinterpret_cast<const float4*>(in);
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const float4 v = p4[i];
        const float c[3] = {v.x, v.y, v.z};
        const bool fin = nf_class(v.x, v.y, v.z) != kNfInf;
        for (int a = 0; a < 3; a++) {
            r[a] = fminf(r[a], c[a]);
            r[3 + a] = fmaxf(r[3 + a], c[a]);
            r[6 + a] = isnan(c[a]) ? r[6 + a] : 1.f;
            const float g = isnan(c[a]) ? 0.f : c[a];
            if (fin) { r[9 + a] = fminf(r[9 + a], g); r[12 + a] = fmaxf(r[12 + a], g); }
        }
    }
    __shared__ float s[4][kNfParts];
    for (int k = 0; k < kNfParts; k++) {
        const bool mx = (k >= 3 && k < 9) || k >= 12;   // max-reduced slots (the flags too)
        for (int d = 32; d > 0; d >>= 1) {
            const float o = __shfl_xor(r[k], d, 64);
            r[k] = mx ? fmaxf(r[k], o) : fminf(r[k], o);
        }
    }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < kNfParts; k++) s[threadIdx.x / 64][k] = r[k];
    __syncthreads();
    if (threadIdx.x < (uint32_t)kNfParts) {
        const int k = threadIdx.x;
        const bool mx = (k >= 3 && k < 9) || k >= 12;
        float v = s[0][k];
        for (int q = 1; q < 4; q++) v = mx ? fmaxf(v, s[q][k]) : fminf(v, s[q][k]);
        part[blockIdx.x * kNfParts + k] = v;
    }
}
__global__ void k_bbox_nf_final(float* part, uint32_t nb) {   // one thread per slot
    const int k = threadIdx.x;
    if (k >= kNfParts) return;
    const bool mx = (k >= 3 && k < 9) || k >= 12;
    float v = part[k];
    for (uint32_t b = 1; b < nb; b++) v = mx ? fmaxf(v, part[b * kNfParts + k]) : fminf(v, part[b * kNfParts + k]);
    part[k] = v;
}

// Stable split of an input into the points without an infinite coordinate and
// those with one, each with its key (keys: the input's, else its index): per
// block of 1024 points the count of the latter, then the scatter.
__global__ __launch_bounds__(1024) void k_nf_count(const Point* __restrict__ in, uint64_t n, uint32_t* cnt) {
    __shared__ uint32_t c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    const uint64_t i = blockIdx.x * 1024ull + threadIdx.x;
    bool inf = false;
    if (i < n) { const float4 v = reinterpret_cast<const float4*>(in)[i]; inf = nf_class(v.x, v.y, v.z) == kNfInf; }
    const uint64_t m = __ballot(inf);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&c, (uint32_t)__popcll(m));
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = c;
}
__global__ __launch_bounds__(1024) void k_nf_scatter(const Point* __restrict__ in, const uint32_t* __restrict__ keys,
                                                     uint64_t n, const uint32_t* __restrict__ ibase, Point* fout,
                                                     uint32_t* fkeys, Point* iout, uint32_t* ikeys) {
    __shared__ uint32_t lds[1024 / 64 + 1];
    const uint64_t i = blockIdx.x * 1024ull + threadIdx.x;
    bool inf = false;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n) { v = reinterpret_cast<const float4*>(in)[i]; inf = nf_class(v.x, v.y, v.z) == kNfInf; }
    uint32_t tot;
    const uint32_t r = block_excl_scan<1024>(inf ? 1u : 0u, lds, &tot);
    if (i >= n) return;
    const uint32_t k = keys ? keys[i] : (uint32_t)i;
    const uint32_t ib = ibase[blockIdx.x];
    if (inf) {
        reinterpret_cast<float4*>(iout)[ib + r] = v;
        ikeys[ib + r] = k;
    } else {
        const uint64_t f = blockIdx.x * 1024ull - ib + threadIdx.x - r;
        reinterpret_cast<float4*>(fout)[f] = v;
        fkeys[f] = k;
    }
}

// ---- the points with an infinite coordinate.  Their cell index on that axis
// saturates at every level (metadata.rs:100-102, `as i32`), so they share no
// cell with the other points, their child cells are not 2c + bit on that axis,
// and within a cell they pile onto a few slots (hex.rs:67-85 with an infinite
// operand).  One sequential pass over them in key order follows the
// reference's per-batch recursion literally: converter.rs:114-139 (levels of
// one batch), cell.rs:70-94 (grid slot, `new < old` keeps the first on ties and
// NaN), cell.rs:108-153 (overflow entries: Vacant / Some / None per child).
// Rare by nature (a data error), so no parallel design: one lane, state in HBM.
constexpr uint32_t kInfNil = 0xFFFFFFFFu;
constexpr uint64_t kInfMax = 1ull << 18;   // points with an infinite coordinate per build
__global__ void k_iota_u32(uint32_t* k, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = (uint32_t)i;
}
struct InfCell {
    int32_t h, x, y, z;
    uint32_t total, number, overflow, nb;
    int32_t child[8][3];
    uint32_t st[8];                  // 0 Vacant (created by this batch), 1 Some, 2 None
    uint32_t len[8], head[8], tail[8];
    uint32_t stamp[8], cnt[8], mode[8];
};
struct InfOut {
    uint32_t ncells, ngrid, nnodes, err, hier;
    uint32_t pad;
    unsigned long long arrivals;
};
struct InfBufs {
    const Point* pts;
    const uint32_t* keys;
    uint32_t n;
    const uint32_t* files;
    uint32_t nfiles;
    InfCell* cells;
    int4* ckey;
    uint32_t* cval;
    int4* skey;
    uint32_t* sval;
    uint32_t hmask;                  // both hash tables: hmask + 1 entries
    Point* gp;                       // grid points in creation order, and their cells
    uint32_t* gcell;
    Point* np;                       // Some-list nodes
    uint32_t* nnext;
    Point* A;
    Point* B;
    Point* ov;                       // one level's overflow: point, cell, entry
    uint32_t* ovc;
    uint32_t* ovb;
    InfOut* out;
    float maxcs;
    uint32_t dim, limit;
};
__device__ __forceinline__ uint32_t inf_hash(int32_t a, int32_t b, int32_t c, int32_t d) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int32_t v : {a, b, c, d}) {
        h ^= (uint32_t)v;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 31;
    }
    return (uint32_t)h;
}
// the value slot of key k (inserted with kInfNil when absent: *fresh)
__device__ __forceinline__ uint32_t* inf_find(int4* keys, uint32_t* vals, uint32_t mask, int4 k, bool& fresh) {
    uint32_t i = inf_hash(k.x, k.y, k.z, k.w) & mask;
    for (;;) {
        if (vals[i] == kInfNil) {
            keys[i] = k;
            fresh = true;
            return &vals[i];
        }
        const int4 q = keys[i];
        if (q.x == k.x && q.y == k.y && q.z == k.z && q.w == k.w) {
            fresh = false;
            return &vals[i];
        }
        i = (i + 1) & mask;
    }
}
__global__ __launch_bounds__(64) void k_inf_build(InfBufs B) {
    if (threadIdx.x != 0) return;
    uint32_t ncells = 0, ngrid = 0, nbump = 0, nfree = kInfNil, err = 0, hier = 0, stamp = 0;
    unsigned long long arrivals = 0;
    for (uint32_t i0 = 0; i0 < B.n && !err;) {
        const uint32_t batch = event_batch(B.files, B.nfiles, B.keys[i0]);
        uint32_t i1 = i0 + 1;
        while (i1 < B.n && event_batch(B.files, B.nfiles, B.keys[i1]) == batch) i1++;
        const Point* cur = B.pts + i0;
        uint32_t ncur = i1 - i0;
        Point* nxt = B.A;
        for (uint32_t h = 0; ncur && !err; h++) {
            if (h >= kMaxDepth) { err |= 1u; break; }   // 2u32.pow(h) overflows (converter.rs:141-145)
            hier = max(hier, h + 1);
            stamp++;
            const float cs = cell_size(B.maxcs, h), cr = hex_radius(sub_cell_size(cs, B.dim));
            const float ccs = cell_size(B.maxcs, h + 1);
            uint32_t nov = 0;
            for (uint32_t k = 0; k < ncur; k++) {      // cell.rs:96-106, one cell after another
                const Point p = cur[k];
                bool fresh;
                uint32_t* cv = inf_find(B.ckey, B.cval, B.hmask,
                                        make_int4((int32_t)h, cell_index1(p.x, cs), cell_index1(p.y, cs), cell_index1(p.z, cs)),
                                        fresh);
                if (fresh) {
                    if (ncells >= B.n) { err |= 2u; break; }
                    InfCell& C = B.cells[ncells];
                    C.h = (int32_t)h;
                    C.x = cell_index1(p.x, cs); C.y = cell_index1(p.y, cs); C.z = cell_index1(p.z, cs);
                    C.total = C.number = C.overflow = C.nb = 0;
                    for (int j = 0; j < 8; j++) C.stamp[j] = 0;
                    *cv = ncells++;
                }
                const uint32_t cid = *cv;
                InfCell& C = B.cells[cid];
                arrivals++;
                const I3 o = hex_from_world(p.x, p.y, p.z, cr);
                uint32_t* sv = inf_find(B.skey, B.sval, B.hmask, make_int4((int32_t)cid, o.x, o.y, o.z), fresh);
                if (fresh) {
                    if (ngrid >= B.n) { err |= 2u; break; }
                    B.gp[ngrid] = p;
                    B.gcell[ngrid] = cid;
                    *sv = ngrid++;
                    C.total++;
                    C.number++;
                    continue;
                }
                float X, Y, Z;
                hex_to_world(o, cr, X, Y, Z);
                const Point old = B.gp[*sv];
                Point ovp = p;
                if (dist2(X, Y, Z, p.x, p.y, p.z) < dist2(X, Y, Z, old.x, old.y, old.z)) {
                    ovp = old;
                    B.gp[*sv] = p;
                }
                B.ov[nov] = ovp;
                B.ovc[nov] = cid;
                nov++;
            }
            // overflow entries (converter.rs:67-68 -> cell.rs:108-153): this
            // batch's count per (cell, child) first, then each entry's transition
            for (uint32_t k = 0; k < nov && !err; k++) {
                const Point q = B.ov[k];
                InfCell& C = B.cells[B.ovc[k]];
                const int32_t cx = cell_index1(q.x, ccs), cy = cell_index1(q.y, ccs), cz = cell_index1(q.z, ccs);
                uint32_t j = 0;
                while (j < C.nb && !(C.child[j][0] == cx && C.child[j][1] == cy && C.child[j][2] == cz)) j++;
                if (j == C.nb) {
                    if (j == 8) { err |= 4u; break; }
                    C.child[j][0] = cx; C.child[j][1] = cy; C.child[j][2] = cz;
                    C.st[j] = 0;
                    C.len[j] = 0;
                    C.head[j] = C.tail[j] = kInfNil;
                    C.stamp[j] = 0;
                    C.nb++;
                }
                if (C.stamp[j] != stamp) { C.stamp[j] = stamp; C.cnt[j] = 0; C.mode[j] = 0; }
                C.cnt[j]++;
                B.ovb[k] = j;
            }
            uint32_t nn = 0;
            for (uint32_t k = 0; k < nov && !err; k++) {
                InfCell& C = B.cells[B.ovc[k]];
                const uint32_t j = B.ovb[k];
                if (C.mode[j] == 0) {
                    const uint32_t c = C.cnt[j];
                    if (C.st[j] == 0) {                   // Vacant
                        if (c <= B.limit) { C.st[j] = 1; C.total += c; C.overflow += c; C.mode[j] = 1; }
                        else { C.st[j] = 2; C.mode[j] = 2; }
                    } else if (C.st[j] == 2) {            // Occupied(None)
                        C.mode[j] = 2;
                    } else if (C.len[j] + c < B.limit) {  // Occupied(Some), still below the limit
                        C.total += c; C.overflow += c; C.mode[j] = 1;
                    } else {                              // Some -> None: the old list goes first
                        C.total -= C.len[j]; C.overflow -= C.len[j];
                        for (uint32_t e = C.head[j]; e != kInfNil;) {
                            nxt[nn++] = B.np[e];
                            const uint32_t f = B.nnext[e];
                            B.nnext[e] = nfree;
                            nfree = e;
                            e = f;
                        }
                        C.st[j] = 2;
                        C.len[j] = 0;
                        C.head[j] = C.tail[j] = kInfNil;
                        C.mode[j] = 2;
                    }
                }
                if (C.mode[j] == 2) {
                    if (nn >= B.n) { err |= 2u; break; }
                    nxt[nn++] = B.ov[k];
                    continue;
                }
                uint32_t e;
                if (nfree != kInfNil) { e = nfree; nfree = B.nnext[e]; }
                else if (nbump < B.n) e = nbump++;
                else { err |= 2u; break; }
                B.np[e] = B.ov[k];
                B.nnext[e] = kInfNil;
                if (C.tail[j] == kInfNil) C.head[j] = e; else B.nnext[C.tail[j]] = e;
                C.tail[j] = e;
                C.len[j]++;
            }
            cur = nxt;
            ncur = nn;
            nxt = nxt == B.A ? B.B : B.A;
        }
        i0 = i1;
    }
    B.out->ncells = ncells;
    B.out->ngrid = ngrid;
    B.out->nnodes = nbump;
    B.out->err = err;
    B.out->hier = hier;
    B.out->arrivals = arrivals;
}

// An input with non-finite coordinates (flags from the first level-0 pass):
// the reference's bounding box (per axis over the non-NaN values, NaN where
// there are none), the extent of the cells the points without an infinite
// coordinate enter (NaN as 0), and, if some coordinate is infinite, those
// points split off from the rest with their keys (the rest are rebinned as
// keyed input).  Plain builds, merges (the existing cloud's seeds take part
// like any point; an existing cloud never has infinite coordinates: its
// metadata.json box would be null, which neither the reference nor pcc_open
// reads back) and keyed (sharded) builds; a level-range build returns an error.
int Engine::enter_nonfinite(uint32_t flags) {
    if (h0_ || max_levels_)
        return fail(-22, "input contains NaN or infinite coordinates (not supported in level-range builds)");
    const uint32_t nb = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((nsrc_ + 255) / 256, 1), kBBoxBlocks);
    float* part = static_cast<float*>(dev_->get((uint64_t)nb * kNfParts * 4));
    k_bbox_nf<<<nb, 256, 0, stream_>>>(src_, nsrc_, part);
    k_bbox_nf_final<<<1, 64, 0, stream_>>>(part, nb);
    HIP_CHECK(hipGetLastError());
    float r[kNfParts];
    HIP_CHECK(hipMemcpyAsync(r, part, sizeof r, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (int a = 0; a < 3; a++) {
        bmin_[a] = r[6 + a] != 0.f ? r[a] : NAN;
        bmax_[a] = r[6 + a] != 0.f ? r[3 + a] : NAN;
        gmin_[a] = r[9 + a];
        gmax_[a] = r[12 + a];
    }
    if (flags & kNfInf) {
        const uint64_t nbk = (nsrc_ + 1023) / 1024;
        uint32_t* cnt = static_cast<uint32_t*>(dev_->get(nbk * 4 + 16));
        uint32_t* tot = cnt + nbk + 1;
        k_nf_count<<<(uint32_t)nbk, 1024, 0, stream_>>>(src_, nsrc_, cnt);
        scan_excl_u32(cnt, cnt, (uint32_t)nbk, tot, dev_->scan, stream_);
        uint32_t ni = 0;
        HIP_CHECK(hipMemcpyAsync(&ni, tot, 4, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        const uint64_t nf = nsrc_ - ni;
        if (nf_cap_ < nf) {
            dev_release(d_nf_pts_); dev_release(d_nf_keys_);
            dev_alloc_t(d_nf_pts_, std::max<uint64_t>(nf, 1) * sizeof(Point));
            dev_alloc_t(d_nf_keys_, std::max<uint64_t>(nf, 1) * 4);
            nf_cap_ = nf;
        }
        if (inf_cap_ < ni) {
            dev_release(d_inf_pts_); dev_release(d_inf_keys_);
            dev_alloc_t(d_inf_pts_, std::max<uint64_t>(ni, 1) * sizeof(Point));
            dev_alloc_t(d_inf_keys_, std::max<uint64_t>(ni, 1) * 4);
            inf_cap_ = ni;
        }
        k_nf_scatter<<<(uint32_t)nbk, 1024, 0, stream_>>>(src_, src_keys_, nsrc_, cnt, d_nf_pts_, d_nf_keys_, d_inf_pts_,
                                                          d_inf_keys_);
        HIP_CHECK(hipGetLastError());
        src_ = d_nf_pts_;
        src_keys_ = d_nf_keys_;
        nsrc_ = nf;
        ninf_ = ni;
    }
    nf_mode_ = true;
    return 0;
}

// The cells of the points with an infinite coordinate (k_inf_build) as host
// cell files.  The other points' cells never saturate an index at the levels
// built (checked here), so the two sets of cells are disjoint.
int Engine::build_infinite() {
    side_.clear();
    if (ninf_ == 0) return 0;
    if (ninf_ > kInfMax) return fail(-22, "more than 2^18 points with infinite coordinates in one build are not supported");
    if (nsrc_ || (prior_ && nseeds_)) {
        float m = prior_ ? prior_max_abs_ : 0.f;   // a merge: every existing cell too
        if (nsrc_)
            for (int a = 0; a < 3; a++) m = std::max(m, std::max(std::fabs(gmin_[a]), std::fabs(gmax_[a])));
        const uint32_t hl = h0_ + (uint32_t)std::max<size_t>(std::max<size_t>(levels_.size(), prior_ ? pdev_.size() : 0), 1) - 1;
        if (!(m / cell_size(cfg_.max_cell_size, hl) < 1.0e9f)) {
            fail(-22, "finite coordinates that saturate a cell index mixed with infinite ones are not supported "
                      "(in a merge, a level range, or beyond 2^24 points)");
            return kInfSaturated;
        }
    }
    return replay_seq(d_inf_pts_, d_inf_keys_, ninf_);
}

// Sub-grid dimensions beyond the dense slot table (> 96; the reference allows
// any, metadata.rs:17-18): every point through the sequential replay of the
// reference's per-batch recursion (k_inf_build: one lane, cell and slot hash
// tables in HBM), cells as side cells.  A correctness path, not a fast one:
// about 1 M arrivals per second.  The bounding box in the reference's form
// (k_bbox_nf: NaN skipped, infinities kept).
// The whole build as the sequential replay (k_inf_build over every point),
// after a parallel attempt that hit geometry it cannot express: the levels and
// statistics of that attempt are dropped, the input is the one it started from.
int Engine::replay_whole(const Point* src, const uint32_t* keys, uint64_t n, const char* why) {
    if (getenv("PCC_VERBOSE")) fprintf(stderr, "[pcc] sequential replay of the whole build: %s\n", why);
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (Level* l : levels_) delete l;
    levels_.clear();
    side_.clear();
    stats_ = BuildStats();
    hierarchies_ = nbatches_ > 0 ? 1u : 0u;
    HIP_CHECK(hipMemsetAsync(dev_->ctr, 0, sizeof(Counters), stream_));
    src_ = src;
    src_keys_ = keys;
    nsrc_ = n;
    nf_mode_ = false;
    ninf_ = 0;
    err_.clear();
    const int rc = build_wide();
    stats_.seq_replay = 1;
    return rc;
}

int Engine::build_wide() {
    if (nsrc_ > kWideMax) return fail(-22, "sub_grid_dimension > 96: more than 2^24 points per build are not supported");
    const uint32_t nb = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((nsrc_ + 255) / 256, 1), kBBoxBlocks);
    float* part = static_cast<float*>(dev_->get((uint64_t)nb * kNfParts * 4));
    k_bbox_nf<<<nb, 256, 0, stream_>>>(src_, nsrc_, part);
    k_bbox_nf_final<<<1, 64, 0, stream_>>>(part, nb);
    HIP_CHECK(hipGetLastError());
    float r[kNfParts];
    HIP_CHECK(hipMemcpyAsync(r, part, sizeof r, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (int a = 0; a < 3; a++) {
        bmin_[a] = r[6 + a] != 0.f ? r[a] : NAN;
        bmax_[a] = r[6 + a] != 0.f ? r[3 + a] : NAN;
    }
    const uint32_t* keys = src_keys_;
    if (!keys) {   // plain or event-table input: the keys are the indices
        uint32_t* k = static_cast<uint32_t*>(dev_->get(nsrc_ * 4));
        k_iota_u32<<<grid_for(nsrc_, 256), 256, 0, stream_>>>(k, nsrc_);
        HIP_CHECK(hipGetLastError());
        keys = k;
    }
    const int rc = replay_seq(src_, keys, nsrc_);
    stats_.levels = hierarchies_;
    stats_.seq_replay = 1;
    return rc;
}

int Engine::replay_seq(const Point* pts, const uint32_t* keys, uint64_t npts) {
    const uint32_t n = (uint32_t)npts;
    uint32_t hc = 16;
    while (hc < 2 * n) hc <<= 1;
    InfBufs B{};
    B.pts = pts;
    B.keys = keys;
    B.n = n;
    B.files = dev_->files;
    B.nfiles = nfiles_dev_;
    B.cells = static_cast<InfCell*>(dev_->get((uint64_t)n * sizeof(InfCell)));
    B.ckey = static_cast<int4*>(dev_->get((uint64_t)hc * 16));
    B.cval = static_cast<uint32_t*>(dev_->get((uint64_t)hc * 4));
    B.skey = static_cast<int4*>(dev_->get((uint64_t)hc * 16));
    B.sval = static_cast<uint32_t*>(dev_->get((uint64_t)hc * 4));
    B.hmask = hc - 1;
    B.gp = static_cast<Point*>(dev_->get((uint64_t)n * 16));
    B.gcell = static_cast<uint32_t*>(dev_->get((uint64_t)n * 4));
    B.np = static_cast<Point*>(dev_->get((uint64_t)n * 16));
    B.nnext = static_cast<uint32_t*>(dev_->get((uint64_t)n * 4));
    B.A = static_cast<Point*>(dev_->get((uint64_t)n * 16));
    B.B = static_cast<Point*>(dev_->get((uint64_t)n * 16));
    B.ov = static_cast<Point*>(dev_->get((uint64_t)n * 16));
    B.ovc = static_cast<uint32_t*>(dev_->get((uint64_t)n * 4));
    B.ovb = static_cast<uint32_t*>(dev_->get((uint64_t)n * 4));
    B.out = static_cast<InfOut*>(dev_->get(sizeof(InfOut)));
    B.maxcs = cfg_.max_cell_size;
    B.dim = cfg_.sub_grid_dimension;
    B.limit = cfg_.cell_point_overflow_limit;
    HIP_CHECK(hipMemsetAsync(B.cval, 0xFF, (uint64_t)hc * 4, stream_));
    HIP_CHECK(hipMemsetAsync(B.sval, 0xFF, (uint64_t)hc * 4, stream_));
    k_inf_build<<<1, 64, 0, stream_>>>(B);
    HIP_CHECK(hipGetLastError());
    InfOut o;
    HIP_CHECK(hipMemcpyAsync(&o, B.out, sizeof o, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    if (o.err & 1u) return fail(-75, "hierarchy depth limit (31) reached: more than cell_point_overflow_limit duplicate points?");
    if (o.err) return fail(-34, "infinite-coordinate build: capacity exceeded (internal error)");
    std::vector<InfCell> cells(o.ncells);
    std::vector<Point> gp(o.ngrid), np(o.nnodes);
    std::vector<uint32_t> gcell(o.ngrid), nnext(o.nnodes);
    if (o.ncells) HIP_CHECK(hipMemcpyAsync(cells.data(), B.cells, (uint64_t)o.ncells * sizeof(InfCell), hipMemcpyDeviceToHost, stream_));
    if (o.ngrid) {
        HIP_CHECK(hipMemcpyAsync(gp.data(), B.gp, (uint64_t)o.ngrid * 16, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipMemcpyAsync(gcell.data(), B.gcell, (uint64_t)o.ngrid * 4, hipMemcpyDeviceToHost, stream_));
    }
    if (o.nnodes) {
        HIP_CHECK(hipMemcpyAsync(np.data(), B.np, (uint64_t)o.nnodes * 16, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipMemcpyAsync(nnext.data(), B.nnext, (uint64_t)o.nnodes * 4, hipMemcpyDeviceToHost, stream_));
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
    side_.resize(o.ncells);
    uint64_t kept = 0;
    for (uint32_t c = 0; c < o.ncells; c++) {
        const InfCell& C = cells[c];
        CellFile& f = side_[c];
        f.h = (uint32_t)C.h;
        f.idx[0] = C.x; f.idx[1] = C.y; f.idx[2] = C.z;
        f.total = C.total; f.number = C.number; f.overflow = C.overflow;
        for (uint32_t j = 0; j < C.nb; j++) {
            CellFile::Entry e;
            for (int a = 0; a < 3; a++) e.child[a] = C.child[j][a];
            e.some = C.st[j] == 1;
            if (e.some)
                for (uint32_t q = C.head[j]; q != kInfNil; q = nnext[q]) e.pts.push_back(np[q]);
            kept += e.pts.size();
            f.entries.push_back(std::move(e));
        }
    }
    for (uint32_t g = 0; g < o.ngrid; g++) side_[gcell[g]].grid.push_back(gp[g]);
    stats_.cells += o.ncells;
    stats_.grid_points += o.ngrid;
    stats_.kept_points += kept;
    stats_.arrivals += o.arrivals;
    hierarchies_ = std::max<uint32_t>(hierarchies_, o.hier);
    return 0;
}

// Whether to fold level-0 pass 0 into pass 1 (k_l0_tile6): the grid must have at
// most two level-0 cells per axis.  Judged from the bounding box of a sample of
// 512 tiles (the exact box decides after the pass; a wrong guess costs that
// pass, then the three-pass binning runs).
// Pass 2 of the folded binning (tile-major pass-1 output): 32 high digits (cell
// parities) or 256 (cells modulo 4); 16-bit in-tile keys unless keys were given.
static void l0_pass2_tm(int fcb, bool keys, uint32_t nblocks, Arena src, Arena dst, const L0Params& P,
                        const L0Unit* units, const uint32_t* starts, uint32_t ngroups, const uint32_t* gcnt,
                        const uint32_t* cnt_scan, const uint32_t* sflag, uint32_t D, uint32_t* dcap, Arena dummy,
                        Counters* ctr, const L0UnitW* uw, const uint2* wt, const uint32_t* cnt6, const uint32_t* ph6,
                        uint32_t ntiles, hipStream_t st) {
    if (fcb == 6 && keys)
        k_l0_down5g<256, true, false><<<nblocks, kL0BS, 0, st>>>(src, dst, P, units, starts, ngroups, gcnt, cnt_scan, sflag,
                                                                 D, dcap, dummy, ctr, uw, wt, cnt6, ph6, ntiles);
    else if (fcb == 6)
        k_l0_down5g<256, true, true><<<nblocks, kL0BS, 0, st>>>(src, dst, P, units, starts, ngroups, gcnt, cnt_scan, sflag,
                                                                D, dcap, dummy, ctr, uw, wt, cnt6, ph6, ntiles);
    else if (keys)
        k_l0_down5g<32, true, false><<<nblocks, kL0BS, 0, st>>>(src, dst, P, units, starts, ngroups, gcnt, cnt_scan, sflag,
                                                                D, dcap, dummy, ctr, uw, wt, cnt6, ph6, ntiles);
    else
        k_l0_down5g<32, true, true><<<nblocks, kL0BS, 0, st>>>(src, dst, P, units, starts, ngroups, gcnt, cnt_scan, sflag,
                                                               D, dcap, dummy, ctr, uw, wt, cnt6, ph6, ntiles);
}

// The folded binning's cell bits from a sample of the tiles' bounding box: 3
// (at most two level-0 cells per axis), 6 (at most four), 0 (no fold).
int Engine::fold_hint(float cs) {
    const uint64_t ntiles = (nsrc_ + kL0Tile - 1) / kL0Tile;
    if (ntiles == 0) return 0;
    const uint32_t nb = (uint32_t)std::min<uint64_t>(ntiles, 512);
    k_bbox_sample<<<nb, 256, 0, stream_>>>(src_, nsrc_, ntiles, nb, dev_->bbox_part);
    k_bbox_final<<<1, 256, 0, stream_>>>(dev_->bbox_part, nb);
    HIP_CHECK(hipGetLastError());
    float bb[6];
    HIP_CHECK(hipMemcpyAsync(bb, dev_->bbox_part, sizeof bb, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    int64_t ext = 0;
    for (int a = 0; a < 3; a++) {
        if (!(std::isfinite(bb[a]) && std::isfinite(bb[3 + a]))) return 0;
        ext = std::max<int64_t>(ext, (int64_t)cell_index1(bb[3 + a], cs) - (int64_t)cell_index1(bb[a], cs));
    }
    return ext < 2 ? 3 : (ext < 4 && getenv("PCC_NO_FOLD4") == nullptr) ? 6 : 0;
}

int Engine::level0_bin() {
    if (nf_mode_ && nsrc_ == 0) {   // every point has an infinite coordinate: no finite cells
        ev_end(ST_L0);
        return 0;
    }
    const uint32_t dim = cfg_.sub_grid_dimension;
    const float cs = cell_size(cfg_.max_cell_size, h0_), csc = cell_size(cfg_.max_cell_size, h0_ + 1);
    L0Params P;
    P.cs = cs;
    P.cr = hex_radius(sub_cell_size(cs, dim));
    P.csc = csc;
    P.crc = hex_radius(sub_cell_size(csc, dim));
    P.inv_cs = 1.0f / P.cs;
    P.inv_cr = 1.0f / P.cr;
    P.inv_csc = 1.0f / P.csc;
    P.inv_crc = 1.0f / P.crc;
    P.exact = 0;
    for (float v : {P.cs, P.cr, P.csc, P.crc})   // div_rc's divisor range
        if (!(std::fabs(v) >= 0x1p-60f && std::fabs(v) <= 0x1p60f)) P.exact = 1;
    const SlabGeom g = slab_geom(dim);
    P.nl = g.nl;
    P.dim2 = 2 * (int32_t)dim;
    if (P.nl > (int32_t)kL0Layers) return fail(-22, "sub_grid_dimension too large for the level-0 layer field");
    uint64_t G = 1;
    bool wide = false;
    P.hashed = 0;
    P.hmask = 0;
    P.hkeys = nullptr;
    P.hcid = nullptr;
    P.ckeys = nullptr;
    // Pass 0 (low 6 bits of the layer: no grid needed) fused with the bounding
    // box, per group of consecutive tiles: k_l0_down6g's blocks walk the same
    // groups with running offsets, so no per-tile counts exist.
    const uint32_t ntiles = (uint32_t)((nsrc_ + kL0Tile - 1) / kL0Tile);
    // pass 1 already run behind the upload (pre6_run) for this very input
    // pass-1 digits (the low 6 layer bits) and pass-2 digits (cell parity + 2 layer
    // bits); a 5 + 6 split (pass-2 runs of ~96 points, 64 pass-2 digits) measured
    // slower in round 4 (level 0 16.6-17.3 against 16.1-17.0 ms, same boxes)
    constexpr int lb = 6;
    constexpr uint32_t R1 = 1u << lb, HB = (uint32_t)(kL0LayerBits - lb);
    const bool landing = !pre6_done_.empty();   // pass 1 ran on landed groups of a borrowed input
    const bool p6 = pre6_ && ntiles && src_ == pre6_src_ && nsrc_ == n_ && !prior_ &&
                    (landing ? (ext_in_ && !ext_keys_ && event_table_ && ntiles == pre6_tcap_)
                             : (!keyed_ && !ext_in_ && src_ == d_in_)) &&
                    h0_ == 0 && !nf_mode_ && dev_->ar[1].p == pre6_ar1_ && ntiles <= pre6_tcap_ &&
                    getenv("PCC_NO_FOLD") == nullptr;
    pre6_ = false;   // (consumed: later levels overwrite the arena)
    // fcb: the fold's cell bits (k_l0_tile6 CB); pass 2 then has (1 << fcb) << HB digits
    const int fcb = (ntiles && !nf_mode_ && getenv("PCC_NO_FOLD") == nullptr) ? (p6 ? 3 : fold_hint(cs)) : 0;
    const uint32_t r2f = fcb ? (1u << fcb) << HB : 0u;
    // (the modulo-4 fold's pair tables are 64 KB per group, written by pass 1 and
    // scanned over the groups: at most kL0Groups6 groups)
    const char* gq = getenv(fcb == 6 ? "PCC_L0_GROUPS6" : "PCC_L0_GROUPS");
    uint32_t ngroups = std::max<uint32_t>(1, std::min<uint32_t>(gq ? std::max<uint32_t>(1, (uint32_t)strtoul(gq, nullptr, 10))
                                                                   : fcb == 6 ? kL0Groups6 : kL0Groups,
                                                                std::min<uint32_t>(ntiles, kBBoxBlocks)));
    const uint32_t tpg = p6 ? pre6_tpg_ : std::max<uint32_t>(1, (ntiles + ngroups - 1) / ngroups);
    ngroups = std::max<uint32_t>(1, (ntiles + tpg - 1) / tpg);
    uint32_t* gcnt0 = static_cast<uint32_t*>(dev_->get(64ull * ngroups * 4 + 64));
    Arena l0dummy{static_cast<float4*>(dev_->get(256ull * kL0BS * kL0IPT * 16)),
                  static_cast<uint32_t*>(dev_->get(256ull * kL0BS * kL0IPT * 4))};
    const bool l0keys = src_keys_ != nullptr;
    // Pass 0 folded into pass 1 (k_l0_tile6) when the grid is expected to have at
    // most two level-0 cells per axis (judged from a sample of the tiles' bounding
    // box; the full box after the pass decides, else the three-pass binning runs).
    bool fold = false;
    int rc = 0;
    uint32_t* cnt6 = nullptr;
    uint32_t* ph6 = nullptr;
    uint32_t* gpar = nullptr;
    if (fcb) {
        cnt6 = static_cast<uint32_t*>(dev_->get(64ull * ntiles * 4));
        ph6 = static_cast<uint32_t*>(dev_->get(64ull * ntiles * 4));
        gpar = static_cast<uint32_t*>(dev_->get(64ull * ngroups * r2f * 4));
        if (p6) {
            // the groups the upload did not complete, then the run records and
            // pair counts in this build's layout (rows of ntiles / ngroups)
            if (landing) {   // the groups whose points had not all landed
                const uint64_t n0 = pre6_ndone_;
                for (uint32_t g = 0; g < ngroups; g++)
                    if (!pre6_done_[g]) pre6_glist_[pre6_ndone_++] = g;
                if (pre6_ndone_ > n0) {
                    HIP_CHECK(hipMemcpyAsync(d_pre6_glist_ + n0, pre6_glist_.data() + n0, (pre6_ndone_ - n0) * 4,
                                             hipMemcpyHostToDevice, stream_));
                    k_l0_tile6<false><<<(uint32_t)(pre6_ndone_ - n0), kL0BS, 0, stream_>>>(
                        src_, nullptr, dev_->ar[1], nsrc_, P, ntiles, tpg, pre6_gcap_, d_pre6_cnt_, d_pre6_ph_,
                        d_pre6_gpar_, dev_->bbox_part, dev_->bbox_flag, l0dummy, 0, (uint32_t)pre6_tcap_,
                        d_pre6_glist_ + n0);
                }
                pre6_ndone_ = n0;   // (the tiles pass 1 ran on while the input landed)
            } else if (ngroups > pre6_gdone_) {
                k_l0_tile6<false><<<ngroups - pre6_gdone_, kL0BS, 0, stream_>>>(
                    src_, nullptr, dev_->ar[1], nsrc_, P, ntiles, tpg, pre6_gcap_, d_pre6_cnt_, d_pre6_ph_, d_pre6_gpar_,
                    dev_->bbox_part, dev_->bbox_flag, l0dummy, pre6_gdone_, (uint32_t)pre6_tcap_);
            }
            HIP_CHECK(hipMemcpy2DAsync(cnt6, (size_t)ntiles * 4, d_pre6_cnt_, (size_t)pre6_tcap_ * 4, (size_t)ntiles * 4, 64,
                                       hipMemcpyDeviceToDevice, stream_));
            HIP_CHECK(hipMemcpy2DAsync(ph6, (size_t)ntiles * 4, d_pre6_ph_, (size_t)pre6_tcap_ * 4, (size_t)ntiles * 4, 64,
                                       hipMemcpyDeviceToDevice, stream_));
            HIP_CHECK(hipMemcpy2DAsync(gpar, (size_t)ngroups * 128, d_pre6_gpar_, (size_t)pre6_gcap_ * 128,
                                       (size_t)ngroups * 128, 64, hipMemcpyDeviceToDevice, stream_));
        } else {
        HIP_CHECK(hipMemsetAsync(dev_->bbox_flag, 0, 4, stream_));
        if (l0keys && fcb == 6)
            k_l0_tile6<true, 6, 6><<<ngroups, kL0BS, 0, stream_>>>(src_, src_keys_, dev_->ar[1], nsrc_, P, ntiles, tpg,
                                                                   ngroups, cnt6, ph6, gpar, dev_->bbox_part,
                                                                   dev_->bbox_flag, l0dummy, 0, ntiles);
        else if (fcb == 6)
            k_l0_tile6<false, 6, 6><<<ngroups, kL0BS, 0, stream_>>>(src_, nullptr, dev_->ar[1], nsrc_, P, ntiles, tpg,
                                                                    ngroups, cnt6, ph6, gpar, dev_->bbox_part,
                                                                    dev_->bbox_flag, l0dummy, 0, ntiles);
        else if (l0keys)
            k_l0_tile6<true><<<ngroups, kL0BS, 0, stream_>>>(src_, src_keys_, dev_->ar[1], nsrc_, P, ntiles, tpg, ngroups,
                                                             cnt6, ph6, gpar, dev_->bbox_part, dev_->bbox_flag, l0dummy,
                                                             0, ntiles);
        else
            k_l0_tile6<false><<<ngroups, kL0BS, 0, stream_>>>(src_, nullptr, dev_->ar[1], nsrc_, P, ntiles, tpg, ngroups,
                                                              cnt6, ph6, gpar, dev_->bbox_part, dev_->bbox_flag, l0dummy,
                                                              0, ntiles);
        }
        k_bbox_final<<<1, 256, 0, stream_>>>(dev_->bbox_part, ngroups);
        HIP_CHECK(hipGetLastError());
        float bb[6];
        uint32_t bad = 0;
        readback({{bb, dev_->bbox_part, sizeof bb}, {&bad, dev_->bbox_flag, 4}});
        if (bad & ~kNfLayer) {   // non-finite coordinates: the exact boxes, infinite points apart, then again
            rc = enter_nonfinite(bad);
            return rc ? rc : level0_bin();
        }
        if (bad) return geom_fail("level-0 binning: layer outside the cell (internal error)");
        fold = true;
        for (int a = 0; a < 3; a++) {
            bmin_[a] = bb[a];
            bmax_[a] = bb[3 + a];
            fold &= (int64_t)cell_index1(bmax_[a], cs) - (int64_t)cell_index1(bmin_[a], cs) < (fcb == 3 ? 2 : 4);
        }
        stats_.pre0_tiles = p6 ? std::min<uint64_t>((uint64_t)(landing ? pre6_ndone_ : pre6_gdone_) * tpg, ntiles) : 0;
    }
    stats_.l0_fold = fold ? (uint32_t)fcb : 0u;
    if (!fold) {
        // the input's tiles already counted while it uploaded (pre0_count): count
        // the rest, then only sum the tiles per group
        const bool pre = pre_tiles_ > 0 && src_ == d_in_ && nsrc_ == n_ && !prior_ && !keyed_ && h0_ == 0 &&
                         getenv("PCC_NO_PRE0") == nullptr;
        if (pre) {
            pre0_count(n_, nullptr, true);
            k_l0_group_from_tiles<<<(ngroups * 64 + 255) / 256, 256, 0, stream_>>>(d_tile6_, ntiles, tpg, ngroups, gcnt0);
            HIP_CHECK(hipMemcpyAsync(dev_->bbox_part, d_prepart_, 6 * sizeof(float), hipMemcpyDeviceToDevice, stream_));
            HIP_CHECK(hipMemcpyAsync(dev_->bbox_flag, d_preflag_, 4, hipMemcpyDeviceToDevice, stream_));
            stats_.pre0_tiles = pre_tiles_;
        } else {
            HIP_CHECK(hipMemsetAsync(dev_->bbox_flag, 0, 4, stream_));
            k_l0_up0g<<<ngroups, kL0BS, 0, stream_>>>(src_, nsrc_, P, tpg, ngroups, gcnt0, dev_->bbox_part, dev_->bbox_flag);
            k_bbox_final<<<1, 256, 0, stream_>>>(dev_->bbox_part, ngroups);
            stats_.pre0_tiles = 0;
        }
        HIP_CHECK(hipGetLastError());
        float bb[6];
        uint32_t bad = 0;
        readback({{bb, dev_->bbox_part, sizeof bb}, {&bad, dev_->bbox_flag, 4}});
        if (!nf_mode_) {
            if (bad & ~kNfLayer) {   // non-finite coordinates: the exact boxes, infinite points apart, then again
                const int rc = enter_nonfinite(bad);
                return rc ? rc : level0_bin();
            }
            for (int a = 0; a < 3; a++) { bmin_[a] = bb[a]; bmax_[a] = bb[3 + a]; }
        }
    }
    const float* glo = nf_mode_ ? gmin_ : bmin_;   // the extent the level-0 grid must cover
    const float* ghi = nf_mode_ ? gmax_ : bmax_;
    for (int a = 0; a < 3; a++) {
        P.lo[a] = cell_index1(glo[a], cs);
        const int64_t ext = (int64_t)cell_index1(ghi[a], cs) - P.lo[a] + 1;
        wide |= ext > (1 << 21);
        P.g[a] = (int32_t)std::min<int64_t>(ext, INT32_MAX);
        G *= (uint64_t)ext;
    }
    if (wide)
        return fail(-27, "level-0 cell grid too large (bounding box spans > 2^21 cells of max_cell_size on an axis)");
    if (G > (1u << 20)) {
        // sparse bounding box: hash set of the occupied level-0 cells, compact ids
        P.hashed = 1;
        uint32_t* cnt = static_cast<uint32_t*>(dev_->get(8));
        for (uint64_t cap = 1u << 20;; cap <<= 1) {
            if (cap > (1ull << 31)) return fail(-27, "too many occupied level-0 cells");
            P.hmask = (uint32_t)(cap - 1);
            unsigned long long* hk = static_cast<unsigned long long*>(dev_->get(cap * 8));
            HIP_CHECK(hipMemsetAsync(hk, 0xFF, cap * 8, stream_));
            HIP_CHECK(hipMemsetAsync(cnt, 0, 8, stream_));
            k_l0_hash_insert<<<grid_for(nsrc_, 256, 8192), 256, 0, stream_>>>(src_, nsrc_, P, hk, cnt, cnt + 1);
            HIP_CHECK(hipGetLastError());
            uint32_t hc2[2];
            HIP_CHECK(hipMemcpyAsync(hc2, cnt, 8, hipMemcpyDeviceToHost, stream_));
            HIP_CHECK(hipStreamSynchronize(stream_));
            if (hc2[1] & 1u) return geom_fail("level-0 binning: point outside the bounding grid (internal error)");
            if ((hc2[1] & 2u) || hc2[0] > cap * 6 / 10) continue;   // too full: grow and rebuild
            uint32_t* hcid = static_cast<uint32_t*>(dev_->get(cap * 4));
            k_l0_hash_flags<<<grid_for(cap, 256, 1u << 30), 256, 0, stream_>>>(hk, (uint32_t)cap, hcid);
            scan_excl_u32(hcid, hcid, (uint32_t)cap, cnt, dev_->scan, stream_);
            unsigned long long* ck = static_cast<unsigned long long*>(dev_->get((uint64_t)hc2[0] * 8));
            k_l0_hash_ids<<<grid_for(cap, 256, 1u << 30), 256, 0, stream_>>>(hk, (uint32_t)cap, hcid, ck);
            HIP_CHECK(hipGetLastError());
            P.hkeys = hk;
            P.hcid = hcid;
            P.ckeys = ck;
            G = hc2[0];
            break;
        }
    }
    const uint64_t D = G * (uint64_t)kL0Layers;
    if (D >= (1ull << 32)) return fail(-27, "too many level-0 slabs (occupied cells x hex layers >= 2^32)");
    uint32_t* hist = static_cast<uint32_t*>(dev_->get(D * 4));
    uint32_t* cnt_scan = static_cast<uint32_t*>(dev_->get(D * 4));
    uint32_t* sflag = static_cast<uint32_t*>(dev_->get(D * 4));
    uint32_t* cflag = static_cast<uint32_t*>(dev_->get(G * 4));
    uint32_t* cscan = static_cast<uint32_t*>(dev_->get(G * 4));
    uint32_t* d_tot = static_cast<uint32_t*>(dev_->get(16));
    HIP_CHECK(hipMemsetAsync(hist, 0, D * 4, stream_));
    int cbits = 0;
    while ((1ull << cbits) < G) cbits++;
    const int rem = kL0LayerBits - 6 + cbits;
    const int passes = std::max(1, (rem + 7) / 8);
    const int per = std::max(1, (rem + passes - 1) / passes);
    // pass 2 without an upsweep (k_l0_down5g) when the rest of the dense id fits
    // one 5-bit pass: pass 1 then counts the (d6, d5) pairs per group (with
    // external keys staged beside the points the pair table must stay <= 16 wide)
    // (the folded pass 1 counts 32-wide pairs with keys staged too: its pair table
    // needs no digit staging array)
    bool g1up = fold || (!P.hashed && passes == 1 && per <= (l0keys ? 4 : 5) && ntiles > 0 &&
                         getenv("PCC_L0_TWO_UPSWEEPS") == nullptr);
    const uint32_t r5 = fold ? r2f : l0keys ? 16u : 32u;
    // capacities fused into the pass-1 upsweep when the level-1 slab grid fits LDS
    L1Grid Q;
    for (int a = 0; a < 3; a++) { Q.lo[a] = 2 * P.lo[a]; Q.g[a] = 2 * P.g[a]; }
    const uint64_t D1w = 8ull * G * kL0Layers;
    const bool fuse_dcap = !g1up && !P.hashed && D1w <= (uint64_t)kHist1Lds && getenv("PCC_NO_FUSED_DCAP") == nullptr;
    const uint32_t D1 = fuse_dcap ? (uint32_t)D1w : 0u;
    uint32_t* H1 = nullptr;
    if (fuse_dcap) {
        H1 = static_cast<uint32_t*>(dev_->get((uint64_t)D1 * 4));
        HIP_CHECK(hipMemsetAsync(H1, 0, (uint64_t)D1 * 4, stream_));
    }
    // LSD passes over the dense slab id (key recomputed from positions every
    // pass): pass 1 on the low 6 layer bits (k_l0_down6g, offsets from pass 0),
    // then either the one-upsweep pass 2 (k_l0_down5g) or the rest of the layer
    // and the cell bits in passes of at most 8 bits, the first of which also
    // builds the dense histogram.
    Arena A0 = dev_->ar[0], A1 = dev_->ar[1];
    // the final pass must land in arena 0
    Arena dst = (passes % 2) ? A1 : A0;
    if (!fold) scan_excl_u32(gcnt0, gcnt0, 64u * ngroups, nullptr, dev_->scan, stream_);
    uint32_t* gcnt = g1up ? static_cast<uint32_t*>(dev_->get(64ull * ngroups * r5 * 4)) : nullptr;
    if (ntiles && !fold) {
        if (l0keys)
            k_l0_down6g<16, true><<<ngroups, kL0BS, 0, stream_>>>(src_, src_keys_, dst, nsrc_, P, gcnt0, ntiles, tpg,
                                                                   ngroups, gcnt, g1up ? 1 : 0, l0dummy, dev_->ctr);
        else
            k_l0_down6g<32, false><<<ngroups, kL0BS, 0, stream_>>>(src_, nullptr, dst, nsrc_, P, gcnt0, ntiles, tpg,
                                                                    ngroups, gcnt, g1up ? 1 : 0, l0dummy, dev_->ctr);
    }
    uint32_t* starts = nullptr;
    L0Unit* dunits = nullptr;
    uint32_t nunits = 0;
    // The folded binning runs from the bounding box's sync to the end of pass 2
    // without a host round trip: tables sized by the grid's slab and cell bounds
    // (D, G), units planned on the device, the totals read once at the end.
    const bool defer = fold && root_xyz_.empty() && !prior_ && getenv("PCC_L0_HOSTPLAN") == nullptr;
    if (g1up) {
        starts = static_cast<uint32_t*>(dev_->get(64ull * (ngroups + 1) * 4));
        if (fold) {
            // run positions of the tile-major output in the digit-partitioned order,
            // segment starts per (d6, group), pair prefixes from the parity slots
            scan_excl_u32(cnt6, cnt6, R1 * ntiles, nullptr, dev_->scan, stream_);
            k_l0_tstarts<<<grid_for((uint64_t)R1 * (ngroups + 1), 256, 1u << 30), 256, 0, stream_>>>(
                cnt6, ntiles, tpg, ngroups, nsrc_, starts, R1);
            L0PMap pm;
            const uint32_t pb = (uint32_t)fcb / 3, pmk = (1u << pb) - 1u;
            for (uint32_t d5 = 0; d5 < 256; d5++) pm.s[d5] = 0xFFFF;
            for (uint32_t d5 = 0; d5 < r2f; d5++) {
                // dense high digit = cell << HB | layer-high bits, cell = (gz * g1 + gy) * g0 + gx
                const uint32_t cell = d5 >> HB, hi = d5 & ((1u << HB) - 1u);
                const uint32_t gx = cell % (uint32_t)P.g[0], gy = (cell / (uint32_t)P.g[0]) % (uint32_t)P.g[1];
                const uint32_t gz = cell / ((uint32_t)P.g[0] * (uint32_t)P.g[1]);
                if (cell >= G) continue;
                // the cell's slot among the pair counts: absolute indices modulo 2 or 4
                const uint32_t par = ((uint32_t)(P.lo[0] + (int32_t)gx) & pmk) |
                                     (((uint32_t)(P.lo[1] + (int32_t)gy) & pmk) << pb) |
                                     (((uint32_t)(P.lo[2] + (int32_t)gz) & pmk) << (2 * pb));
                pm.s[d5] = (uint16_t)((par << HB) | hi);
            }
            if (fcb == 6)
                k_l0_gprefix_par<lb, 6><<<R1, 1024, 0, stream_>>>(gpar, gcnt, ngroups, (uint32_t)D, pm, hist, dev_->ctr);
            else
                k_l0_gprefix_par<lb><<<R1, 1024, 0, stream_>>>(gpar, gcnt, ngroups, (uint32_t)D, pm, hist, dev_->ctr);
        } else {
            if (l0keys) k_l0_gprefix<16><<<64, 1024, 0, stream_>>>(gcnt, ngroups, (uint32_t)D, hist, dev_->ctr);
            else k_l0_gprefix<32><<<64, 1024, 0, stream_>>>(gcnt, ngroups, (uint32_t)D, hist, dev_->ctr);
            k_l0_gstarts<<<grid_for(64ull * (ngroups + 1), 256, 1u << 30), 256, 0, stream_>>>(gcnt0, ngroups, nsrc_, starts);
        }
        HIP_CHECK(hipGetLastError());
        // the segment starts go to pinned host memory now; the unit plan is made
        // after the one host sync of the level (below).  The folded binning plans
        // its units on the device (k_l0_uplan).
        const uint64_t nst = 64ull * (ngroups + 1);
        if (!defer && dev_->hst_cap < nst) {
            if (dev_->hst) (void)hipHostFree(dev_->hst);
            HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&dev_->hst), nst * 4, hipHostMallocDefault));
            dev_->hst_cap = nst;
        }
        if (!defer) HIP_CHECK(hipMemcpyAsync(dev_->hst, starts, nst * 4, hipMemcpyDeviceToHost, stream_));
    }
    HIP_CHECK(hipGetLastError());
    Arena src = dst;
    dst = (dst.p == A0.p) ? A1 : A0;
    const Arena p1out = src, p2dst = dst;
    uint32_t tots[3];
    Counters hc;
    // the upsweep passes (when pass 2 is not the one-upsweep kernel), tables, the
    // level's host sync
    {
        src = p1out;
        dst = p2dst;
        uint32_t* counts = g1up ? nullptr : static_cast<uint32_t*>(dev_->get(((uint64_t)ntiles << per) * 4 + 64));
        for (int p = 0, shift = 6; p < passes && !g1up; p++, shift += per) {
            switch (per) {
                case 1: l0_pass<1>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                case 2: l0_pass<2>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                case 3: l0_pass<3>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                case 4: l0_pass<4>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                case 5: l0_pass<5>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                case 6: l0_pass<6>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                case 7: l0_pass<7>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
                default: l0_pass<8>(p, passes, src, dst, nsrc_, P, shift, counts, ntiles, hist, (uint32_t)D, dev_->ctr, Q, H1, D1, dev_->scan, stream_); break;
            }
            src = dst;
            dst = (dst.p == A0.p) ? A1 : A0;
        }
        // slab / cell tables from the dense histogram
        k_l0_flags<<<grid_for(std::max<uint64_t>(D, G), 256, 1u << 30), 256, 0, stream_>>>(hist, (uint32_t)D, P.nl, sflag, cflag, (uint32_t)G);
        scan_excl_u32(hist, cnt_scan, (uint32_t)D, d_tot + 0, dev_->scan, stream_);
        scan_excl_u32(sflag, sflag, (uint32_t)D, d_tot + 1, dev_->scan, stream_);
        scan_excl_u32(cflag, cscan, (uint32_t)G, d_tot + 2, dev_->scan, stream_);
        if (!defer) {
            readback({{tots, d_tot, 12}, {&hc, dev_->ctr, sizeof hc}});
            if (hc.err) return geom_fail("level-0 binning: point outside the bounding grid (internal error)");
        }
    }
    if (defer) {   // upper bounds until the totals are read (below)
        tots[0] = (uint32_t)nsrc_;
        tots[1] = (uint32_t)D;
        tots[2] = (uint32_t)G;
    }
    if (tots[0] != nsrc_) return fail(-5, "level-0 histogram mismatch");
    Level* L = new Level();
    L->dev = dev_;
    levels_.push_back(L);
    L->h = h0_;
    L->ncells = tots[2];
    L->nslabs = tots[1];
    L->arena = 0;
    L->arrivals = nsrc_;
    L->alloc(L->cell_idx, 3ull * L->ncells);
    L->alloc(L->cell_sb, L->ncells);
    L->alloc(L->cell_slab0, L->ncells + 1ull);
    L->alloc(L->slab_cell, L->nslabs);
    L->alloc(L->slab_layer, L->nslabs);
    L->alloc(L->slab_off, L->nslabs);
    L->alloc(L->slab_n, L->nslabs);
    L->alloc(L->big_list, L->nslabs);
    L->alloc(L->small_list, L->nslabs);
    L->alloc(L->dcap, (uint64_t)L->nslabs * kDests);
    k_l0_tables<<<grid_for(std::max<uint64_t>(D, G), 256, 1u << 30), 256, 0, stream_>>>(
        hist, cnt_scan, sflag, cflag, cscan, (uint32_t)D, (uint32_t)G, P, L->cell_idx, L->cell_sb, L->cell_slab0,
        L->slab_cell, L->slab_layer, L->slab_off, L->slab_n, defer ? d_tot : nullptr);
    if (!defer) k_set_u32<<<1, 1, 0, stream_>>>(L->cell_slab0 + L->ncells, L->nslabs);
    if (defer) {   // pass 2 of the folded binning, planned on the device
        // units of ~n / 8192 points; with 256 pass-2 digits n / 2048 (each unit
        // flushes 256 x 24 capacity counters)
        const uint64_t target = std::max<uint64_t>(nsrc_ / (fcb == 6 ? 2048 : 8192), 4ull * kL0Tile);
        const uint32_t umax = (uint32_t)(64 + (nsrc_ + target - 1) / target);
        const uint32_t wmax = (uint32_t)((nsrc_ + kL0Tile - 1) / kL0Tile) + umax;
        L0UnitW* duw = static_cast<L0UnitW*>(dev_->get((uint64_t)umax * sizeof(L0UnitW)));
        uint2* dwt = static_cast<uint2*>(dev_->get((uint64_t)wmax * sizeof(uint2)));
        uint32_t* dcnt = static_cast<uint32_t*>(dev_->get(16));
        uint32_t* dwn = static_cast<uint32_t*>(dev_->get((uint64_t)umax * 4));
        HIP_CHECK(hipMemsetAsync(L->dcap, 0, (uint64_t)L->nslabs * kDests * 4, stream_));
        k_l0_uplan<<<(umax + 255) / 256, 256, 0, stream_>>>(starts, ngroups, tpg, ntiles, (uint32_t)target, umax, duw,
                                                            dwn, dcnt, R1, getenv("PCC_L0_ROWS") ? 0 : 1);
        scan_excl_u32(dwn, dwn, umax, dcnt + 1, dev_->scan, stream_);
        k_l0_uplan_w0<<<(umax + 255) / 256, 256, 0, stream_>>>(duw, dwn, umax);
        k_l0_wplan<<<grid_for(wmax, 256, 1u << 30), 256, 0, stream_>>>(duw, 0, 0, cnt6, ntiles, dwt, dcnt);
        l0_pass2_tm(fcb, l0keys, umax, src, dst, P, nullptr, starts, ngroups, gcnt, cnt_scan, sflag, (uint32_t)D,
                    L->dcap, l0dummy, dev_->ctr, duw, dwt, cnt6, ph6, ntiles, stream_);
        HIP_CHECK(hipGetLastError());
    } else if (g1up) {   // pass 2 into arena 0, with the capacities
        // Units: runs of consecutive segments of one d6 bucket, about nsrc / 8192
        // points each, in bucket order (a segment is never split; with the default
        // groups a segment is at most 4 x the target).  Planned on the host while
        // the table kernels above run.
        const uint32_t* st = dev_->hst;
        const char* udiv = getenv("PCC_L0_UNIT_DIV");
        const uint64_t ud = udiv ? std::max<uint64_t>(1, strtoull(udiv, nullptr, 10)) : 8192;
        const uint64_t target = std::max<uint64_t>(nsrc_ / ud, 4ull * kL0Tile);
        std::vector<L0Unit> units;
        units.reserve(ud + 128);
        for (uint32_t d6 = 0; d6 < 64; d6++) {
            const uint32_t* row = st + (uint64_t)d6 * (ngroups + 1);
            uint32_t g0 = 0;
            uint64_t acc = 0;
            for (uint32_t gg = 0; gg < ngroups; gg++) {
                const uint64_t sz = row[gg + 1] - row[gg];
                if (acc && acc + sz > target) {
                    units.push_back(L0Unit{d6, g0, gg, 0});
                    g0 = gg;
                    acc = 0;
                }
                acc += sz;
            }
            if (acc) units.push_back(L0Unit{d6, g0, ngroups, 0});
        }
        nunits = (uint32_t)units.size();
        dunits = static_cast<L0Unit*>(dev_->get(std::max<uint64_t>(nunits, 1) * sizeof(L0Unit)));
        if (nunits)
            HIP_CHECK(hipMemcpyAsync(dunits, units.data(), nunits * sizeof(L0Unit), hipMemcpyHostToDevice, stream_));
        HIP_CHECK(hipMemsetAsync(L->dcap, 0, (uint64_t)L->nslabs * kDests * 4, stream_));
        L0UnitW* duw = nullptr;
        uint2* dwt = nullptr;
        if (fold && nunits) {   // the units' windows over the tile-major runs (k_l0_wplan)
            std::vector<L0UnitW> uw(nunits);
            uint32_t nwin = 0;
            for (uint32_t u = 0; u < nunits; u++) {
                const L0Unit& U = units[u];
                const uint32_t* row = st + (uint64_t)U.d6 * (ngroups + 1);
                L0UnitW& W = uw[u];
                W.d6 = U.d6;
                W.a = row[U.g0];
                W.b = row[U.g1];
                W.t0 = U.g0 * tpg;
                W.t1 = std::min<uint32_t>(U.g1 * tpg, ntiles);
                W.w0 = nwin;
                W.pad_g0 = U.g0;
                W.pad = 0;
                nwin += (W.b - W.a + kL0Tile - 1) / kL0Tile;
            }
            duw = static_cast<L0UnitW*>(dev_->get((uint64_t)nunits * sizeof(L0UnitW)));
            dwt = static_cast<uint2*>(dev_->get(std::max<uint64_t>(nwin, 1) * sizeof(uint2)));
            HIP_CHECK(hipMemcpyAsync(duw, uw.data(), nunits * sizeof(L0UnitW), hipMemcpyHostToDevice, stream_));
            k_l0_wplan<<<grid_for(nwin, 256, 1u << 30), 256, 0, stream_>>>(duw, nunits, nwin, cnt6, ntiles, dwt, nullptr);
            l0_pass2_tm(fcb, l0keys, nunits, src, dst, P, dunits, starts, ngroups, gcnt, cnt_scan, sflag, (uint32_t)D,
                        L->dcap, l0dummy, dev_->ctr, duw, dwt, cnt6, ph6, ntiles, stream_);
        } else if (nunits && r5 == 16) {
            k_l0_down5g<16, false><<<nunits, kL0BS, 0, stream_>>>(src, dst, P, dunits, starts, ngroups, gcnt, cnt_scan,
                                                                   sflag, (uint32_t)D, L->dcap, l0dummy, dev_->ctr,
                                                                   nullptr, nullptr, nullptr, nullptr, 0);
        } else if (nunits) {
            k_l0_down5g<32, false><<<nunits, kL0BS, 0, stream_>>>(src, dst, P, dunits, starts, ngroups, gcnt, cnt_scan,
                                                                   sflag, (uint32_t)D, L->dcap, l0dummy, dev_->ctr,
                                                                   nullptr, nullptr, nullptr, nullptr, 0);
        }
        HIP_CHECK(hipGetLastError());
    }
    if (!root_xyz_.empty() && L->ncells) {   // sub-tree build: the roots' spill batches
        int32_t* rx = static_cast<int32_t*>(dev_->get(root_xyz_.size() * 4));
        uint32_t* rs = static_cast<uint32_t*>(dev_->get(root_sb_.size() * 4));
        HIP_CHECK(hipMemcpyAsync(rx, root_xyz_.data(), root_xyz_.size() * 4, hipMemcpyHostToDevice, stream_));
        HIP_CHECK(hipMemcpyAsync(rs, root_sb_.data(), root_sb_.size() * 4, hipMemcpyHostToDevice, stream_));
        k_root_sb<<<grid_for(L->ncells, 256, 1u << 30), 256, 0, stream_>>>(L->cell_idx, L->ncells, rx, rs,
                                                                            (uint32_t)root_sb_.size(), L->cell_sb, dev_->ctr);
        HIP_CHECK(hipGetLastError());
    }
    if (prior_ && !pdev_.empty() && L->nslabs) {   // merge: each level-0 slab's record in the existing cloud
        L->alloc(L->slab_prior, L->nslabs);
        k_prior_lookup0<<<grid_for(L->nslabs, 256, 1u << 30), 256, 0, stream_>>>(
            L->cell_idx, L->slab_cell, L->slab_layer, L->nslabs, pdev_[0].cells, pdev_[0].cell_slab0, pdev_[0].slab_layer,
            pdev_[0].ncells, L->slab_prior);
    }
    k_l0_lists<<<grid_for(L->nslabs, 256, 1u << 30), 256, 0, stream_>>>(L->slab_n, L->nslabs, L->big_list,
                                                                          L->small_list, dev_->ctr, defer ? d_tot + 1 : nullptr);
    if (defer) {   // the level's one sync after the bounding box's: totals, lists, errors
        readback({{tots, d_tot, 12}, {&hc, dev_->ctr, sizeof hc}});
        ev_end(ST_L0);
        if (hc.err) return geom_fail("level-0 binning: point outside the bounding grid (internal error)");
        if (tots[0] != nsrc_) return fail(-5, "level-0 histogram mismatch");
        L->ncells = tots[2];
        L->nslabs = tots[1];
        L->max_slab = hc.max_slab;
        L->nbig = hc.nbig;
        L->nsmall = hc.nsmall;
        stats_.cells += L->ncells;
        stats_.slabs += L->nslabs;
        stats_.arrivals += nsrc_;
        return 0;
    }
    {
        readback({{&hc, dev_->ctr, sizeof hc}});
        L->max_slab = hc.max_slab;
        if (g1up) {
            // capacities counted by k_l0_down5g
        } else if (fuse_dcap) {
            const uint64_t nd = (uint64_t)L->nslabs * kDests;
            k_l0_dcap_from1<<<grid_for(nd, 256, 1u << 30), 256, 0, stream_>>>(H1, P, Q, L->cell_idx, L->slab_cell,
                                                                              L->slab_layer, L->nslabs, L->dcap);
        } else {
            run_dcap(L);
        }
    }
    HIP_CHECK(hipGetLastError());
    ev_end(ST_L0);
    readback({{&hc, dev_->ctr, sizeof hc}});
    if (hc.err) return geom_fail("level-0 capacities: routing error (internal error)");
    L->nbig = hc.nbig;
    L->nsmall = hc.nsmall;
    stats_.cells += L->ncells;
    stats_.slabs += L->nslabs;
    stats_.arrivals += nsrc_;
    return 0;
}

// capacities (arrivals per child slab) of level L's slabs
void Engine::run_dcap(Level* L) {
    const float csc = cell_size(cfg_.max_cell_size, L->h + 1);
    DcapParams D;
    D.A = dev_->ar[L->arena];
    D.cell_idx = L->cell_idx;
    D.slab_cell = L->slab_cell;
    D.slab_layer = L->slab_layer;
    D.slab_off = L->slab_off;
    D.slab_n = L->slab_n;
    D.dcap = L->dcap;
    D.ctr = dev_->ctr;
    D.csc = csc;
    D.inv_csc = 1.0f / csc;
    D.crc = hex_radius(sub_cell_size(csc, cfg_.sub_grid_dimension));
    D.inv_crc = 1.0f / D.crc;
    D.check = (L->h + 1 < kMaxDepth) ? 1u : 0u;
    HIP_CHECK(hipMemsetAsync(L->dcap, 0, (uint64_t)L->nslabs * kDests * 4, stream_));
    // blocks of one slab: enough to cover its arrivals in <= 64 strides, at most 128
    const uint32_t y = std::min<uint32_t>(128, std::max<uint32_t>(1, (L->max_slab + 256 * 64 - 1) / (256 * 64)));
    if (L->nslabs) k_dcap<<<dim3(L->nslabs, y), 256, 0, stream_>>>(D);
    HIP_CHECK(hipGetLastError());
}

int Engine::run_level(uint32_t li) {
    Level* L = levels_[li];
    const uint32_t h = L->h;   // absolute level (h0_ + li)
    const uint32_t dim = cfg_.sub_grid_dimension;
    const SlabGeom g = slab_geom(dim);
    const float cs = cell_size(cfg_.max_cell_size, h);
    const Arena& in = dev_->ar[L->arena];
    const Arena& nx = dev_->ar[1 - L->arena];
    const uint64_t ND = (uint64_t)L->nslabs * kDests;
    L->alloc(L->dest_off, ND);
    L->alloc(L->dest_n, ND);
    L->alloc(L->gcap, ND * kDests);
    L->alloc(L->grid_off, L->nslabs);
    L->alloc(L->slab_grid_n, L->nslabs);
    L->alloc(L->bkt_state, 8ull * L->ncells);
    L->alloc(L->bkt_off, 8ull * L->ncells);
    L->alloc(L->bkt_n, 8ull * L->ncells);
    L->alloc(L->bkt_sb, 8ull * L->ncells);
    L->alloc(L->bkt_nd, 8ull * L->ncells);
    L->alloc(L->grid, L->arrivals);
    L->kept_cap = std::min<uint64_t>(L->arrivals, 8ull * L->ncells * cfg_.cell_point_overflow_limit);
    L->alloc(L->kept, L->kept_cap);
    if (cfg_.cell_point_overflow_limit > (uint32_t)kKeptMax) L->alloc(L->ksort, 2 * std::max<uint64_t>(L->kept_cap, 1));
    uint32_t* scratch = static_cast<uint32_t*>(dev_->get(16));
    // output regions from exclusive scans (no allocation atomics in the slab kernels).
    // Merge: each child slab's region starts with room for its injected seeds.
    const bool inject = prior_ && L->slab_prior && h + 1 < pdev_.size();
    if (inject) {
        L->alloc(L->room, ND);
        uint32_t* capr = static_cast<uint32_t*>(dev_->get(ND * 4));
        k_room<<<grid_for(ND, 256, 1u << 30), 256, 0, stream_>>>(L->slab_prior, L->nslabs, pdev_[h].slabs,
                                                                 pdev_[h + 1].slabs, L->dcap, L->room, capr);
        scan_excl_u32(capr, L->dest_off, (uint32_t)ND, scratch, dev_->scan, stream_);
        k_add_room<<<grid_for(ND, 256, 1u << 30), 256, 0, stream_>>>(L->dest_off, L->room, ND);
        HIP_CHECK(hipGetLastError());
    } else {
        scan_excl_u32(L->dcap, L->dest_off, (uint32_t)ND, scratch, dev_->scan, stream_);
    }
    scan_excl_u32(L->slab_n, L->grid_off, L->nslabs, scratch + 1, dev_->scan, stream_);
    // per-level counters, and the child-slab capacities against the next arena
    // (on the device: no host round trip; reported at the level's sync)
    // (PCC_TEST_ARENA_CAP: tests shrink the arena seen by the check and the region
    // clamps, so the clamped kernels and the error path run)
    uint64_t acap = dev_->cap;
    if (const char* tc = getenv("PCC_TEST_ARENA_CAP")) acap = std::min<uint64_t>(acap, strtoull(tc, nullptr, 10));
    k_level_begin<<<1, 1, 0, stream_>>>(dev_->ctr, scratch, acap);
    SlabParams SP;
    SP.in = in;
    SP.nx = nx;
    SP.grid = L->grid;
    SP.cell_idx = L->cell_idx;
    SP.cell_sb = L->cell_sb;
    SP.slab_cell = L->slab_cell;
    SP.slab_layer = L->slab_layer;
    SP.slab_off = L->slab_off;
    SP.slab_n = L->slab_n;
    SP.grid_off = L->grid_off;
    SP.dcap = L->dcap;
    SP.dest_off = L->dest_off;
    SP.slab_grid_n = L->slab_grid_n;
    SP.dest_n = L->dest_n;
    SP.gcap = L->gcap;
    SP.check_gchild = (h + 2 < kMaxDepth) ? 1 : 0;
    SP.kf_lo = 0;
    SP.kf_n = 0;
    if (prior_ && h < forced_lo_.size()) {
        SP.kf_lo = (uint32_t)forced_lo_[h];
        SP.kf_n = (uint32_t)(nseeds_ - forced_lo_[h]);
    }
    SP.ctr = dev_->ctr;
    SP.inj = reinterpret_cast<const float4*>(d_inj_);
    SP.inj_keys = d_inj_keys_;
    SP.cs = cs;
    SP.G = level_geo(cfg_, h);
    SP.inj_rec = d_inj_rec_;
    SP.tx = g.tx;
    SP.ty = g.ty;
    SP.stamps = nullptr;
#ifdef PCC_STAMPS
    unsigned long long* stamps = static_cast<unsigned long long*>(dev_->get(2 * 16 * 8));
    HIP_CHECK(hipMemsetAsync(stamps, 0, 2 * 16 * 8, stream_));
#endif
    // merge, levels >= 1: the slab kernels read this level's seeds in place from
    // the seed array (the room in front of the emissions stays unwritten)
    const bool seeds_in_place = prior_ && h >= 1 && L->slab_prior && h < pdev_.size();
    const bool verbose = getenv("PCC_VERBOSE") != nullptr;
    const auto tv0 = std::chrono::steady_clock::now();
    if (verbose) {
        HIP_CHECK(hipStreamSynchronize(stream_));
        fprintf(stderr, "[pcc] level %u: cells %u slabs %u (dense %u, small %u) arrivals %llu max_slab %u\n", h, L->ncells,
                L->nslabs, L->nbig, L->nsmall, (unsigned long long)L->arrivals, L->max_slab);
    }
    // the small slabs' descriptors and class counts first: their readback
    // completes while the dense kernel runs, so the small kernels queue behind
    // it without a host round trip in between
    SmallDesc* wd = nullptr;
    SmallDesc* bd = nullptr;
    uint32_t hcnt[4] = {0, 0, 0, 0};
    if (L->nsmall) {
        wd = static_cast<SmallDesc*>(dev_->get((uint64_t)L->nsmall * 3 * sizeof(SmallDesc)));
        bd = static_cast<SmallDesc*>(dev_->get((uint64_t)L->nsmall * sizeof(SmallDesc)));
        uint32_t* cnt = static_cast<uint32_t*>(dev_->get(16));
        HIP_CHECK(hipMemsetAsync(cnt, 0, 16, stream_));
        k_small_desc<<<grid_for(L->nsmall, 256, 1u << 30), 256, 0, stream_>>>(
            L->small_list, L->nsmall, L->slab_cell, L->slab_layer, L->slab_off, L->slab_n, L->cell_idx, L->cell_sb,
            L->dest_off, L->dcap, wd, bd, cnt, seeds_in_place ? L->slab_prior : nullptr,
            seeds_in_place ? pdev_[h].slabs : nullptr, acap);
        readback_begin({{hcnt, cnt, 16}});
    }
    if (L->nbig) {
        SP.list = L->big_list;
        // skewed sizes (the largest slab well above the mean): largest first, so
        // the big ones do not start last and leave the chip idle behind them
        const uint32_t* dlist = L->big_list;
        if (PCC_LPT && L->nbig > 256 && L->nbig <= (1u << 17) &&   // (one block: up to ~0.1 ms)
            (double)L->max_slab * L->nbig > 1.5 * (double)L->arrivals) {
            uint32_t* sorted = static_cast<uint32_t*>(dev_->get((uint64_t)L->nbig * 4));
            k_lpt_order<<<1, 1024, 0, stream_>>>(L->big_list, L->nbig, L->slab_n, L->max_slab, sorted);
            dlist = sorted;
            if (verbose) fprintf(stderr, "[pcc]   dense slabs launched largest first\n");
        }
        SmallDesc* dd = static_cast<SmallDesc*>(dev_->get((uint64_t)L->nbig * sizeof(SmallDesc)));
        k_dense_desc<<<grid_for(L->nbig, 256, 1u << 30), 256, 0, stream_>>>(dlist, L->nbig, L->slab_cell,
                                                                           L->slab_layer, L->slab_off, L->slab_n,
                                                                           L->cell_idx, L->cell_sb, L->dest_off,
                                                                           L->dcap, dd,
                                                                           seeds_in_place ? L->slab_prior : nullptr,
                                                                           seeds_in_place ? pdev_[h].slabs : nullptr, acap);
        SP.ddesc = dd;
#ifdef PCC_STAMPS
        SP.stamps = stamps;
#endif
        ev_begin(ST_DENSE);
        // NaN rules: NaN input points, or NaN seeds of the existing cloud
        const bool nf = nf_mode_ || (prior_ && prior_nan_);
        if (seeds_in_place && nf) k_slab<true, true, true><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        else if (seeds_in_place) k_slab<true, false, true><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        else if (SP.kf_n && nf) k_slab<false, true, true><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        else if (SP.kf_n) k_slab<false, false, true><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        else if (nf) k_slab<false, true, false><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        else if (L->max_slab > kJMaskNarrow) k_slab<false, false, false><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        else k_slab<false, false, false, false><<<L->nbig, kDenseBS, 0, stream_>>>(SP);
        ev_end(ST_DENSE);
        if (verbose) {
            HIP_CHECK(hipStreamSynchronize(stream_));
            fprintf(stderr, "[pcc]   dense slabs %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tv0).count());
        }
    }
    if (L->nsmall) {
        SP.list = L->small_list;
#ifdef PCC_STAMPS
        SP.stamps = stamps + 16;
#endif
        ev_begin(ST_SMALL);
        readback_end();
        for (int c = 0; c < 3; c++) {
            if (!hcnt[c]) continue;
            SP.wdesc = wd + (uint64_t)c * L->nsmall;
            SP.nwave = hcnt[c];
            // one workgroup per slab: the dispatcher hands a finished wave's
            // CU slot to the next slab (a persistent grid of resident waves
            // walking the list was 1.6x slower at level 3 of config 4)
            const uint32_t gr = hcnt[c];
            // (merge levels: the classes of 128-511 arrivals install whole chunks of
            // grid seeds from their records; the smallest class has few whole chunks)
            if (seeds_in_place && c >= 1) {
                if (c == 1) k_slab_wave<kWaveMax / 128, true><<<gr, 64, 0, stream_>>>(SP);
                else k_slab_wave<kWaveMax / 64, true><<<gr, 64, 0, stream_>>>(SP);
            } else {
                if (c == 0) k_slab_wave<kWaveMax / 256><<<gr, 64, 0, stream_>>>(SP);
                else if (c == 1) k_slab_wave<kWaveMax / 128><<<gr, 64, 0, stream_>>>(SP);
                else k_slab_wave<kWaveMax / 64><<<gr, 64, 0, stream_>>>(SP);
            }
        }
        if (hcnt[3]) {
            SP.sdesc = bd;
            SP.nlist = hcnt[3];
            k_slab_small<<<hcnt[3], kSmallBS, 0, stream_>>>(SP);
        }
        ev_end(ST_SMALL);
    }
    HIP_CHECK(hipGetLastError());
    BucketParams BP;
    BP.nx = nx;
    BP.files = dev_->files;
    BP.nfiles = nfiles_dev_;
    BP.cell_sb = L->cell_sb;
    BP.cell_idx = L->cell_idx;
    BP.prior = (prior_ && h < pdev_.size()) ? pdev_[h].cells : nullptr;
    BP.nprior = (prior_ && h < pdev_.size()) ? pdev_[h].ncells : 0u;
    BP.kept = L->kept;
    BP.kept_cap = L->kept_cap;
    BP.ksort = L->ksort;
    BP.cell_slab0 = L->cell_slab0;
    BP.dest_off = L->dest_off;
    BP.dest_n = L->dest_n;
    BP.bkt_state = L->bkt_state;
    BP.bkt_off = L->bkt_off;
    BP.bkt_n = L->bkt_n;
    BP.bkt_sb = L->bkt_sb;
    BP.bkt_nd = L->bkt_nd;
    BP.room = inject ? L->room : nullptr;
    BP.ctr = dev_->ctr;
    // raw last level (set_max_levels(m, raw)): every bucket forwards all its
    // emissions (limit 0), the caller resolves the buckets across ranks
    BP.L = (raw_last_ && max_levels_ && li + 1 == max_levels_) ? 0u : cfg_.cell_point_overflow_limit;
    const uint32_t nb = 8 * L->ncells;
    ev_begin(ST_BUCKET);
    BP.dlist = static_cast<uint32_t*>(dev_->get(nb * 4ull));
    BP.dcount = static_cast<uint32_t*>(dev_->get(8));   // count, ticket
    // (PCC_BKT_SPLIT_MIN: another threshold, for tests of the two launches on small inputs)
    const char* bsm = getenv("PCC_BKT_SPLIT_MIN");
    const uint32_t split_min = bsm ? (uint32_t)strtoul(bsm, nullptr, 10) : kBktSplitMin;
    const bool bkt_split = getenv("PCC_BKT_ONE") == nullptr && nb >= split_min;
    if (bkt_split) HIP_CHECK(hipMemsetAsync(BP.dcount, 0, 8, stream_));
    // a level of many buckets (most of them short kept lists, e.g. the last
    // level) in two launches; a few buckets in one (the second launch and its
    // counter cost more than they save there).  PCC_BKT_ONE: always one (A/B).
    if (!bkt_split) {
        k_bucket<kBktBS, kKeptMax><<<nb, kBktBS, 0, stream_>>>(BP);
    } else {
        k_bucket<kBktSmallBS, kKeptSmall><<<nb, kBktSmallBS, 0, stream_>>>(BP);
        if (BP.L > (uint32_t)kKeptSmall)   // two resident workgroups per CU (64 KB of LDS each)
            k_bucket<kBktBS, kKeptMax, true><<<std::min<uint32_t>(nb, 512), kBktBS, 0, stream_>>>(BP);
    }
    ev_end(ST_BUCKET);
    HIP_CHECK(hipGetLastError());
    // this level's grid points (one scan instead of per-slab global atomics)
    uint32_t* gsc = static_cast<uint32_t*>(dev_->get((uint64_t)L->nslabs * 4 + 16));
    uint32_t* gtot = static_cast<uint32_t*>(dev_->get(16));
    scan_excl_u32(L->slab_grid_n, gsc, L->nslabs, gtot, dev_->scan, stream_);
    ev_begin(ST_NEXT);
    uint32_t* flag = static_cast<uint32_t*>(dev_->get(nb * 4ull));
    uint32_t* ndv = static_cast<uint32_t*>(dev_->get(nb * 4ull));
    uint32_t* tots = static_cast<uint32_t*>(dev_->get(16));
    k_next_flags<<<grid_for(nb, 256, 1u << 30), 256, 0, stream_>>>(L->bkt_state, L->bkt_nd, nb, flag, ndv);
    scan_excl_u32(flag, flag, nb, tots + 0, dev_->scan, stream_);
    scan_excl_u32(ndv, ndv, nb, tots + 1, dev_->scan, stream_);
    ev_end(ST_NEXT);
#ifdef PCC_STAMPS
    {
        unsigned long long hs[32];
        HIP_CHECK(hipMemcpyAsync(hs, stamps, sizeof hs, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        const char* nm[16] = {"prologue", "claimA", "routeA", "B0wait", "rounds", "rndwait", "stores", "tail",
                              "pass2", "#rounds", "#steps", "p2sync", "ldwait/epi", "math", "episcan", "episync"};
        for (int v = 0; v < 2; v++) {
            if (!hs[16 * v + 10]) continue;
            fprintf(stderr, "[stamps] level %u %s waves*steps=%llu  cycles/step:", h, v ? "small" : "dense", hs[16 * v + 10]);
            for (int q = 0; q < 16; q++)
                if (q != 9 && q != 10) fprintf(stderr, " %s=%.0f", nm[q], (double)hs[16 * v + q] / hs[16 * v + 10]);
            fprintf(stderr, " rounds/step=%.2f\n", (double)hs[16 * v + 9] / hs[16 * v + 10]);
        }
    }
#endif
    uint32_t ht[2], hg = 0;
    Counters hc;
    readback({{&hg, gtot, 4}, {ht, tots, 8}, {&hc, dev_->ctr, sizeof hc}});
    L->kept_used = hc.kept_cur;
    stats_.grid_points += hg;
    stats_.kept_points += hc.kept_cur;
    if (hc.err & ERR_ARENA) {
        char buf[160];
        snprintf(buf, sizeof buf,
                 "internal: the child-slab capacities of level %u exceed the next level's arena (their regions "
                 "were clamped to it; device flags 0x%x)", h, hc.err);
        return fail(-5, buf);
    }
    if (hc.err) {
        geom_fault_ = (hc.err & ~(uint32_t)(ERR_SLOT_RANGE | ERR_LAYER | ERR_OCTANT | ERR_SEL)) == 0;
        char buf[200];
        snprintf(buf, sizeof buf,
                 "device error flags 0x%x at level %u (1 slot range, 2 layer, 4 octant, 8 sel, 16 kept cap, 64 capacity, "
                 "128 claim, 256 slab > 2^28 arrivals, 512 child capacities beyond the arena)",
                 hc.err, h);
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
        N->alloc(N->dcap, (uint64_t)N->nslabs * kDests);
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
        Q.gcap = L->gcap;
        Q.ndcap = N->dcap;
        Q.ncell_idx = N->cell_idx;
        Q.ncell_sb = N->cell_sb;
        Q.ncell_slab0 = N->cell_slab0;
        Q.nslab_cell = N->slab_cell;
        Q.nslab_layer = N->slab_layer;
        Q.nslab_off = N->slab_off;
        Q.nslab_n = N->slab_n;
        Q.nbig_list = N->big_list;
        Q.nsmall_list = N->small_list;
        Q.slab_prior = inject ? L->slab_prior : nullptr;
        Q.room = inject ? L->room : nullptr;
        Q.prec = inject ? pdev_[h].slabs : nullptr;
        Q.prec_next = inject ? pdev_[h + 1].slabs : nullptr;
        if (inject) N->alloc(N->slab_prior, N->nslabs);
        Q.nslab_prior = inject ? N->slab_prior : nullptr;
        Q.ctr = dev_->ctr;
        ev_begin(ST_NEXT);
        k_next_emit<<<nb, 256, 0, stream_>>>(Q);
        k_set_u32<<<1, 1, 0, stream_>>>(N->cell_slab0 + N->ncells, N->nslabs);
        if (inject && N->nslabs && getenv("PCC_COPY_SEEDS"))   // diagnostic: copy the seeds into their room
            k_inject_seeds<<<std::min<uint32_t>(N->nslabs, 65536), 256, 0, stream_>>>(
                N->slab_prior, N->slab_off, N->nslabs, pdev_[h + 1].slabs, reinterpret_cast<const float4*>(d_inj_),
                d_inj_keys_, dev_->ar[N->arena], N->slab_n);
        ev_end(ST_NEXT);
        HIP_CHECK(hipGetLastError());
        readback({{&hc, dev_->ctr, sizeof hc}});
        N->nbig = hc.nbig;
        N->nsmall = hc.nsmall;
        N->arrivals = hc.arrivals_next;
        N->max_slab = hc.max_slab;
        stats_.arrivals += hc.arrivals_next;
        stats_.cells += N->ncells;
        stats_.slabs += N->nslabs;
    }
    return 0;
}

// Grid winners of one level compacted on the device (slab s's n_s winners from
// its capacity-sized region to cgo[s] = sum of the earlier slabs' winners), so
// the D2H moves the winners only (about a third of the regions at config 4).
__global__ __launch_bounds__(256) void k_compact_grid(const Point* __restrict__ grid, const uint32_t* __restrict__ off,
                                                      const uint32_t* __restrict__ n, const uint32_t* __restrict__ cgo,
                                                      uint32_t nslabs, Point* __restrict__ dst) {
    for (uint32_t s = blockIdx.x; s < nslabs; s += gridDim.x) {
        const float4* src = reinterpret_cast<const float4*>(grid) + off[s];
        float4* d = reinterpret_cast<float4*>(dst) + cgo[s];
        for (uint32_t i = threadIdx.x; i < n[s]; i += 256) d[i] = src[i];
    }
}

uint32_t Engine::num_levels() const { return (uint32_t)levels_.size(); }

int Engine::built_cells(std::vector<int32_t>& hxyz) {
    hxyz.clear();
    for (Level* L : levels_) {
        std::vector<int32_t> idx(3ull * L->ncells);
        if (!idx.empty()) HIP_CHECK(hipMemcpyAsync(idx.data(), L->cell_idx, idx.size() * 4, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
        for (uint32_t c = 0; c < L->ncells; c++) {
            hxyz.push_back((int32_t)L->h);
            hxyz.insert(hxyz.end(), idx.begin() + 3ull * c, idx.begin() + 3ull * c + 3);
        }
    }
    return 0;
}

void Engine::set_max_levels(uint32_t m, bool raw) {
    max_levels_ = m;
    raw_last_ = raw && m;
}

void Engine::set_root_spill_batches(const int32_t* xyz, const uint32_t* sb, uint64_t n) {
    std::vector<uint64_t> ord(n);
    for (uint64_t i = 0; i < n; i++) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
        return std::lexicographical_compare(xyz + 3 * a, xyz + 3 * a + 3, xyz + 3 * b, xyz + 3 * b + 3);
    });
    root_xyz_.clear();
    root_sb_.clear();
    for (uint64_t i : ord) {
        root_xyz_.insert(root_xyz_.end(), xyz + 3 * i, xyz + 3 * i + 3);
        root_sb_.push_back(sb[i]);
    }
}

int Engine::pending_info(uint64_t& ncells, uint64_t& npoints) const {
    ncells = pending_ ? pending_->ncells : 0;
    npoints = pending_ ? pending_->arrivals : 0;
    return 0;
}

int Engine::export_pending(int32_t* xyz, uint32_t* sb, uint64_t* cell_n, Point* dpts, uint32_t* dkeys) {
    if (!pending_) return 0;
    Level* P = pending_;
    const uint64_t mk = dev_->mark();
    uint32_t* off = static_cast<uint32_t*>(dev_->get((uint64_t)P->nslabs * 4 + 16));
    uint32_t* tot = static_cast<uint32_t*>(dev_->get(16));
    scan_excl_u32(P->slab_n, off, P->nslabs, tot, dev_->scan, stream_);
    if (P->nslabs)
        k_export_slabs<<<std::min<uint32_t>(P->nslabs, 65536), 256, 0, stream_>>>(
            dev_->ar[P->arena], P->slab_off, P->slab_n, off, P->nslabs, reinterpret_cast<float4*>(dpts), dkeys);
    HIP_CHECK(hipGetLastError());
    std::vector<uint32_t> slab0(P->ncells + 1ull), hoff(P->nslabs + 1ull);
    HIP_CHECK(hipMemcpyAsync(xyz, P->cell_idx, 3ull * P->ncells * 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(sb, P->cell_sb, (uint64_t)P->ncells * 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(slab0.data(), P->cell_slab0, slab0.size() * 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(hoff.data(), off, (uint64_t)P->nslabs * 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    hoff[P->nslabs] = (uint32_t)P->arrivals;
    for (uint32_t c = 0; c < P->ncells; c++) cell_n[c] = hoff[slab0[c + 1]] - hoff[slab0[c]];
    dev_->release(mk);
    return 0;
}

HostPoints::~HostPoints() {
    if (p) munmap(p, cap * sizeof(Point));
}
void HostPoints::resize(uint64_t m) {
    if (m > cap) {
        if (p) munmap(p, cap * sizeof(Point));
        const uint64_t c = std::max<uint64_t>(m, 1);
        void* q = mmap(nullptr, c * sizeof(Point), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (q == MAP_FAILED) throw std::bad_alloc();
        madvise(q, c * sizeof(Point), MADV_HUGEPAGE);
        p = static_cast<Point*>(q);
        cap = c;
    }
    n = m;
}

int Engine::download_level(uint32_t i, LevelHost& H, HostPoints& grid, HostPoints& kept) {
    if (i >= levels_.size()) return -EINVAL;
    Level* L = levels_[i];
    H = LevelHost();
    H.h = L->h;
    auto cp = [&](auto& vec, auto* dptr, uint64_t n) {
        vec.resize(n);
        if (n) HIP_CHECK(hipMemcpyAsync(vec.data(), dptr, n * sizeof(vec[0]), hipMemcpyDeviceToHost, stream_));
    };
    cp(H.cell_idx, L->cell_idx, 3ull * L->ncells);
    cp(H.cell_slab0, L->cell_slab0, L->ncells + 1ull);
    cp(H.slab_grid_n, L->slab_grid_n, L->nslabs);
    cp(H.bkt_state, L->bkt_state, 8ull * L->ncells);
    cp(H.bkt_off, L->bkt_off, 8ull * L->ncells);
    cp(H.bkt_n, L->bkt_n, 8ull * L->ncells);
    // compacted winners
    const uint64_t mark = dev_->mark();
    uint32_t* cgo = static_cast<uint32_t*>(dev_->get(((uint64_t)L->nslabs + 1) * 4));
    uint32_t* tot = static_cast<uint32_t*>(dev_->get(4));
    uint32_t nwin = 0;
    if (L->nslabs) {
        scan_excl_u32(L->slab_grid_n, cgo, L->nslabs, tot, dev_->scan, stream_);
        HIP_CHECK(hipMemcpyAsync(&nwin, tot, 4, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipStreamSynchronize(stream_));
    }
    cp(H.slab_grid_off, cgo, L->nslabs);
    grid.resize(nwin);
    if (nwin) {
        Point* d = static_cast<Point*>(dev_->get((uint64_t)nwin * sizeof(Point)));
        k_compact_grid<<<std::min<uint32_t>(L->nslabs, 65536), 256, 0, stream_>>>(L->grid, L->grid_off, L->slab_grid_n,
                                                                                cgo, L->nslabs, d);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(grid.data(), d, (uint64_t)nwin * sizeof(Point), hipMemcpyDeviceToHost, stream_));
    }
    kept.resize(L->kept_used);
    if (L->kept_used) HIP_CHECK(hipMemcpyAsync(kept.data(), L->kept, (uint64_t)L->kept_used * sizeof(Point), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    dev_->release(mark);
    H.grid_base = 0;
    H.kept_base = 0;
    return 0;
}

// Grid winners of built level i per cell, compacted on the device (the sharded
// step's partial level-0 cells travel to their writers without a host copy).
// cgo = exclusive scan of the slabs' winner counts (slab order = cell order).
int Engine::grid_cells(uint32_t i, uint64_t& ncells, uint64_t& npoints) {
    if (i >= levels_.size()) return -EINVAL;
    Level* L = levels_[i];
    ncells = L->ncells;
    npoints = 0;
    if (!L->nslabs) return 0;
    const uint64_t mk = dev_->mark();
    uint32_t* cgo = static_cast<uint32_t*>(dev_->get(((uint64_t)L->nslabs + 1) * 4));
    uint32_t* tot = static_cast<uint32_t*>(dev_->get(4));
    uint32_t nwin = 0;
    scan_excl_u32(L->slab_grid_n, cgo, L->nslabs, tot, dev_->scan, stream_);
    HIP_CHECK(hipMemcpyAsync(&nwin, tot, 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    dev_->release(mk);
    npoints = nwin;
    return 0;
}

int Engine::export_grid(uint32_t i, int32_t* xyz, uint64_t* cell_n, Point* dpts) {
    if (i >= levels_.size()) return -EINVAL;
    Level* L = levels_[i];
    if (!L->ncells) return 0;
    const uint64_t mk = dev_->mark();
    uint32_t* cgo = static_cast<uint32_t*>(dev_->get(((uint64_t)L->nslabs + 1) * 4));
    uint32_t* tot = static_cast<uint32_t*>(dev_->get(4));
    std::vector<uint32_t> slab0(L->ncells + 1ull), hoff(L->nslabs + 1ull, 0);
    if (L->nslabs) {
        scan_excl_u32(L->slab_grid_n, cgo, L->nslabs, tot, dev_->scan, stream_);
        k_compact_grid<<<std::min<uint32_t>(L->nslabs, 65536), 256, 0, stream_>>>(L->grid, L->grid_off, L->slab_grid_n,
                                                                                cgo, L->nslabs, dpts);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(hoff.data(), cgo, (uint64_t)L->nslabs * 4, hipMemcpyDeviceToHost, stream_));
        HIP_CHECK(hipMemcpyAsync(hoff.data() + L->nslabs, tot, 4, hipMemcpyDeviceToHost, stream_));
    }
    HIP_CHECK(hipMemcpyAsync(xyz, L->cell_idx, 3ull * L->ncells * 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(slab0.data(), L->cell_slab0, slab0.size() * 4, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    dev_->release(mk);
    for (uint32_t c = 0; c < L->ncells; c++) cell_n[c] = hoff[slab0[c + 1]] - hoff[slab0[c]];
    return 0;
}

int Engine::download(std::vector<LevelHost>& out, std::vector<Point>& grid, std::vector<Point>& kept) {
    out.clear();
    grid.clear();
    kept.clear();
    HostPoints g, k;
    for (uint32_t i = 0; i < levels_.size(); i++) {
        LevelHost H;
        const int rc = download_level(i, H, g, k);
        if (rc) return rc;
        H.grid_base = grid.size();
        H.kept_base = kept.size();
        grid.insert(grid.end(), g.data(), g.data() + g.size());
        kept.insert(kept.end(), k.data(), k.data() + k.size());
        out.push_back(std::move(H));
    }
    return 0;
}

}  // namespace pcc

namespace pcc {
// ------------------------------------------------------------------ sharding
// Level-0 ownership for the multi-GPU build: every level-h cell has a unique
// level-0 ancestor, so level-0 cells are the unit of ownership.  The grid is
// spanned by the GLOBAL bounding box (all-reduced by the caller); a point's
// linear cell id is ((ix - lo.x) * dims.y + (iy - lo.y)) * dims.z + (iz - lo.z).
namespace {
struct ShardScratch {
    int device = -1;
    hipStream_t st = nullptr;
    uint32_t* buf[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t cap = 0;
    float* part = nullptr;
    float* nfpart = nullptr;   // shard_bbox_nonfinite's per-block partials
    uint32_t* flag = nullptr;
    uint32_t* cnt = nullptr;
    uint64_t* tab = nullptr;
    uint64_t* rt = nullptr;   // bucket resolution tables and sort buffers (shard_resolve_buckets)
    unsigned long long* ks = nullptr;   // its sort scratch of kept lists above kKeptMax
    uint64_t ks_cap = 0;
    uint64_t rt_cap = 0;
    SortTemp sort;
    ~ShardScratch() {
        for (auto* b : buf) (void)hipFree(b);
        (void)hipFree(part); (void)hipFree(nfpart); (void)hipFree(flag); (void)hipFree(cnt); (void)hipFree(tab); (void)hipFree(rt); (void)hipFree(ks);
        (void)hipFree(sort.counts); (void)hipFree(sort.scan.bsums);
        if (st) (void)hipStreamDestroy(st);
    }
};
thread_local std::unique_ptr<ShardScratch> t_shard;

ShardScratch& shard_scratch(int device) {
    HIP_CHECK(hipSetDevice(device));
    if (!t_shard || t_shard->device != device) {
        t_shard = std::make_unique<ShardScratch>();
        t_shard->device = device;
        HIP_CHECK(hipStreamCreateWithFlags(&t_shard->st, hipStreamNonBlocking));
        HIP_CHECK(hipMalloc(&t_shard->part, kBBoxBlocks * 6 * sizeof(float)));
        HIP_CHECK(hipMalloc(&t_shard->flag, 4));
        HIP_CHECK(hipMalloc(&t_shard->cnt, 64 * 4));
        HIP_CHECK(hipMalloc(&t_shard->tab, 132 * 8));
    }
    return *t_shard;
}

// A point with an infinite coordinate (its cells saturate, metadata.rs:100-102,
// and meet no finite point's: Engine::build_infinite) belongs to no grid cell;
// with inf0 it is routed with unit 0, so that one rank builds all of them.
__device__ __forceinline__ bool has_inf(float x, float y, float z) {
    return isinf(x) || isinf(y) || isinf(z);
}
__device__ __forceinline__ uint32_t shard_cell(const ShardGrid& g, float x, float y, float z) {
    const int32_t ix = cell_index1(x, g.cs) - g.lo[0], iy = cell_index1(y, g.cs) - g.lo[1], iz = cell_index1(z, g.cs) - g.lo[2];
    const bool in = ix >= 0 && iy >= 0 && iz >= 0 && (uint32_t)ix < g.dims[0] && (uint32_t)iy < g.dims[1] && (uint32_t)iz < g.dims[2];
    return in ? ((uint32_t)ix * g.dims[1] + (uint32_t)iy) * g.dims[2] + (uint32_t)iz : 0xFFFFFFFFu;
}

// Slab mode (dim2 > 0): the unit is the level-0 slab, id = cell * kL0Layers +
// local hex z-layer, the layer exactly as the engine's level-0 binning computes
// it (l0_layer: t = trunc(z / r0), minus the cell's first layer dim2*iz - 2).
struct ShardSlabs {
    float cr;        // level-0 hex radius (0: cell mode)
    int32_t dim2;    // 2 * sub_grid_dimension
};
template <bool INF0 = true>
__device__ __forceinline__ uint32_t shard_unit(const ShardGrid& g, const ShardSlabs& m, float x, float y, float z) {
    if (has_inf(x, y, z)) return INF0 ? 0u : 0xFFFFFFFFu;
    const uint32_t c = shard_cell(g, x, y, z);
    if (m.dim2 == 0 || c == 0xFFFFFFFFu) return c;
    const int32_t iz = cell_index1(z, g.cs);
    const int64_t ll = (int64_t)sat_i32(z / m.cr) - ((int64_t)m.dim2 * iz - 2);
    if (ll < 0 || ll >= (int64_t)kL0Layers) return 0xFFFFFFFFu;
    return c * kL0Layers + (uint32_t)ll;
}

constexpr int kShBS = 256;
// per-block LDS histogram (ncells <= kShLds), else global atomics.  BBOX: the
// same pass also takes the block's bounding box (part, as k_bbox) and flags
// non-finite coordinates (nf); points outside the grid are counted in bad.
constexpr uint32_t kShLds = 16384;
template <bool BBOX>
__global__ __launch_bounds__(kShBS) void k_shard_hist(const Point* __restrict__ in, uint64_t n, ShardGrid g,
                                                      ShardSlabs m, uint32_t ncells, uint32_t* hist, uint32_t* bad,
                                                      float* part, uint32_t* nf) {
    extern __shared__ uint32_t h[];   // ncells words when ncells <= kShLds (dynamic: small grids keep occupancy)
    const bool lds = ncells <= kShLds;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool nfin = false;
    if (lds)
        for (uint32_t i = threadIdx.x; i < ncells; i += kShBS) h[i] = 0;
    __syncthreads();
    const float4* p4 = reinterpret_cast<const float4*>(in);
    uint32_t nbad = 0;
    constexpr int U = 4;   // loads in flight per thread
    const uint64_t stride = (uint64_t)gridDim.x * kShBS;
    for (uint64_t i0 = blockIdx.x * (uint64_t)kShBS + threadIdx.x; i0 < n; i0 += U * stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = i0 + u * stride;
            v[u] = p4[i < n ? i : n - 1];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (i0 + u * stride >= n) break;
            if constexpr (BBOX) {
                nfin |= !(isfinite(v[u].x) && isfinite(v[u].y) && isfinite(v[u].z));
                mn[0] = fminf(mn[0], v[u].x); mn[1] = fminf(mn[1], v[u].y); mn[2] = fminf(mn[2], v[u].z);
                mx[0] = fmaxf(mx[0], v[u].x); mx[1] = fmaxf(mx[1], v[u].y); mx[2] = fmaxf(mx[2], v[u].z);
            }
            // the fused pass over a guessed grid counts an infinite point as
            // outside it (the caller then histograms the true grid)
            const uint32_t c = shard_unit<!BBOX>(g, m, v[u].x, v[u].y, v[u].z);
            if (c == 0xFFFFFFFFu) { nbad++; continue; }
            if (lds) atomicAdd(&h[c], 1u); else wave_aggregated_add(hist, c);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
    if constexpr (BBOX) {
        for (int d = 32; d > 0; d >>= 1)
            for (int a = 0; a < 3; a++) {
                mn[a] = fminf(mn[a], __shfl_xor(mn[a], d, 64));
                mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], d, 64));
            }
        __shared__ float sbb[kShBS / 64][6];
        if (nfin) atomicOr(nf, 1u);
        if ((threadIdx.x & 63) == 0)
            for (int a = 0; a < 3; a++) { sbb[threadIdx.x / 64][a] = mn[a]; sbb[threadIdx.x / 64][3 + a] = mx[a]; }
        __syncthreads();
        if (threadIdx.x < 6) {
            float r = sbb[0][threadIdx.x];
            for (int q = 1; q < kShBS / 64; q++)
                r = threadIdx.x < 3 ? fminf(r, sbb[q][threadIdx.x]) : fmaxf(r, sbb[q][threadIdx.x]);
            part[blockIdx.x * 6 + threadIdx.x] = r;
        }
    }
    __syncthreads();
    if (lds)
        for (uint32_t i = threadIdx.x; i < ncells; i += kShBS)
            if (h[i]) atomicAdd(&hist[i], h[i]);
}

// Stable partition by destination rank in two passes over the points (no sort,
// no random gather): per 4096-point tile the points per destination
// (k_route_count), an exclusive scan over (destination, tile), then every tile
// writes its points in index order to its runs (k_route_scatter).  Ranks inside
// a 256-point chunk come from wave peer masks and per-wave counts in LDS.
constexpr int kRtBS = 256, kRtIPT = 16, kRtTile = kRtBS * kRtIPT, kRtW = kRtBS / 64;
__device__ __forceinline__ uint32_t route_dest_rank(const ShardGrid& g, const ShardSlabs& m, const uint32_t* owner,
                                                    uint32_t nranks, const float4& v, uint32_t& bad) {
    const uint32_t u = shard_unit(g, m, v.x, v.y, v.z);
    uint32_t o = u == 0xFFFFFFFFu ? 0xFFFFFFFFu : owner[u];
    if (o >= nranks) { bad = 1u; o = 0; }
    return o;
}

__global__ __launch_bounds__(kRtBS) void k_route_count(const Point* __restrict__ in, uint32_t n, ShardGrid g,
                                                       ShardSlabs m, const uint32_t* __restrict__ owner,
                                                       uint32_t nranks, uint32_t ntiles, uint32_t* counts,
                                                       uint32_t* flag) {
    __shared__ uint32_t c[64];
    if (threadIdx.x < 64) c[threadIdx.x] = 0;
    __syncthreads();
    const float4* p4 = reinterpret_cast<const float4*>(in);
    const uint32_t tile = blockIdx.x;
    uint32_t bad = 0;
#pragma unroll 4
    for (int r = 0; r < kRtIPT; r++) {
        const uint32_t i = tile * (uint32_t)kRtTile + (uint32_t)r * kRtBS + threadIdx.x;
        const bool valid = i < n;
        uint32_t o = 64;
        if (valid) o = route_dest_rank(g, m, owner, nranks, p4[i], bad);
        const uint64_t peers = wave_peers<7>(o, valid);
        if (valid && mask_rank(peers) == 0) atomicAdd(&c[o], (uint32_t)__popcll(peers));
    }
    if (bad) atomicOr(flag, 1u);
    __syncthreads();
    if (threadIdx.x < nranks) counts[(uint64_t)threadIdx.x * ntiles + tile] = c[threadIdx.x];
}

__global__ __launch_bounds__(kRtBS) void k_route_scatter(const Point* __restrict__ in, uint32_t n, ShardGrid g,
                                                         ShardSlabs m, const uint32_t* __restrict__ owner,
                                                         uint32_t nranks, uint32_t ntiles,
                                                         const uint32_t* __restrict__ base, uint32_t key0,
                                                         Point* __restrict__ out, uint32_t* __restrict__ keys,
                                                         unsigned long long* __restrict__ bm, uint32_t nwords) {
    __shared__ uint32_t run[64];
    __shared__ uint32_t wc[2][kRtW][64];
    const uint32_t tid = threadIdx.x, w = tid / 64, lane = tid & 63;
    const uint32_t tile = blockIdx.x;
    if (tid < nranks) run[tid] = base[(uint64_t)tid * ntiles + tile];
    const float4* p4 = reinterpret_cast<const float4*>(in);
    float4* o4 = reinterpret_cast<float4*>(out);
    uint32_t bad = 0;
    for (int r = 0; r < kRtIPT; r++) {
        const uint32_t par = (uint32_t)r & 1u;
        const uint32_t i = tile * (uint32_t)kRtTile + (uint32_t)r * kRtBS + tid;
        const bool valid = i < n;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t o = 64;
        if (valid) {
            v = p4[i];
            o = route_dest_rank(g, m, owner, nranks, v, bad);
        }
        const uint64_t peers = wave_peers<7>(o, valid);
        const uint32_t rk = mask_rank(peers);
        wc[par][w][lane] = 0;   // this wave's row (the other parity is still read by the run update)
        __builtin_amdgcn_wave_barrier();
        if (valid && rk == 0) wc[par][w][o] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[o] + rk;
            for (uint32_t q = 0; q < w; q++) pos += wc[par][q][o];
            o4[pos] = v;
            if (keys) keys[pos] = key0 + i;
            // membership bitmap: the wave's 64 indices are one aligned word
            if (bm && rk == 0) bm[(uint64_t)o * nwords + (i >> 6)] = peers;
        }
        __syncthreads();
        if (tid < nranks) {
            uint32_t t = 0;
            for (uint32_t q = 0; q < (uint32_t)kRtW; q++) t += wc[par][q][tid];
            run[tid] += t;
        }
    }
    (void)bad;
}

// per destination: its first position (scan value at (r, tile 0)); the end from the total
__global__ void k_route_totals(const uint32_t* base, uint32_t ntiles, uint32_t nranks, const uint32_t* total,
                               uint32_t* first) {
    const uint32_t r = threadIdx.x;
    if (r < nranks) first[r] = base[(uint64_t)r * ntiles];
    if (r == nranks) first[r] = *total;
}
// One-pass form (pcc_shard_route_bitmaps_hist).  The rank's own unit histogram
// (the points per unit that pcc_shard_histogram / pcc_shard_slab_histogram counted
// over the same points, computed anyway for the plan) gives every destination's
// total, so its first position is known before a point is read; each 4096-point
// tile then takes its offsets inside the destinations from its predecessors by
// decoupled look-back (publish the tile's counts, walk back to the nearest
// inclusive prefix) and scatters in index order as k_route_scatter does: one
// read of the points instead of two.  Tiles are numbered by a ticket, so every
// predecessor a tile waits for is already running.  A histogram that does not
// match the points sets flag bit 2 (prefixes above a total, or the last tile's
// prefix unequal to it) and no store leaves the send buffer.
constexpr unsigned long long kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = (1ull << 62) - 1;

__global__ __launch_bounds__(256) void k_route_dest_totals(const uint32_t* __restrict__ hist, uint32_t nunits,
                                                           const uint32_t* __restrict__ owner, uint32_t nranks,
                                                           unsigned long long* __restrict__ tot, uint32_t* flag) {
    __shared__ unsigned long long s[64];
    if (threadIdx.x < 64) s[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < nunits; u += gridDim.x * 256u) {
        const uint32_t h = hist[u];
        if (!h) continue;
        const uint32_t o = owner[u];
        if (o >= nranks) { atomicOr(flag, 1u); continue; }
        atomicAdd(&s[o], (unsigned long long)h);
    }
    __syncthreads();
    if (threadIdx.x < nranks && s[threadIdx.x]) atomicAdd(&tot[threadIdx.x], s[threadIdx.x]);
}

__global__ __launch_bounds__(kRtBS) void k_route_lb(const Point* __restrict__ in, uint32_t n, ShardGrid g, ShardSlabs m,
                                                    const uint32_t* __restrict__ owner, uint32_t nranks, uint32_t ntiles,
                                                    const unsigned long long* __restrict__ tot,
                                                    unsigned long long* __restrict__ status, uint32_t* ticket,
                                                    Point* __restrict__ out, unsigned long long* __restrict__ bm,
                                                    uint32_t nwords, uint32_t* flag) {
    __shared__ uint32_t run[64], cnt[64];
    __shared__ uint32_t wc[2][kRtW][64];
    __shared__ uint32_t s_tile;
    const uint32_t tid = threadIdx.x, w = tid / 64, lane = tid & 63;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    if (tid < 64) cnt[tid] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const float4* p4 = reinterpret_cast<const float4*>(in);
    float4* o4 = reinterpret_cast<float4*>(out);
    // pass 1 (registers): the tile's points, and per row the destination, wave
    // rank and wave count (o | rk << 8 | pc << 16; o = 64: no point); bitmap words
    float4 v[kRtIPT];
    uint32_t meta[kRtIPT];
    uint32_t bad = 0;
#pragma unroll
    for (int r = 0; r < kRtIPT; r++) {
        const uint32_t i = tile * (uint32_t)kRtTile + (uint32_t)r * kRtBS + tid;
        v[r] = p4[i < n ? i : n - 1];
    }
#pragma unroll
    for (int r = 0; r < kRtIPT; r++) {
        const uint32_t i = tile * (uint32_t)kRtTile + (uint32_t)r * kRtBS + tid;
        const bool valid = i < n;
        uint32_t o = 64;
        if (valid) o = route_dest_rank(g, m, owner, nranks, v[r], bad);
        const uint64_t peers = wave_peers<7>(o, valid);
        const uint32_t rk = mask_rank(peers), pc = (uint32_t)__popcll(peers);
        meta[r] = o | (rk << 8) | (pc << 16);
        if (valid && rk == 0) {
            atomicAdd(&cnt[o], pc);
            bm[(uint64_t)o * nwords + (i >> 6)] = peers;   // the wave's 64 indices: one aligned word
        }
    }
    if (bad) atomicOr(flag, 1u);
    __syncthreads();
    // look-back, one thread per destination
    if (tid < nranks) {
        const uint32_t c = cnt[tid];
        unsigned long long* st = status + (uint64_t)tile * nranks + tid;
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(st, kLbInc | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(st, kLbAgg | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (uint32_t p = tile; p-- > 0;) {
                const unsigned long long* sp = status + (uint64_t)p * nranks + tid;
                unsigned long long sv;
                while (((sv = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 62) == 0)
                    __builtin_amdgcn_s_sleep(1);
                excl += sv & kLbVal;
                if ((sv >> 62) == 2) break;
            }
            __hip_atomic_store(st, kLbInc | (excl + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        uint64_t start = 0;
        for (uint32_t q = 0; q < tid; q++) start += tot[q];
        if (excl + c > tot[tid]) atomicOr(flag, 2u);                             // more points than counted
        if (tile + 1 == ntiles && excl + c != tot[tid]) atomicOr(flag, 2u);   // fewer
        run[tid] = (uint32_t)(start + excl);
    }
    // pass 2: scatter in index order (k_route_scatter's ranks, from the registers)
    for (int r = 0; r < kRtIPT; r++) {
        const uint32_t par = (uint32_t)r & 1u;
        const uint32_t i = tile * (uint32_t)kRtTile + (uint32_t)r * kRtBS + tid;
        const uint32_t o = meta[r] & 0xFFu, rk = (meta[r] >> 8) & 0xFFu;
        const bool valid = i < n && o < nranks;
        wc[par][w][lane] = 0;   // this wave's row (the other parity is still read by the run update)
        __builtin_amdgcn_wave_barrier();
        if (valid && rk == 0) wc[par][w][o] = meta[r] >> 16;
        __syncthreads();
        if (valid) {
            uint32_t pos = run[o] + rk;
            for (uint32_t q = 0; q < w; q++) pos += wc[par][q][o];
            if (pos < n) o4[pos] = v[r];
        }
        __syncthreads();
        if (tid < nranks) {
            uint32_t t = 0;
            for (uint32_t q = 0; q < (uint32_t)kRtW; q++) t += wc[par][q][tid];
            run[tid] += t;
        }
    }
}

// Keys of received points from the senders' membership bitmaps (concatenated in
// sender order): word popcounts, their exclusive scan (= the received rows'
// positions), then every word writes the keys of its set bits in order.
__global__ void k_bm_pop(const unsigned long long* __restrict__ bm, uint32_t nw, uint32_t* __restrict__ pc) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w < nw) pc[w] = (uint32_t)__popcll(bm[w]);
}
__global__ void k_bm_keys(const unsigned long long* __restrict__ bm, uint32_t nw, const uint32_t* __restrict__ pos,
                          const uint64_t* __restrict__ wstart, const uint64_t* __restrict__ key0, uint32_t nsrc,
                          uint32_t* __restrict__ keys, uint32_t nkeys) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    uint32_t sidx = 0;
    while (sidx + 1 < nsrc && wstart[sidx + 1] <= w) sidx++;
    const uint32_t kb = (uint32_t)(key0[sidx] + 64ull * (w - wstart[sidx]));
    unsigned long long m = bm[w];
    uint32_t p = pos[w];
    while (m && p < nkeys) {   // (more bits than received rows: the caller reports the mismatch)
        const uint32_t b = (uint32_t)__ffsll((long long)m) - 1u;
        keys[p++] = kb + b;
        m &= m - 1ull;
    }
}

// Rank-local start of global batch start key gs[i]: the received points with a
// smaller global key (senders in rank = key order; wstart[s] = the first word of
// sender s's row, wstart[nsrc] = nw; pos = exclusive word popcount prefix,
// *total its sum).
__global__ void k_bm_starts(const unsigned long long* __restrict__ bm, const uint32_t* __restrict__ pos,
                            const uint32_t* __restrict__ total, const uint64_t* __restrict__ wstart,
                            const uint64_t* __restrict__ key0, uint32_t nsrc, const uint64_t* __restrict__ gs,
                            uint64_t nb, uint64_t* __restrict__ out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= nb) return;
    const uint64_t g = gs[i];
    const uint32_t nw = (uint32_t)wstart[nsrc];
    auto at = [&](uint64_t w) -> uint64_t { return w < nw ? pos[w] : *total; };
    if (nsrc == 0 || g < key0[0]) { out[i] = 0; return; }
    uint32_t s = 0;
    while (s + 1 < nsrc && key0[s + 1] <= g) s++;
    const uint64_t off = g - key0[s], w = off >> 6, ws = wstart[s], we = wstart[s + 1];
    if (ws + w >= we) { out[i] = at(we); return; }   // past sender s's points
    const uint32_t b = (uint32_t)(off & 63u);
    const unsigned long long below = b ? (bm[ws + w] & ((1ull << b) - 1ull)) : 0ull;
    out[i] = at(ws + w) + (uint64_t)__popcll(below);
}

// ---- shared cells' overflow buckets, resolved over every rank's emissions
// (cell.rs:108-153; the numpy statement is pcconv/dist.py::resolve_bucket).
// Emissions arrive in segments (a cell's arrivals from one rank: sorted runs per
// slab, not sorted as a whole); a bucket's keys are distinct.  Nothing is
// sorted but the kept lists: a bucket of tot > L points spills, at the batch of
// its want-th smallest key (want = L, or L + 1 when its first batch holds
// exactly L), found by a 4-pass radix select over the bucket's keys; a bucket of
// tot <= L keeps its list (unless tot == L over two batches, then it spills at
// its largest key), ranked by key in LDS.  The rows are walked in chunks of at
// most kRsChunk rows of one segment (one bucket per workgroup).
constexpr uint32_t kRsChunk = 4096;   // (kKeptMax: the kept-list capacity, as k_bucket's)
struct BucketTabs {
    const uint32_t* files;      // 4 u32 per file: start lo/hi, first batch, batch size
    uint32_t nfiles;
    const uint64_t* start;      // per segment: first row, rows, bucket
    const uint64_t* len;
    const uint64_t* segb;
    const uint64_t* inoff;      // per segment: rows of the bucket's earlier segments
    const uint64_t* tot;        // per bucket: rows
    const uint64_t* boff;       // per bucket: its segments bsegs[boff[b] .. boff[b+1]), in order
    const uint64_t* bsegs;
    const uint64_t* chunk;      // per chunk: segment | row offset in it << 32 (rows: min(kRsChunk, rest))
    uint32_t nchunks;
    uint32_t* hist;             // per bucket 256 digit counts (radix select)
    uint32_t* sel;              // per bucket: prefix, rank left, kmin, kmax, fk, first, next key, pad
    uint64_t* out;              // per bucket: state | spill batch << 32
    uint64_t* base;             // per bucket: kept base, sub base (exclusive scans)
    unsigned long long* ksort;  // limit > kKeptMax: sort scratch of the kept lists above the LDS
                                // capacity, at twice their kept base (nullptr otherwise)
    uint32_t nbuckets, limit;
};
enum { SEL_PREFIX, SEL_RANK, SEL_KMIN, SEL_KMAX, SEL_FK, SEL_FIRST, SEL_NEXT, SEL_PAD, SEL_W };
static_assert(SEL_W % 2 == 0, "whole u64 words per bucket");

// one pass over a chunk: pass 0 = min / max key of every bucket and the top
// key byte's histogram; passes 1-3 the next bytes among the keys that match the
// selected prefix (pass 1 also counts the keys below the first batch's end);
// pass 4 the least key above the selected one.  Buckets of tot <= L only take
// part in pass 0.
__global__ __launch_bounds__(256) void k_rsel(BucketTabs T, const uint32_t* __restrict__ keys, int pass) {
    __shared__ uint32_t h[256];
    __shared__ uint32_t red[3];
    const uint64_t cw = T.chunk[blockIdx.x];
    const uint32_t sg = (uint32_t)cw, o = (uint32_t)(cw >> 32);
    const uint32_t b = (uint32_t)T.segb[sg];
    const bool sel = T.tot[b] > T.limit;
    if (pass > 0 && !sel) return;   // block-uniform
    const uint64_t r0 = T.start[sg] + o;
    const uint32_t n = (uint32_t)min<uint64_t>(kRsChunk, T.len[sg] - o);
    uint32_t* S = T.sel + (uint64_t)b * SEL_W;
    const int shift = 24 - 8 * (pass < 4 ? pass : 3);
    const uint32_t hi = pass == 0 ? 0u : (pass >= 4 ? 0xFFFFFFFFu : 0xFFFFFFFFu << (32 - 8 * pass));
    const uint32_t pref = S[SEL_PREFIX], fk = S[SEL_FK];
    h[threadIdx.x] = 0;
    if (threadIdx.x < 3) red[threadIdx.x] = threadIdx.x == 0 ? 0xFFFFFFFFu : 0u;
    __syncthreads();
    uint32_t mn = 0xFFFFFFFFu, mx = 0, below = 0;
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        const uint32_t k = keys[r0 + i];
        if (pass == 0) {
            mn = min(mn, k);
            mx = max(mx, k);
        }
        if (pass == 4) {
            if (k > pref) mn = min(mn, k);
        } else if (sel && ((k ^ pref) & hi) == 0) {
            atomicAdd(&h[(k >> shift) & 255u], 1u);
        }
        if (pass == 1) below += k < fk ? 1u : 0u;
    }
    // wave reductions, then one LDS atomic per wave
    for (int d = 32; d >= 1; d >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, d, 64));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
        below += (uint32_t)__shfl_xor((int)below, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&red[0], mn);
        atomicMax(&red[1], mx);
        atomicAdd(&red[2], below);
    }
    __syncthreads();
    if (pass < 4 && sel && h[threadIdx.x]) atomicAdd(&T.hist[(uint64_t)b * 256 + threadIdx.x], h[threadIdx.x]);
    if (threadIdx.x == 0) {
        if (pass == 0) {
            atomicMin(&S[SEL_KMIN], red[0]);
            atomicMax(&S[SEL_KMAX], red[1]);
        }
        if (pass == 1) atomicAdd(&S[SEL_FIRST], red[2]);
        if (pass == 4) atomicMin(&S[SEL_NEXT], red[0]);
    }
}
// per bucket after pass p < 4: the digit holding the rank-th smallest key,
// appended to the prefix; after pass 0 also the end of the first key's batch
__global__ void k_rsel_pick(BucketTabs T, int pass) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= T.nbuckets) return;
    uint32_t* S = T.sel + (uint64_t)b * SEL_W;
    if (pass == 0) S[SEL_FK] = first_key_after(T.files, T.nfiles, event_batch(T.files, T.nfiles, S[SEL_KMIN]));
    if (T.tot[b] <= T.limit) return;
    uint32_t* hb = T.hist + (uint64_t)b * 256;
    uint32_t rank = S[SEL_RANK], d = 0;
    for (; d < 255; d++) {
        const uint32_t c = hb[d];
        if (rank < c) break;
        rank -= c;
    }
    for (uint32_t q = 0; q < 256; q++) hb[q] = 0;
    S[SEL_RANK] = rank;
    S[SEL_PREFIX] |= d << (24 - 8 * pass);
}
// states, spill batches, and the exclusive scans of kept / spilled rows (one block)
__global__ __launch_bounds__(1024) void k_bkt_state(BucketTabs T) {
    __shared__ uint64_t part[1024][2];
    const uint32_t L = T.limit, per = (T.nbuckets + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * per, b1 = min(b0 + per, T.nbuckets);
    uint64_t ak = 0, as = 0;
    for (uint32_t b = b0; b < b1; b++) {
        const uint32_t* S = T.sel + (uint64_t)b * SEL_W;
        const uint64_t tot = T.tot[b];
        uint64_t st = 1;
        if (tot > L) {   // want = L, or L + 1 when the first batch holds exactly L
            const uint32_t k = S[SEL_FIRST] == L ? S[SEL_NEXT] : S[SEL_PREFIX];
            st = 2ull | ((uint64_t)event_batch(T.files, T.nfiles, k) << 32);
        } else if (tot == L && tot > 0) {
            const uint32_t e1 = event_batch(T.files, T.nfiles, S[SEL_KMAX]);
            if (event_batch(T.files, T.nfiles, S[SEL_KMIN]) != e1) st = 2ull | ((uint64_t)e1 << 32);
        }
        T.out[b] = st;
        if ((uint32_t)st == 1) ak += tot; else as += tot;
    }
    part[threadIdx.x][0] = ak;
    part[threadIdx.x][1] = as;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t k = 0, q = 0;
        for (int t = 0; t < 1024; t++) {
            const uint64_t a = part[t][0], c = part[t][1];
            part[t][0] = k;
            part[t][1] = q;
            k += a;
            q += c;
        }
    }
    __syncthreads();
    ak = part[threadIdx.x][0];
    as = part[threadIdx.x][1];
    for (uint32_t b = b0; b < b1; b++) {
        T.base[2 * b] = ak;
        T.base[2 * b + 1] = as;
        if ((uint32_t)T.out[b] == 1) ak += T.tot[b]; else as += T.tot[b];
    }
}
// spilled buckets: every row (pts + keys) to sub base + earlier segments of its bucket + its index
__global__ void k_bkt_sub(BucketTabs T, const Point* __restrict__ pts, const uint32_t* __restrict__ keys,
                          Point* __restrict__ sub, uint32_t* __restrict__ sub_keys) {
    const uint64_t cw = T.chunk[blockIdx.x];
    const uint32_t sg = (uint32_t)cw, o = (uint32_t)(cw >> 32);
    const uint32_t b = (uint32_t)T.segb[sg];
    if ((uint32_t)T.out[b] != 2) return;
    const uint64_t r0 = T.start[sg] + o, d0 = T.base[2 * b + 1] + T.inoff[sg] + o;
    const uint32_t n = (uint32_t)min<uint64_t>(kRsChunk, T.len[sg] - o);
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        reinterpret_cast<float4*>(sub)[d0 + i] = reinterpret_cast<const float4*>(pts)[r0 + i];
        sub_keys[d0 + i] = keys[r0 + i];
    }
}
// kept buckets (one workgroup each): the bucket's keys in LDS, every row's rank
// = the keys below its own (distinct keys), row to kept base + rank.  A list
// above the LDS capacity (limit > kKeptMax) is bitonic-sorted as packed words
// (key << 32 | row) in the global scratch at twice its kept base, as k_bucket
// does (a power-of-two padding below twice the list never reaches the next
// list's; the workgroup barrier orders the scratch's accesses: one workgroup owns it)
__global__ __launch_bounds__(1024) void k_bkt_kept(BucketTabs T, const Point* __restrict__ pts,
                                                   const uint32_t* __restrict__ keys, Point* __restrict__ kept) {
    __shared__ uint32_t sk[kKeptMax];
    __shared__ uint32_t sr[kKeptMax];
    const uint32_t b = blockIdx.x;
    if ((uint32_t)T.out[b] != 1 || T.tot[b] == 0) return;
    const uint32_t tot = (uint32_t)T.tot[b];
    if (tot > (uint32_t)kKeptMax) {
        if (!T.ksort) return;   // (the host allocates it whenever such a list can be kept)
        unsigned long long* sw = T.ksort + 2 * T.base[2 * b];
        uint32_t o = 0;
        for (uint64_t j = T.boff[b]; j < T.boff[b + 1]; j++) {
            const uint64_t sg = T.bsegs[j], r0 = T.start[sg];
            const uint32_t n = (uint32_t)T.len[sg];
            for (uint32_t i = threadIdx.x; i < n; i += 1024)
                sw[o + i] = ((unsigned long long)keys[r0 + i] << 32) | (uint32_t)(r0 + i);
            o += n;
        }
        uint32_t np2 = 1;
        while (np2 < tot) np2 <<= 1;
        for (uint32_t i = tot + threadIdx.x; i < np2; i += 1024) sw[i] = ~0ull;
        __syncthreads();
        for (uint32_t kk = 2; kk <= np2; kk <<= 1)
            for (uint32_t jj = kk >> 1; jj > 0; jj >>= 1) {
                for (uint32_t p = threadIdx.x; p < np2 / 2; p += 1024) {
                    const uint32_t i = ((p & ~(jj - 1)) << 1) | (p & (jj - 1)), ix = i | jj;
                    const bool up = (i & kk) == 0;
                    const unsigned long long a = sw[i], c = sw[ix];
                    if ((a > c) == up) { sw[i] = c; sw[ix] = a; }
                }
                __syncthreads();
            }
        const uint64_t kb = T.base[2 * b];
        for (uint32_t i = threadIdx.x; i < tot; i += 1024)
            reinterpret_cast<float4*>(kept)[kb + i] = reinterpret_cast<const float4*>(pts)[(uint32_t)sw[i]];
        return;
    }
    uint32_t o = 0;
    for (uint64_t j = T.boff[b]; j < T.boff[b + 1]; j++) {
        const uint64_t sg = T.bsegs[j], r0 = T.start[sg];
        const uint32_t n = (uint32_t)T.len[sg];
        for (uint32_t i = threadIdx.x; i < n; i += 1024) {
            sk[o + i] = keys[r0 + i];
            sr[o + i] = (uint32_t)(r0 + i);
        }
        o += n;
    }
    __syncthreads();
    const uint64_t kb = T.base[2 * b];
    for (uint32_t i = threadIdx.x; i < tot; i += 1024) {
        const uint32_t k = sk[i];
        uint32_t r = 0;
        for (uint32_t q = 0; q < tot; q++) r += sk[q] < k ? 1u : 0u;
        reinterpret_cast<float4*>(kept)[kb + r] = reinterpret_cast<const float4*>(pts)[sr[i]];
    }
}

}  // namespace

int shard_keys_from_bitmaps(const uint64_t* dbm, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                            uint32_t* dkeys, uint64_t nkeys, int device) {
    ShardScratch& S = shard_scratch(device);
    if (nsrc == 0 || nsrc > 64) return -EINVAL;
    std::vector<uint64_t> tab(2 * nsrc + 1);
    uint64_t nw = 0;
    for (uint32_t s = 0; s < nsrc; s++) {
        tab[s] = nw;
        tab[nsrc + 1 + s] = key0[s];
        nw += nwords[s];
    }
    tab[nsrc] = nw;
    if (nw >= (1ull << 32) || nkeys >= (1ull << 32)) return -EOVERFLOW;
    if (S.cap < nw + 2 * 65) {
        for (auto*& b : S.buf) { (void)hipFree(b); b = nullptr; HIP_CHECK(hipMalloc(&b, std::max<uint64_t>(nw + 2 * 65, 1) * 4)); }
        S.cap = nw + 2 * 65;
    }
    uint64_t* dtab = S.tab;   // word start per sender, the end, first key per sender (<= 129 words)
    HIP_CHECK(hipMemcpyAsync(dtab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, S.st));
    uint32_t total = 0;
    if (nw) {
        const auto* bm = reinterpret_cast<const unsigned long long*>(dbm);
        k_bm_pop<<<(uint32_t)((nw + 255) / 256), 256, 0, S.st>>>(bm, (uint32_t)nw, S.buf[0]);
        scan_excl_u32(S.buf[0], S.buf[0], (uint32_t)nw, S.buf[1], S.sort.scan, S.st);
        k_bm_keys<<<(uint32_t)((nw + 255) / 256), 256, 0, S.st>>>(bm, (uint32_t)nw, S.buf[0], dtab, dtab + nsrc + 1,
                                                                  nsrc, dkeys, (uint32_t)nkeys);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(&total, S.buf[1], 4, hipMemcpyDeviceToHost, S.st));
    }
    HIP_CHECK(hipStreamSynchronize(S.st));
    return total == nkeys ? 0 : -EBADMSG;
}

int shard_batch_starts(const uint64_t* dbm, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                       const uint64_t* gstarts, uint64_t nb, uint64_t* local, int device) {
    ShardScratch& S = shard_scratch(device);
    if (nsrc == 0 || nsrc > 64) return -EINVAL;
    std::vector<uint64_t> tab(2 * nsrc + 1);
    uint64_t nw = 0;
    for (uint32_t s = 0; s < nsrc; s++) {
        tab[s] = nw;
        tab[nsrc + 1 + s] = key0[s];
        if (s && key0[s] < key0[s - 1]) return -EINVAL;   // senders in key order
        nw += nwords[s];
    }
    tab[nsrc] = nw;
    if (nw >= (1ull << 32)) return -EOVERFLOW;
    for (uint64_t b = 1; b < nb; b++)
        if (gstarts[b] < gstarts[b - 1]) return -EINVAL;
    if (!nb) return 0;
    if (S.cap < nw + 2 * 65) {
        for (auto*& b : S.buf) { (void)hipFree(b); b = nullptr; HIP_CHECK(hipMalloc(&b, std::max<uint64_t>(nw + 2 * 65, 1) * 4)); }
        S.cap = nw + 2 * 65;
    }
    uint64_t* dtab = S.tab;
    HIP_CHECK(hipMemcpyAsync(dtab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, S.st));
    HIP_CHECK(hipMemsetAsync(S.buf[1], 0, 4, S.st));
    const auto* bm = reinterpret_cast<const unsigned long long*>(dbm);
    if (nw) {
        k_bm_pop<<<(uint32_t)((nw + 255) / 256), 256, 0, S.st>>>(bm, (uint32_t)nw, S.buf[0]);
        scan_excl_u32(S.buf[0], S.buf[0], (uint32_t)nw, S.buf[1], S.sort.scan, S.st);
    }
    uint64_t* dgs = nullptr;
    HIP_CHECK(hipMalloc(&dgs, nb * 16));
    HIP_CHECK(hipMemcpyAsync(dgs, gstarts, nb * 8, hipMemcpyHostToDevice, S.st));
    k_bm_starts<<<(uint32_t)((nb + 255) / 256), 256, 0, S.st>>>(bm, S.buf[0], S.buf[1], dtab, dtab + nsrc + 1, nsrc,
                                                                 dgs, nb, dgs + nb);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(local, dgs + nb, nb * 8, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    HIP_CHECK(hipFree(dgs));
    return 0;
}

int shard_resolve_buckets(const uint64_t* seg_n, const uint32_t* seg_bucket, uint64_t nseg, uint32_t nbuckets,
                          const Point* dpts, const uint32_t* dkeys, const uint64_t* file_points, uint64_t nfiles,
                          uint32_t batch, uint32_t limit, uint32_t* state, uint32_t* spill_batch, uint64_t* kept_n,
                          Point* dkept, Point* dsub, uint32_t* dsub_keys, uint64_t* nkept, uint64_t* nsub, int device) {
    ShardScratch& S = shard_scratch(device);
    *nkept = *nsub = 0;
    if (!nbuckets) return 0;
    if (!nfiles || nseg == 0) return -EINVAL;
    if (limit == 0 || limit > (1u << 24)) return -EINVAL;   // (the engine's limit, Engine::open)
    batch = std::max<uint32_t>(batch, 1);
    std::vector<uint64_t> tot(nbuckets, 0), boff(nbuckets + 1ull, 0), start(nseg), segb(nseg), inoff(nseg), chunks;
    uint64_t nrows = 0;
    for (uint64_t s = 0; s < nseg; s++) {
        const uint32_t b = seg_bucket[s];
        if (b >= nbuckets) return -EINVAL;
        start[s] = nrows;
        inoff[s] = tot[b];
        nrows += seg_n[s];
        tot[b] += seg_n[s];
        segb[s] = b;
        boff[b + 1]++;
        if (seg_n[s] >= (1ull << 32)) return -EOVERFLOW;
        for (uint64_t o = 0; o < seg_n[s]; o += kRsChunk) chunks.push_back(s | (o << 32));
    }
    if (nrows >= (1ull << 32) || nseg >= (1ull << 32)) return -EOVERFLOW;
    for (uint32_t b = 0; b < nbuckets; b++) boff[b + 1] += boff[b];
    std::vector<uint64_t> bsegs(nseg), fill(boff.begin(), boff.end() - 1);
    for (uint64_t s = 0; s < nseg; s++) bsegs[fill[seg_bucket[s]]++] = s;
    // file table as the engine's (lib.rs:31-52: batches restart at every file,
    // an empty file is one empty batch)
    std::vector<uint32_t> ft;
    uint64_t g = 0;
    uint32_t eb = 0;
    for (uint64_t f = 0; f < nfiles; f++) {
        ft.insert(ft.end(), {(uint32_t)g, (uint32_t)(g >> 32), eb, batch});
        g += file_points[f];
        eb += (uint32_t)std::max<uint64_t>(1, (file_points[f] + batch - 1) / batch);
    }
    const uint64_t nch = chunks.size();
    const uint64_t wf = (ft.size() + 1) / 2;
    const uint64_t w_start = wf, w_len = w_start + nseg, w_segb = w_len + nseg, w_inoff = w_segb + nseg,
                   w_tot = w_inoff + nseg, w_boff = w_tot + nbuckets, w_bsegs = w_boff + nbuckets + 1,
                   w_chunk = w_bsegs + nseg, w_sel = w_chunk + nch,                     // SEL_W u32 per bucket
                   w_hist = w_sel + (uint64_t)nbuckets * SEL_W / 2,                      // 256 u32 per bucket
                   w_out = w_hist + (uint64_t)nbuckets * 128, w_base = w_out + nbuckets,
                   words = w_base + 2ull * nbuckets;
    if (S.rt_cap < words) {
        (void)hipFree(S.rt);
        S.rt = nullptr;
        HIP_CHECK(hipMalloc(&S.rt, words * 8));
        S.rt_cap = words;
    }
    std::vector<uint64_t> blob(w_out, 0);
    memcpy(blob.data(), ft.data(), ft.size() * 4);
    memcpy(blob.data() + w_start, start.data(), nseg * 8);
    memcpy(blob.data() + w_len, seg_n, nseg * 8);
    memcpy(blob.data() + w_segb, segb.data(), nseg * 8);
    memcpy(blob.data() + w_inoff, inoff.data(), nseg * 8);
    memcpy(blob.data() + w_tot, tot.data(), nbuckets * 8ull);
    memcpy(blob.data() + w_boff, boff.data(), boff.size() * 8);
    memcpy(blob.data() + w_bsegs, bsegs.data(), nseg * 8);
    if (nch) memcpy(blob.data() + w_chunk, chunks.data(), nch * 8);
    uint32_t* sel0 = reinterpret_cast<uint32_t*>(blob.data() + w_sel);
    for (uint32_t b = 0; b < nbuckets; b++) {   // select the L-th smallest key (rank L - 1)
        uint32_t* q = sel0 + (uint64_t)b * SEL_W;
        q[SEL_RANK] = limit - 1;
        q[SEL_KMIN] = 0xFFFFFFFFu;
        q[SEL_NEXT] = 0xFFFFFFFFu;
    }
    BucketTabs T;
    T.files = reinterpret_cast<const uint32_t*>(S.rt);
    T.nfiles = (uint32_t)nfiles;
    T.start = S.rt + w_start;
    T.len = S.rt + w_len;
    T.segb = S.rt + w_segb;
    T.inoff = S.rt + w_inoff;
    T.tot = S.rt + w_tot;
    T.boff = S.rt + w_boff;
    T.bsegs = S.rt + w_bsegs;
    T.chunk = S.rt + w_chunk;
    T.nchunks = (uint32_t)nch;
    T.sel = reinterpret_cast<uint32_t*>(S.rt + w_sel);
    T.hist = reinterpret_cast<uint32_t*>(S.rt + w_hist);
    T.out = S.rt + w_out;
    T.base = S.rt + w_base;
    T.nbuckets = nbuckets;
    T.limit = limit;
    // kept lists above the LDS capacity: their sort scratch (twice the rows any
    // kept bucket can hold, i.e. of the buckets with tot <= limit)
    T.ksort = nullptr;
    uint64_t kmax_rows = 0;
    bool big = false;
    for (uint32_t b = 0; b < nbuckets; b++)
        if (tot[b] <= limit) {
            kmax_rows += tot[b];
            big |= tot[b] > (uint64_t)kKeptMax;
        }
    if (big) {
        if (S.ks_cap < 2 * kmax_rows) {
            (void)hipFree(S.ks);
            S.ks = nullptr;
            HIP_CHECK(hipMalloc(&S.ks, 2 * kmax_rows * 8));
            S.ks_cap = 2 * kmax_rows;
        }
        T.ksort = S.ks;
    }
    HIP_CHECK(hipMemcpyAsync(S.rt, blob.data(), w_out * 8, hipMemcpyHostToDevice, S.st));   // (hist: zeros)
    const uint32_t pb = (nbuckets + 63) / 64;
    for (int pass = 0; pass <= 4; pass++) {
        if (nch) k_rsel<<<(uint32_t)nch, 256, 0, S.st>>>(T, dkeys, pass);
        if (pass < 4) k_rsel_pick<<<pb, 64, 0, S.st>>>(T, pass);
    }
    k_bkt_state<<<1, 1024, 0, S.st>>>(T);
    if (nch) k_bkt_sub<<<(uint32_t)nch, 256, 0, S.st>>>(T, dpts, dkeys, dsub, dsub_keys);
    k_bkt_kept<<<nbuckets, 1024, 0, S.st>>>(T, dpts, dkeys, dkept);
    HIP_CHECK(hipGetLastError());
    std::vector<uint64_t> out(nbuckets);
    HIP_CHECK(hipMemcpyAsync(out.data(), T.out, nbuckets * 8ull, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    uint64_t ok = 0, os = 0;
    for (uint32_t b = 0; b < nbuckets; b++) {
        state[b] = (uint32_t)out[b];
        spill_batch[b] = (uint32_t)(out[b] >> 32);
        kept_n[b] = state[b] == 1 ? tot[b] : 0;
        (state[b] == 1 ? ok : os) += tot[b];
    }
    *nkept = ok;
    *nsub = os;
    return 0;
}

int shard_synth(Point* dst, uint64_t idx0, uint64_t n, uint64_t seed, int kind, float lo, float ext, int device) {
    ShardScratch& S = shard_scratch(device);
    if (n) k_synth_at<<<grid_for(n, 256, 1 << 20), 256, 0, S.st>>>(dst, idx0, n, seed, kind, lo, ext);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(S.st));
    return 0;
}

int shard_bbox(const Point* d, uint64_t n, float bmin[3], float bmax[3], int device) {
    ShardScratch& S = shard_scratch(device);
    for (int a = 0; a < 3; a++) { bmin[a] = INFINITY; bmax[a] = -INFINITY; }
    if (!n) return 0;
    HIP_CHECK(hipMemsetAsync(S.flag, 0, 4, S.st));
    const unsigned nbb = grid_for(n, kBBoxBS, kBBoxBlocks);
    k_bbox<<<nbb, kBBoxBS, 0, S.st>>>(d, n, S.part, S.flag);
    k_bbox_final<<<1, 256, 0, S.st>>>(S.part, nbb);
    HIP_CHECK(hipGetLastError());
    float bb[6];
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(bb, S.part, sizeof bb, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipMemcpyAsync(&bad, S.flag, 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    if (bad) return -EDOM;   // non-finite coordinates: shard_bbox_nonfinite
    for (int a = 0; a < 3; a++) { bmin[a] = bb[a]; bmax[a] = bb[3 + a]; }
    return 0;
}

// The reference's box and the cell extent of an input with non-finite
// coordinates (k_bbox_nf's kNfParts values, reduced over the points).
int shard_bbox_nonfinite(const Point* d, uint64_t n, float parts[15], int device) {
    ShardScratch& S = shard_scratch(device);
    for (int a = 0; a < 3; a++) {
        parts[a] = INFINITY; parts[3 + a] = -INFINITY; parts[6 + a] = 0.f;
        parts[9 + a] = INFINITY; parts[12 + a] = -INFINITY;
    }
    if (!n) return 0;
    const uint32_t nb = (uint32_t)std::min<uint64_t>((n + 255) / 256, kBBoxBlocks);
    if (!S.nfpart) HIP_CHECK(hipMalloc(&S.nfpart, (size_t)kBBoxBlocks * kNfParts * 4));
    k_bbox_nf<<<nb, 256, 0, S.st>>>(d, n, S.nfpart);
    k_bbox_nf_final<<<1, 64, 0, S.st>>>(S.nfpart, nb);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(parts, S.nfpart, kNfParts * 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    return 0;
}

static ShardSlabs shard_slabs(const ShardGrid& g, uint32_t dim) {
    ShardSlabs m;
    m.cr = dim ? hex_radius(sub_cell_size(g.cs, dim)) : 0.0f;
    m.dim2 = 2 * (int32_t)dim;
    return m;
}

int shard_histogram(const Point* d, uint64_t n, const ShardGrid& g, uint32_t* dhist, int device, uint32_t dim) {
    ShardScratch& S = shard_scratch(device);
    const uint64_t nc = (uint64_t)g.dims[0] * g.dims[1] * g.dims[2] * (dim ? kL0Layers : 1u);
    if (nc >= (1ull << 32)) return -EOVERFLOW;
    HIP_CHECK(hipMemsetAsync(dhist, 0, nc * 4, S.st));
    HIP_CHECK(hipMemsetAsync(S.flag, 0, 4, S.st));
    const size_t smem = nc <= kShLds ? (size_t)nc * 4 : 0;
    if (n) k_shard_hist<false><<<grid_for(n, kShBS, 2048), kShBS, smem, S.st>>>(d, n, g, shard_slabs(g, dim), (uint32_t)nc,
                                                                                dhist, S.flag, nullptr, nullptr);
    HIP_CHECK(hipGetLastError());
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(&bad, S.flag, 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    return bad ? -ERANGE : 0;
}

// The local bounding box and the slab (dim > 0) or cell histogram over a grid
// guessed before the box is known, in one pass: points outside the guess are
// counted in *outside (the caller falls back to shard_histogram on the true
// grid when any rank has some).  -EDOM: non-finite coordinates.
int shard_bbox_histogram(const Point* d, uint64_t n, const ShardGrid& g, uint32_t dim, uint32_t* dhist, float bmin[3],
                         float bmax[3], uint64_t* outside, int device) {
    ShardScratch& S = shard_scratch(device);
    for (int a = 0; a < 3; a++) { bmin[a] = INFINITY; bmax[a] = -INFINITY; }
    *outside = 0;
    const uint64_t nc = (uint64_t)g.dims[0] * g.dims[1] * g.dims[2] * (dim ? kL0Layers : 1u);
    if (nc >= (1ull << 32)) return -EOVERFLOW;
    HIP_CHECK(hipMemsetAsync(dhist, 0, nc * 4, S.st));
    if (!n) { HIP_CHECK(hipStreamSynchronize(S.st)); return 0; }
    HIP_CHECK(hipMemsetAsync(S.flag, 0, 4, S.st));
    HIP_CHECK(hipMemsetAsync(S.cnt, 0, 4, S.st));
    const size_t smem = nc <= kShLds ? (size_t)nc * 4 : 0;
    const uint32_t nb = grid_for(n, kShBS, std::min<uint32_t>(2048, kBBoxBlocks));
    k_shard_hist<true><<<nb, kShBS, smem, S.st>>>(d, n, g, shard_slabs(g, dim), (uint32_t)nc, dhist, S.cnt, S.part,
                                                  S.flag);
    k_bbox_final<<<1, 256, 0, S.st>>>(S.part, nb);
    HIP_CHECK(hipGetLastError());
    float bb[6];
    uint32_t nf = 0, out = 0;
    HIP_CHECK(hipMemcpyAsync(bb, S.part, sizeof bb, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipMemcpyAsync(&nf, S.flag, 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipMemcpyAsync(&out, S.cnt, 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    if (nf) return -EDOM;
    for (int a = 0; a < 3; a++) { bmin[a] = bb[a]; bmax[a] = bb[3 + a]; }
    *outside = out;
    return 0;
}

// Bounding box of a sample of the points (one tile of kL0Tile in every
// ntiles / 512): the guess the fused pass above is made over.
int shard_bbox_sample(const Point* d, uint64_t n, float bmin[3], float bmax[3], int device) {
    ShardScratch& S = shard_scratch(device);
    for (int a = 0; a < 3; a++) { bmin[a] = INFINITY; bmax[a] = -INFINITY; }
    if (!n) return 0;
    const uint64_t ntiles = (n + kL0Tile - 1) / kL0Tile;
    const uint32_t nb = (uint32_t)std::min<uint64_t>(ntiles, 512);
    k_bbox_sample<<<nb, 256, 0, S.st>>>(d, n, ntiles, nb, S.part);
    k_bbox_final<<<1, 256, 0, S.st>>>(S.part, nb);
    HIP_CHECK(hipGetLastError());
    float bb[6];
    HIP_CHECK(hipMemcpyAsync(bb, S.part, sizeof bb, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    for (int a = 0; a < 3; a++) {
        if (!(std::isfinite(bb[a]) && std::isfinite(bb[3 + a]))) return -EDOM;
        bmin[a] = bb[a];
        bmax[a] = bb[3 + a];
    }
    return 0;
}

int shard_route(const Point* d, uint64_t n, uint32_t key0, const ShardGrid& g, const uint32_t* downer, uint32_t nranks,
                Point* dsend, uint32_t* dkeys, uint64_t* counts, int device, uint32_t dim, uint64_t* dbm) {
    ShardScratch& S = shard_scratch(device);
    if (nranks == 0 || nranks > 64) return -EINVAL;
    if (n >= (1ull << 32)) return -EOVERFLOW;
    const uint32_t n32 = (uint32_t)n;
    const uint32_t ntiles = (uint32_t)((n + kRtTile - 1) / kRtTile);
    const uint64_t nc = (uint64_t)ntiles * nranks;
    if (S.cap < nc + 2 * 65) {
        for (auto*& b : S.buf) { (void)hipFree(b); b = nullptr; HIP_CHECK(hipMalloc(&b, std::max<uint64_t>(nc + 2 * 65, 1) * 4)); }
        S.cap = nc + 2 * 65;
    }
    HIP_CHECK(hipMemsetAsync(S.flag, 0, 4, S.st));
    uint32_t first[65] = {};
    if (n) {
        const ShardSlabs m = shard_slabs(g, dim);
        k_route_count<<<ntiles, kRtBS, 0, S.st>>>(d, n32, g, m, downer, nranks, ntiles, S.buf[0], S.flag);
        scan_excl_u32(S.buf[0], S.buf[1], (uint32_t)nc, S.buf[2], S.sort.scan, S.st);
        const uint32_t nwords = (uint32_t)((n + 63) / 64);
        if (dbm) HIP_CHECK(hipMemsetAsync(dbm, 0, (uint64_t)nranks * nwords * 8, S.st));
        k_route_scatter<<<ntiles, kRtBS, 0, S.st>>>(d, n32, g, m, downer, nranks, ntiles, S.buf[1], key0, dsend, dkeys,
                                                    reinterpret_cast<unsigned long long*>(dbm), nwords);
        k_route_totals<<<1, 128, 0, S.st>>>(S.buf[1], ntiles, nranks, S.buf[2], S.buf[3]);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(first, S.buf[3], (nranks + 1) * 4, hipMemcpyDeviceToHost, S.st));
    }
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(&bad, S.flag, 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    for (uint32_t r = 0; r < nranks; r++) counts[r] = n ? (uint64_t)(first[r + 1] - first[r]) : 0;
    return bad ? -ERANGE : 0;
}

int shard_route_hist(const Point* d, uint64_t n, const ShardGrid& g, const uint32_t* downer, uint32_t nranks,
                     const uint32_t* dhist, Point* dsend, uint64_t* dbm, uint64_t* counts, int device, uint32_t dim) {
    ShardScratch& S = shard_scratch(device);
    if (nranks == 0 || nranks > 64) return -EINVAL;
    if (n >= (1ull << 32)) return -EOVERFLOW;
    const uint64_t nunits = (uint64_t)g.dims[0] * g.dims[1] * g.dims[2] * (dim ? kL0Layers : 1u);
    if (nunits >= (1ull << 32)) return -EOVERFLOW;
    const uint32_t n32 = (uint32_t)n;
    const uint32_t ntiles = (uint32_t)((n + kRtTile - 1) / kRtTile);
    // status words (ntiles x nranks u64), the totals (64 u64) and the ticket, in u32 units
    const uint64_t need = ((uint64_t)ntiles * nranks + 64 + 1) * 2;
    if (S.cap < need) {
        for (auto*& b : S.buf) { (void)hipFree(b); b = nullptr; HIP_CHECK(hipMalloc(&b, std::max<uint64_t>(need, 1) * 4)); }
        S.cap = need;
    }
    unsigned long long* status = reinterpret_cast<unsigned long long*>(S.buf[0]);
    unsigned long long* tot = status + (uint64_t)ntiles * nranks;
    uint32_t* ticket = reinterpret_cast<uint32_t*>(tot + 64);
    HIP_CHECK(hipMemsetAsync(S.buf[0], 0, need * 4, S.st));
    HIP_CHECK(hipMemsetAsync(S.flag, 0, 4, S.st));
    if (nunits)
        k_route_dest_totals<<<(uint32_t)std::min<uint64_t>((nunits + 255) / 256, 1024), 256, 0, S.st>>>(
            dhist, (uint32_t)nunits, downer, nranks, tot, S.flag);
    if (n) {
        const uint32_t nwords = (uint32_t)((n + 63) / 64);
        HIP_CHECK(hipMemsetAsync(dbm, 0, (uint64_t)nranks * nwords * 8, S.st));
        k_route_lb<<<ntiles, kRtBS, 0, S.st>>>(d, n32, g, shard_slabs(g, dim), downer, nranks, ntiles, tot, status,
                                              ticket, dsend, reinterpret_cast<unsigned long long*>(dbm), nwords, S.flag);
    }
    HIP_CHECK(hipGetLastError());
    unsigned long long ht[64];
    uint32_t bad = 0;
    HIP_CHECK(hipMemcpyAsync(ht, tot, nranks * 8, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipMemcpyAsync(&bad, S.flag, 4, hipMemcpyDeviceToHost, S.st));
    HIP_CHECK(hipStreamSynchronize(S.st));
    uint64_t sum = 0;
    for (uint32_t r = 0; r < nranks; r++) { counts[r] = ht[r]; sum += ht[r]; }
    if ((bad & 2u) || sum != n) return -EBADMSG;
    return bad ? -ERANGE : 0;
}

}  // namespace pcc
