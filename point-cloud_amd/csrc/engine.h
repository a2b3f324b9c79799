// engine.h — device-resident hierarchy/LOD build for MI355X (gfx950).
//
// Reference path replaced: point-converter/src/converter.rs:96-139
// (add_points_batch -> add_points_in_hierarchy, per batch, per level) together
// with cell.rs:70-153 (grid LOD + overflow buckets).  The engine runs the
// SURVEY.md Appendix C level-synchronous restatement: all batches at once,
// one pass per level over "slabs" = (cell, hex z-layer), each slab processed
// by one workgroup with its slot table in LDS.  See DESIGN.md.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <sys/mman.h>
#include <memory>
#include <string>
#include <type_traits>
#include <initializer_list>
#include <utility>
#include <vector>

#include <hip/hip_runtime.h>

namespace pcc {

struct Point { float x, y, z; uint8_t rgba[4]; };  // == point.rs:8-14 on-disk record (16 B)
static_assert(sizeof(Point) == 16, "Point must be 16 bytes");

struct Config {                     // metadata.rs:67-88
    uint32_t cell_point_overflow_limit = 5000;
    uint32_t sub_grid_dimension = 96;
    float max_cell_size = 1000.0f;
};

// Host copy of one level's results (filled by Engine::download()).
struct LevelHost {
    uint32_t h = 0;
    std::vector<int32_t> cell_idx;      // 3 per cell
    std::vector<uint32_t> cell_slab0;   // ncells + 1
    std::vector<uint32_t> slab_grid_off, slab_grid_n;
    std::vector<uint32_t> bkt_state;    // 8 per cell: 0 absent, 1 kept (Some), 2 spilled (None)
    std::vector<uint32_t> bkt_off, bkt_n;
    uint64_t grid_base = 0;             // offset of this level's winner region in the downloaded grid array
    uint64_t kept_base = 0;             // offset of this level's kept lists in the downloaded kept array
};

// Host staging for downloaded points: uninitialised (no zero fill) and advised
// for transparent huge pages, grown only, so a level's D2H is not paced by
// first-touch page faults.
struct HostPoints {
    Point* p = nullptr;
    uint64_t n = 0, cap = 0;
    HostPoints() = default;
    HostPoints(const HostPoints&) = delete;
    HostPoints& operator=(const HostPoints&) = delete;
    ~HostPoints();
    void resize(uint64_t m);
    Point* data() { return p; }
    const Point* data() const { return p; }
    uint64_t size() const { return n; }
};

// Existing cloud loaded for an incremental merge (lib.rs:86-101 +
// converter.rs:187-207).  Its points are "seeds" with
// keys below every new point's (keys 0 .. S-1, a pseudo batch 0): per level h,
// first the grid points of every level-h cell, then the points of every kept
// (Some) list in stored order; forced_lo[h] = first key of level h's kept seeds.
//
// Only TOUCHED cells are rebuilt (cells that receive new arrivals; the
// reference loads a cell only when a batch touches it, converter.rs:160-207):
//   * level-0 seeds enter the level-0 binning ahead of the new points (seeds0,
//     key order);
//   * a level-h >= 1 seed is injected straight into its own slab: the parent
//     level reserves room in front of each child slab's emission region
//     (child_seed counts), and when the child cell is created (its bucket is
//     None and receives new emissions) its seeds are copied there;
//   * at its own level a grid seed takes its slot first (it precedes every new
//     point, so it wins every tie), and a kept seed (key >= forced_lo[h]) is a
//     forced emission into its bucket, ahead of the new emissions;
//   * untouched cells stay exactly as they were (the caller keeps them).
// A level-h slab with seeds always has its parent slab at level h-1: its
// points passed that layer, and the first arrival of a slab always takes a slot.
struct PriorCell { int32_t x, y, z; uint32_t st; };   // st: 2 bits per octant: 0 absent, 1 Some, 2 None
constexpr uint32_t kNoPriorSlab = 0xFFFFFFFFu;
struct PriorSlabRec {                                  // one (cell, hex layer) of the existing cloud
    uint32_t seed_off, nseed;                          // level >= 1: its seeds in PriorState::inj
    uint32_t ngrid, pad;                               // of them grid points (the first ngrid, one per slot)
    uint32_t child[24];                                // its child slabs' records at level h+1 (kNoPriorSlab: none)
    uint32_t dcap[24];                                 // its seeds per child slab (their capacities)
};
struct PriorLevel {
    std::vector<PriorCell> cells;                      // sorted by (x, y, z)
    std::vector<uint32_t> cell_slab0;                  // ncells + 1: each cell's records, ascending layer
    std::vector<int32_t> slab_layer;
    std::vector<PriorSlabRec> slabs;
};
// std::allocator that default-initialises: large host arrays that are filled
// right after their allocation (by several threads) are not zero-filled first.
// Arrays of 2 MB or more are mapped 2 MB-aligned with transparent huge pages
// advised: the first touch of a 16 GB cloud then takes ~8k page faults, not ~4M.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = DefaultInitAlloc<U>; };
    DefaultInitAlloc() = default;
    template <class U> DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    static constexpr size_t kHuge = size_t(2) << 20;
    T* allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < kHuge) return std::allocator<T>::allocate(n);
        const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
        void* q = mmap(nullptr, len + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (q == MAP_FAILED) throw std::bad_alloc();
        const uintptr_t b0 = reinterpret_cast<uintptr_t>(q), a = (b0 + kHuge - 1) & ~uintptr_t(kHuge - 1);
        if (a > b0) munmap(q, a - b0);
        if (b0 + len + kHuge > a + len) munmap(reinterpret_cast<void*>(a + len), b0 + len + kHuge - (a + len));
        madvise(reinterpret_cast<void*>(a), len, MADV_HUGEPAGE);
        return reinterpret_cast<T*>(a);
    }
    void deallocate(T* p, size_t n) noexcept {
        const size_t bytes = n * sizeof(T);
        if (bytes < kHuge) {
            std::allocator<T>::deallocate(p, n);
            return;
        }
        munmap(p, (bytes + kHuge - 1) & ~(kHuge - 1));
    }
    template <class U> void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
template <class T> using HostVec = std::vector<T, DefaultInitAlloc<T>>;

// One cell file as Cell::read_from sees it (cell.rs:183-229, Header::read_from
// cell.rs:300-335): grid points in file order, overflow entries in file order
// (n == 0 <=> None, cell.rs:210-212).  Also the engine's cells of points with
// an infinite coordinate (Engine::side_cells).
struct CellFile {
    uint32_t h = 0;
    int32_t idx[3] = {0, 0, 0};
    uint32_t total = 0, number = 0, overflow = 0;
    HostVec<Point> grid;
    struct Entry {
        int32_t child[3];
        bool some;
        HostVec<Point> pts;
    };
    std::vector<Entry> entries;
};

struct PriorState {
    uint64_t nseeds = 0;                               // S: every existing point
    HostVec<Point> seeds0;                             // level-0 seeds, key order (keys 0 .. seeds0.size()-1)
    HostVec<Point> inj;                                // levels >= 1, grouped by level, cell, slab: grid then kept
    HostVec<uint32_t> inj_keys;
    std::vector<uint64_t> forced_lo;                   // per prior level
    std::vector<PriorLevel> levels;
    bool has_nan = false;                              // some seed has a NaN coordinate (the NaN slot rules apply)
    float max_abs = 0.f;                               // largest |finite coordinate| of a seed
};

struct StageProfile {
    double level0_ms = 0, dense_ms = 0, small_ms = 0, bucket_ms = 0, next_ms = 0;
    uint64_t dense_arrivals = 0, small_arrivals = 0;
    uint32_t dense_launches = 0, small_launches = 0;
};

struct BuildStats {
    uint32_t levels = 0;
    uint64_t cells = 0, slabs = 0, arrivals = 0;   // arrivals = W
    uint64_t grid_points = 0, kept_points = 0;
    double ms_total = 0, ms_level0_bin = 0;
    uint64_t pre0_tiles = 0;                       // level-0 pass-0 tiles counted while the input uploaded
    uint32_t l0_fold = 0;                          // level-0 binning with pass 0 folded into pass 1
    uint32_t seq_replay = 0;                       // the whole build ran as the sequential replay
    std::vector<double> ms_level;                  // per level (slab + bucket kernels)
};

// Engine::readback: up to four small device ranges (multiples of 4 bytes)
struct RbSrc { const uint32_t* p[4]; uint32_t n[4]; };
struct RbPart { void* host; const void* dev; size_t bytes; };
constexpr uint32_t kReadbackWords = 1024;

class Engine {
public:
    Engine(const Config& cfg, int device, hipStream_t stream = nullptr);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    // Reserve device input capacity for n points (also sizes the arenas).
    void reserve(uint64_t n);
    // Append a "file": n points (host or device pointer) = ceil(n/batch) batches
    // (lib.rs:31-52: a file end is a batch boundary).  batch >= 1.
    void add_file_host(const Point* pts, uint64_t n, uint32_t batch);
    void add_file_device(const Point* dpts, uint64_t n, uint32_t batch);
    // Streaming upload of one file (HIP-stream scheduler): host pieces are
    // staged through a ring of pinned buffers and copied on a copy stream while
    // the caller reads the next piece.  stream_end(keep): the file is the first
    // `keep` points pushed (a truncated file keeps its complete batches).
    void stream_begin(uint64_t expected);
    void stream_push(const Point* pts, uint64_t n);
    uint64_t stream_end(uint64_t keep, uint32_t batch);
    void stream_cancel();   // the open file contributes nothing
    // A file whose reader yields k empty batches (ASCII PLY quirk, ply.rs:43-51).
    void add_empty_batches(uint32_t k) { nbatches_ += k; }
    // Synthetic input generated straight into HBM (bench / tests).
    void add_file_synth(uint64_t seed, int kind, uint64_t n, uint32_t batch, float lo, float ext);

    // Sharded build.  declare_files() fixes the GLOBAL file/batch
    // structure (points per file, in CLI order) without adding points; then
    // add_keyed_device() appends this shard's points with their global input
    // indices (keys, ascending).  Event batches come from the global table.
    void declare_files(const uint64_t* file_points, uint64_t nfiles, uint32_t batch);
    // Rank-local keys: input point i (a borrowed or added device input in key
    // order, keys = indices) belongs to event batch eb[k] for the last k with
    // starts[k] <= i; total_batches = the global batch count (lib.rs:31-52).
    void set_event_table(const uint64_t* starts, const uint32_t* eb, uint64_t n, uint64_t total_batches);
    // Points [first, last) of the borrowed input (set_keyed_external, keys NULL)
    // are in place: level-0 pass 1 of the groups they complete runs behind.
    // after: a stream whose work so far wrote those points (NULL: already in place).
    int input_landed(uint64_t first, uint64_t last, hipStream_t after);
    void add_keyed_device(const Point* dpts, const uint32_t* dkeys, uint64_t n);
    // Zero-copy variant: the build reads this shard's n points and keys straight
    // from caller memory (e.g. the buffers an exchange received into), which must
    // stay valid and unchanged until the next build() returns.  Replaces any
    // keyed input; no other input may be added afterwards.
    void set_keyed_external(const Point* dpts, const uint32_t* dkeys, uint64_t n);
    // Level ranges (sharded build of a heavy level-0 cell).
    // set_max_levels(m): build levels h0 .. h0+m-1 only; the next level's
    // arrivals stay on the device as the "pending" level, exported per cell
    // (contiguous, slab order, each slab in key order) with the spill batch of
    // its parent bucket.  set_root_level(h0) + set_root_spill_batches(): build
    // a sub-tree whose input is such exported arrivals of level-h0 cells.
    // raw: the last built level forwards every emission (no bucket lists; the
    // caller resolves those buckets, e.g. across the ranks sharing a cell)
    void set_max_levels(uint32_t m, bool raw = false);
    void set_root_level(uint32_t h0) { h0_ = h0; }
    void set_root_spill_batches(const int32_t* xyz, const uint32_t* sb, uint64_t n);
    int pending_info(uint64_t& ncells, uint64_t& npoints) const;
    int export_pending(int32_t* xyz, uint32_t* sb, uint64_t* cell_n, Point* dpts, uint32_t* dkeys);
    // Drops all input (points, keys, files) but keeps device allocations.
    void clear_input();
    // Incremental merge: the existing cloud's state (kept until the engine dies).
    void set_prior(const PriorState& p);
    bool has_prior() const { return prior_; }

    // Run the whole build on the device.  Returns 0 or a negative error code
    // (message in last_error()).  Input must already be resident.
    int build();
    int download(std::vector<LevelHost>& levels, std::vector<Point>& grid, std::vector<Point>& kept);
    // one level (grid winners compacted on the device); H's bases are 0
    int download_level(uint32_t i, LevelHost& H, HostPoints& grid, HostPoints& kept);
    // level i's grid winners per cell into device memory (cell order, each cell's
    // slabs in layer order); cells' (x, y, z) and winner counts on the host
    int grid_cells(uint32_t i, uint64_t& ncells, uint64_t& npoints);
    int export_grid(uint32_t i, int32_t* xyz, uint64_t* cell_n, Point* dpts);
    uint32_t num_levels() const;
    // (h, x, y, z) of every cell the last build produced (merge: the touched cells)
    int built_cells(std::vector<int32_t>& hxyz);

    uint64_t num_points() const { return n_; }
    uint32_t num_batches() const { return nbatches_; }
    const float* bbox_min() const { return bmin_; }
    const float* bbox_max() const { return bmax_; }
    uint32_t hierarchies() const { return hierarchies_; }
    // The cells of the points with an infinite coordinate (built apart, see
    // build_infinite()); empty for other inputs.  Not part of any level.
    const std::vector<CellFile>& side_cells() const { return side_; }
    const BuildStats& stats() const { return stats_; }
    void set_profiling(bool on) { profiling_ = on; }
    const StageProfile& profile() const { return prof_; }
    const std::string& last_error() const { return err_; }
    hipStream_t stream() const { return stream_; }

    // device pointer of the input (16 B AoS points), for benchmarking
    Point* device_input() { return d_in_; }
    // the new points of this build (own buffer or the borrowed keyed input)
    const Point* input_points() const { return ext_in_ ? ext_in_ : d_in_; }

private:
    struct Level;     // device tables of one level
    struct Dev;       // device buffers
    int fail(int code, const std::string& msg);
    int geom_fail(const char* msg);
    void ev_begin(int stage);
    void ev_end(int stage);
    void ev_collect();
    int level0_bin();
    int fold_hint(float cs);
    int enter_nonfinite(uint32_t flags);
    int build_infinite();
    void readback(std::initializer_list<RbPart> parts);
    void readback_begin(std::initializer_list<RbPart> parts);
    void readback_end();
    std::vector<RbPart> rb_parts_;
    hipEvent_t rb_ev_ = nullptr;
    int build_wide();
    int replay_whole(const Point* src, const uint32_t* keys, uint64_t n, const char* why);
    bool geom_fault_ = false;   // run_level: only hexagon / slot geometry flags (saturated indices)
    int replay_seq(const Point* pts, const uint32_t* keys, uint64_t n);
    // level-0 pass 0 behind the host-to-device copy (add_file_host, streamed files)
    void pre0_count(uint64_t upto, hipEvent_t after, bool all);
    void pre0_reset();
    int run_level(uint32_t li);
    void run_dcap(Level* L);
    void quiesce();
    void free_all();
    void free_prior();

    Config cfg_;
    int device_;
    hipStream_t stream_;
    bool own_stream_ = false;
    struct Staging { Point* host = nullptr; hipEvent_t done = nullptr; bool busy = false; };
    static constexpr uint64_t kStagePts = 4ull << 20;   // 64 MB per pinned buffer
    static constexpr int kStages = 4;
    Staging stage_[kStages];
    int stage_i_ = 0;
    hipStream_t copy_ = nullptr;
    uint64_t stream_n_ = 0;                              // points pushed into the open file
    // level-0 pass 0 of the uploaded prefix: 64 layer-digit counts per tile, the
    // running bounding box (+ per-block partials) and the non-finite flag
    static constexpr uint64_t kPrePiece = 32ull << 20;  // points per copy piece of add_file_host (512 MB)
    static constexpr uint32_t kPreBlocks = 1024;
    uint16_t* d_tile6_ = nullptr;
    uint64_t tile6_cap_ = 0, pre_tiles_ = 0;
    // Folded level-0 pass 1 (k_l0_tile6) behind the upload instead of pass 0,
    // when the first landed piece's sample box spans at most two level-0 cells
    // per axis: groups of pre6_tpg_ tiles as their copies land, run records with
    // a row stride of the reserved capacity's tiles (pre6_tcap_), compacted when
    // the build takes them over (level0_bin).
    bool pre_decided_ = false, pre6_ = false;
    uint32_t pre6_tpg_ = 0, pre6_gdone_ = 0, pre6_gcap_ = 0;
    uint64_t pre6_tcap_ = 0;
    uint32_t* d_pre6_cnt_ = nullptr;
    uint32_t* d_pre6_ph_ = nullptr;
    uint32_t* d_pre6_gpar_ = nullptr;
    uint64_t pre6_alloc_tiles_ = 0, pre6_alloc_groups_ = 0;
    const void* pre6_ar1_ = nullptr;
    void* d_pre6_dummy_ = nullptr;       // k_l0_tile6's scratch for its entry stores (persistent, not the build pool)
    bool pre6_run(uint64_t upto, hipEvent_t after, bool all);
    // Borrowed device input landing in pieces (a sharded rank's exchange):
    // level-0 pass 1 runs on every group of tiles whose points have all landed.
    std::vector<std::pair<uint64_t, uint64_t>> landed_;   // disjoint, sorted point ranges
    std::vector<uint8_t> pre6_done_;                      // per group: pass 1 run (landing mode)
    const Point* pre6_src_ = nullptr;                     // the input pass 1 ran on
    uint32_t* d_pre6_glist_ = nullptr;                    // group lists of the landing launches (in launch order)
    std::vector<uint32_t> pre6_glist_;                    // (host copy: the async uploads' source)
    uint64_t pre6_glist_cap_ = 0;
    uint64_t pre6_ndone_ = 0;                             // groups run
    hipEvent_t land_ev_ = nullptr;                        // the landing stream's progress
    float* d_prepart_ = nullptr;
    uint32_t* d_preflag_ = nullptr;
    hipEvent_t pre_ev_ = nullptr;
    uint64_t n_ = 0, cap_ = 0;
    uint32_t nbatches_ = 0;
    std::vector<uint64_t> file_start_;   // first point index per file
    std::vector<uint32_t> file_eb0_;     // first batch index per file
    std::vector<uint32_t> file_batch_;   // batch size per file
    Point* d_in_ = nullptr;
    uint32_t* d_keys_ = nullptr;         // keyed (sharded) input: global key per point
    uint32_t h0_ = 0, max_levels_ = 0;   // level range (set_root_level / set_max_levels)
    bool raw_last_ = false;
    Level* pending_ = nullptr;           // the first level not built (max_levels_)
    std::vector<int32_t> root_xyz_;      // root cells (sorted) and their spill batches
    std::vector<uint32_t> root_sb_;
    const Point* ext_in_ = nullptr;      // set_keyed_external(): borrowed input instead of d_in_/d_keys_
    const uint32_t* ext_keys_ = nullptr;
    // build source: d_in_ (n_ points) or, when merging, [seeds | d_in_]
    const Point* src_ = nullptr;
    uint64_t nsrc_ = 0;
    uint32_t nfiles_dev_ = 0;            // entries of the device file table
    bool prior_ = false;
    Point* d_seeds_ = nullptr;           // level-0 seeds (key order)
    uint64_t nseeds0_ = 0;
    bool prior_nan_ = false;      // a seed has a NaN coordinate: the slab kernels' NaN rules apply
    float prior_max_abs_ = 0.f;   // largest |finite coordinate| of a seed
    uint64_t nseeds_ = 0;                // S (all levels)
    Point* d_inj_ = nullptr;             // level >= 1 seeds, grouped by slab
    uint32_t* d_inj_keys_ = nullptr;
    unsigned long long* d_inj_rec_ = nullptr;   // per grid seed of levels >= 1: its slot-table record (k_seed_rec)
    struct PriorDev {                    // one prior level on the device
        PriorCell* cells = nullptr;
        uint32_t* cell_slab0 = nullptr;
        int32_t* slab_layer = nullptr;
        PriorSlabRec* slabs = nullptr;
        uint32_t ncells = 0, nslabs = 0;
    };
    std::vector<PriorDev> pdev_;
    Point* d_comb_ = nullptr;
    uint64_t comb_cap_ = 0;
    uint32_t* d_ckeys_ = nullptr;        // merge of keyed input: seed keys 0..S-1, then S + key
    uint64_t ckeys_cap_ = 0;
    const uint32_t* src_keys_ = nullptr; // keys of src_ (nullptr: key = index)
    bool comb_ok_ = false;
    std::vector<uint64_t> forced_lo_;
    uint64_t keys_cap_ = 0;
    bool keyed_ = false;
    uint64_t declared_total_ = 0;        // keyed input: global points of the declared files
    bool event_table_ = false;            // set_event_table: file_* hold the rank-local batch table
    Dev* dev_ = nullptr;
    std::vector<Level*> levels_;
    float bmin_[3] = {0, 0, 0}, bmax_[3] = {0, 0, 0};
    // Inputs with non-finite coordinates (enter_nonfinite): the level-0 grid
    // spans the points without an infinite coordinate, NaN taken as 0 (gmin_ /
    // gmax_); when some coordinate is infinite those points are split off with
    // their keys (d_nf_*) from the infinite ones (d_inf_*, built apart).
    bool nf_mode_ = false;
    float gmin_[3] = {0, 0, 0}, gmax_[3] = {0, 0, 0};
    Point* d_nf_pts_ = nullptr;
    uint32_t* d_nf_keys_ = nullptr;
    uint64_t nf_cap_ = 0;
    Point* d_inf_pts_ = nullptr;
    uint32_t* d_inf_keys_ = nullptr;
    uint64_t inf_cap_ = 0, ninf_ = 0;
    std::vector<CellFile> side_;         // their cells (host copy)
    uint32_t hierarchies_ = 0;
    BuildStats stats_;
    bool profiling_ = false;
    StageProfile prof_;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_used_;
    std::vector<hipEvent_t> ev_pool_;
    std::string err_;
    bool built_ = false;
};

// ---- sharded build helpers; synchronous, on an internal stream
// of `device`.  Cell id = ((ix-lo.x)*dims.y + (iy-lo.y))*dims.z + (iz-lo.z).
struct ShardGrid {
    int32_t lo[3];
    uint32_t dims[3];
    float cs;          // level-0 cell size
};
int shard_synth(Point* dst, uint64_t idx0, uint64_t n, uint64_t seed, int kind, float lo, float ext, int device);
int shard_bbox(const Point* d, uint64_t n, float bmin[3], float bmax[3], int device);
int shard_bbox_nonfinite(const Point* d, uint64_t n, float parts[15], int device);
int shard_batch_starts(const uint64_t* dbm, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                       const uint64_t* gstarts, uint64_t nb, uint64_t* local, int device);
// dim > 0: slab mode, unit = cell * 256 + level-0 hex z-layer of a dim sub-grid
int shard_histogram(const Point* d, uint64_t n, const ShardGrid& g, uint32_t* dhist, int device, uint32_t dim = 0);
// one pass: local bbox + histogram over a guessed grid (points outside it counted)
int shard_bbox_histogram(const Point* d, uint64_t n, const ShardGrid& g, uint32_t dim, uint32_t* dhist, float bmin[3],
                         float bmax[3], uint64_t* outside, int device);
int shard_bbox_sample(const Point* d, uint64_t n, float bmin[3], float bmax[3], int device);
// dkeys (global key per routed point) or dbm (nranks x ceil(n/64) membership words), either may be null
int shard_route(const Point* d, uint64_t n, uint32_t key0, const ShardGrid& g, const uint32_t* downer, uint32_t nranks,
                Point* dsend, uint32_t* dkeys, uint64_t* counts, int device, uint32_t dim = 0, uint64_t* dbm = nullptr);
int shard_route_hist(const Point* d, uint64_t n, const ShardGrid& g, const uint32_t* downer, uint32_t nranks,
                     const uint32_t* dhist, Point* dsend, uint64_t* dbm, uint64_t* counts, int device, uint32_t dim);
int shard_keys_from_bitmaps(const uint64_t* dbm, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                            uint32_t* dkeys, uint64_t nkeys, int device);
// pcc_shard_resolve_buckets (pcconv.h)
int shard_resolve_buckets(const uint64_t* seg_n, const uint32_t* seg_bucket, uint64_t nseg, uint32_t nbuckets,
                          const Point* dpts, const uint32_t* dkeys, const uint64_t* file_points, uint64_t nfiles,
                          uint32_t batch, uint32_t limit, uint32_t* state, uint32_t* spill_batch, uint64_t* kept_n,
                          Point* dkept, Point* dsub, uint32_t* dsub_keys, uint64_t* nkept, uint64_t* nsub, int device);

// Frees the device buffers closed converters left in the process-wide cache
// (engine.hip dev_alloc); returns the bytes freed.  Buffers in use stay.
size_t release_device_cache();

}  // namespace pcc
