/*
 * pcconv.h — C ABI of the MI355X-native point-converter build (libpcconv.so).
 *
 * Drop-in boundary for the reference crate `point-converter`
 * (Seiichi-Yahiro/point-cloud @ 2024-08-07).  The reference has no FFI; this
 * ABI exposes exactly the library surface its callers use, in plain C types,
 * so a Rust (or any) host can bind it with an `extern "C"` block
 * (INTEGRATION.md shows the binding).  Each entry point names the reference
 * interface it replaces (paths relative to the reference root).
 *
 * Conventions (mirroring the reference):
 *   - points are the 16-byte on-disk record of point-converter/src/point.rs:8-14;
 *   - one pcc_add_points* call == one input file: ceil(n / batch_size) batches
 *     of lib.rs:31-52 (a call boundary is a batch boundary);
 *   - results are identical to the sequential reference (cell membership, slot
 *     winners, overflow lists and their order, headers, metadata values);
 *   - every function returns 0 or a negative errno-style code; the message is
 *     available from pcc_last_error() (thread-local).  Where the reference
 *     panics (I/O errors, converter.rs:84,170-171,203) this ABI returns an error.
 *   - one converter per thread; the build itself runs on one GPU (HIP stream).
 */
#ifndef PCCONV_H
#define PCCONV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* point.rs:8-14 Point { pos: Vec3, color: [u8; 4] } == on-disk layout (point.rs:26-37) */
typedef struct pcc_point {
    float x, y, z;
    uint8_t rgba[4];
} pcc_point;

typedef struct pcc_options {
    uint32_t batch_size;                /* lib.rs:32 get_batch(10_000) */
    int32_t device;                     /* HIP device ordinal */
    /* MetadataConfig defaults (metadata.rs:80-88); ignored when out_dir already
       holds a metadata.json, whose config wins (lib.rs:86-101). */
    uint32_t cell_point_overflow_limit; /* 5000 */
    uint32_t sub_grid_dimension;        /* 96 */
    float max_cell_size;                /* 1000.0 */
    uint32_t reserved;
} pcc_options;

typedef struct pcc_stats {
    uint64_t number_of_points;          /* metadata.number_of_points */
    uint32_t hierarchies;               /* metadata.hierarchies */
    uint32_t levels;
    uint64_t cells;                     /* cell files */
    uint64_t slabs;                     /* (cell, hex z-layer) work units over all levels */
    uint64_t arrivals;                  /* W = sum over levels of points handed to cells */
    uint64_t grid_points, kept_points;  /* grid winners + points kept in Some(list) buckets == number_of_points */
    double build_ms;                    /* device build wall time (inputs resident in HBM) */
    float bbox_min[3], bbox_max[3];
    uint64_t level0_early_tiles;        /* level-0 tiles (3072 points) whose first pass ran before
                                           pcc_build (behind the upload pieces or pcc_input_landed) */
    uint32_t level0_fold;               /* level-0 binning: 0 the three/four-pass path; 3 / 6 the two-pass
                                           fold over cells named by their indices modulo 2 / modulo 4 */
    uint32_t sequential_replay;         /* 1: the whole build ran as the sequential replay on the GPU
                                           (sub_grid_dimension > 97, or hexagon indices saturated at deep
                                           levels, e.g. NaN-collapsed points far from the origin) */
} pcc_stats;

/* Per-stage device time of the last pcc_build (HIP events on the engine stream;
 * only filled when profiling is on). */
typedef struct pcc_profile {
    double level0_ms;                   /* bbox + level-0 slab binning (radix sort + gather) */
    double dense_ms, small_ms;          /* slab kernels (dense LDS table / hashed), all levels */
    double bucket_ms, next_ms;          /* bucket resolution, next-level table build */
    uint64_t dense_arrivals, small_arrivals;
    uint32_t dense_launches, small_launches;
} pcc_profile;

typedef struct pcc_converter pcc_converter;

/* Fill defaults: batch 10 000, device 0, MetadataConfig::default(). */
int pcc_options_default(pcc_options* opt);

/* lib.rs:86-101 load_metadata + converter.rs:79-94 Converter::new.
 * Creates out_dir.  An existing metadata.json supplies the config; when it
 * describes a non-empty cloud, every h_{h}/c_*.bin cell is loaded as the
 * starting state (converter.rs:187-207 load_or_create_cell) and the points added
 * afterwards are merged into it (incremental merge: the result equals converting
 * the old and the new files in one run).  With pcc_declare_files (sharded
 * input) the merge runs on this rank's keys: its seeds, then its new points. */
int pcc_open(const char* out_dir, const pcc_options* opt, pcc_converter** out);

/* pcc_open for one rank of a sharded merge (the load of
 * converter.rs:187-207 restricted to the rank's own cells): only the cells of
 * the n level-0 subtrees in l0_cells (x, y, z triples) are loaded, and only
 * those are rewritten by pcc_write_cells.  Level-0 subtrees are independent
 * (a level-h cell's ancestor is its index >> h), so the union over ranks of
 * the rewritten subtrees equals a single-GPU merge. */
int pcc_open_subtrees(const char* out_dir, const pcc_options* opt, const int32_t* l0_cells, uint64_t n,
                      pcc_converter** out);

/* converter.rs:106-112 add_points_batch over ceil(n/batch) consecutive slices
 * (lib.rs:31-52).  Host memory; copied to the device; caller keeps ownership. */
int pcc_add_points(pcc_converter* c, const pcc_point* pts, uint64_t n);

/* One file delivered in pieces (the CLI's readers use it; a host reading a
 * file in chunks would too): pcc_begin_file, then pcc_append_points for each
 * piece in file order, then pcc_end_file(keep) -- the file is the first `keep`
 * points appended (a reader error keeps the complete batches, lib.rs:31-52).
 * The pieces are staged through pinned host buffers and copied to the device
 * on a copy stream while the caller reads the next piece.  pcc_cancel_file:
 * the open file contributes nothing (not even a batch). */
int pcc_begin_file(pcc_converter* c, uint64_t expected_points);
int pcc_append_points(pcc_converter* c, const pcc_point* pts, uint64_t n);
int pcc_end_file(pcc_converter* c, uint64_t keep_points);
int pcc_cancel_file(pcc_converter* c);

/* Same as pcc_add_points for points already resident in device memory. */
int pcc_add_points_device(pcc_converter* c, const pcc_point* dev_pts, uint64_t n);

/* One input file whose reader yields k empty batches (the reference's ASCII PLY
 * branch drops every point, ply.rs:43-51, but still counts batches). */
int pcc_add_empty_batches(pcc_converter* c, uint32_t k);

/* Deterministic synthetic file generated in HBM (kind 0 uniform
 * in [lo, lo+extent)^3, kind 1 clustered blobs, kind 2 the config-3 Gaussian
 * mixture: 32 clusters, sigma 10*2^U[0,3), Box-Muller); used by bench.py and tests. */
int pcc_add_synthetic(pcc_converter* c, uint64_t seed, int kind, uint64_t n, float lo, float extent);

/* Runs the hierarchy/LOD build on the GPU (converter.rs:114-139 for every
 * batch at once).  Timed region of bench.py.  Calling it again re-runs the
 * whole build from the resident input (benchmark steps). */
int pcc_build(pcc_converter* c);

/* converter.rs:218-238 save_cache + save_metadata: writes h_{h}/c_{x}_{y}_{z}.bin, then
 * metadata.json.  Builds first if needed. */
int pcc_write(pcc_converter* c);

/* converter.rs:241-246 Drop: build (if needed), write everything, free. */
int pcc_finish(pcc_converter* c);

/* Incremental merge without files: the built cloud of `src` (built now if
 * needed) becomes the starting state of the freshly opened `dst`, exactly as if
 * src had been written to dst's directory and dst opened on it (bench.py
 * config 5).  Same config required. */
int pcc_adopt_prior(pcc_converter* dst, pcc_converter* src);

/* Free without writing anything.  Large device buffers go to a process-wide
 * cache and are reused by the next converter on the same device. */
int pcc_close(pcc_converter* c);

/* Frees the cached device buffers of closed converters (e.g. before the GUI
 * hands the GPU to the renderer); returns the bytes freed.  No reference
 * counterpart: the reference's Converter drop frees host memory only. */
uint64_t pcc_release_device_cache(void);

/* One cell of the built cloud as the reference holds it in memory (cell.rs:33-38
 * Cell, Header cell.rs:238-261): the header values exactly as Cell::write_to
 * stores them (cell.rs:155-181, 280-298), the grid points (points_grid; their
 * order is unspecified, like the FxHashMap iteration of cell.rs:158-160) and the
 * overflow entries (child index at h+1; count 0 == None, i.e. forwarded;
 * otherwise the Some list in stored order), entries ordered by child octant. */
typedef struct pcc_cell_view {
    uint32_t hierarchy;                 /* CellId cell.rs:14-18 */
    int32_t x, y, z;
    uint32_t total_number_of_points, number_of_points, number_of_overflow_points;
    float size, sub_cell_size, pos[3];
    const pcc_point* grid;              /* number_of_points records */
    uint32_t entries;                   /* overflow entries, <= 8 (cell.rs:162) */
    int32_t child[8][3];
    uint32_t count[8];
    const pcc_point* list[8];
} pcc_cell_view;

/* Called once per cell; the view's pointers are valid during the call only.  A
 * nonzero return stops the walk and becomes pcc_visit_cells' return value. */
typedef int (*pcc_cell_visitor)(const pcc_cell_view* cell, void* user);

/* Every cell of the built cloud, level by level (builds first if needed): the
 * in-memory counterpart of pcc_write (the GUI keeps cells in memory,
 * src/plugins/converter.rs:553-592).  Sharded converters visit their own cells. */
int pcc_visit_cells(pcc_converter* c, pcc_cell_visitor fn, void* user);

int pcc_get_stats(const pcc_converter* c, pcc_stats* out);

/* Enable per-stage HIP-event timing of subsequent builds (bench.py). */
int pcc_set_profiling(pcc_converter* c, int on);
int pcc_get_profile(const pcc_converter* c, pcc_profile* out);

/* Device pointer of the converter's resident input (n points), for timing. */
const pcc_point* pcc_device_input(const pcc_converter* c);

/* lib.rs:11-60 convert_from_paths: every file in order, one converter, then
 * finish.  Logs like the reference CLI.  Inputs by extension (lib.rs:62-84):
 * ".ply" (binary LE/BE; ASCII as empty batches, ply.rs:43-51), ".las"
 * (uncompressed LAS 1.0-1.4; LAZ point data is reported and skipped), ".json"
 * (another converted cloud's metadata.json, own.rs, in a fixed enumeration). */
int pcc_convert_files(const char* out_dir, const char* const* paths, size_t npaths, const pcc_options* opt);

/* ---- Sharded multi-GPU build -------------------------------
 * The reference converter is single-threaded (converter.rs:72-139) and has no
 * multi-device notion; these entry points split ONE conversion across ranks by
 * level-0 cell.  Every level-h cell has a unique level-0 ancestor
 * (converter.rs:32-47 group_points at h+1 of a point of cell c lands in a child
 * of c), so level-0 subtrees are independent and each rank builds the cells it
 * owns, in global key order, with the global batch structure.  The collectives
 * (bbox/histogram all-reduce, all-to-all-v of points) belong to the caller
 * (pcconv/dist.py over RCCL).  All calls are synchronous. */
typedef struct pcc_shard_grid {
    int32_t lo[3];        /* level-0 cell index of the global bbox minimum (metadata.rs:100-102) */
    uint32_t dims[3];     /* cells per axis spanned by the global bbox */
    float cell_size;      /* metadata.rs:91-93 cell_size(0) */
} pcc_shard_grid;

/* Level-0 grid spanned by the global bounding box (host only, no device). */
int pcc_shard_grid_from_bbox(const float gmin[3], const float gmax[3], float max_cell_size, pcc_shard_grid* out);

/* Largest-first greedy placement (host only, no device): item i of weight w[i]
 * goes, heaviest first (ties by index), to the least loaded rank (ties by
 * rank); owner[i] and the final load per rank.  The ownership plan's inner loop
 * (pcconv/dist.py _lpt / assign_owners), identical on every rank. */
int pcc_shard_lpt(const double* w, uint64_t n, uint32_t world, uint32_t* owner, double* load);
/* The plan's shared-cell search (host only; pcconv/dist.py plan_split): the
 * ncand non-empty level-0 cells, heaviest first, with their whole-cell weights
 * whole_w[i]; the first kmax of them (the only ones that can be shared) with
 * their slabs' weights slab_w[slab_off[i] .. slab_off[i+1]) and their level-1
 * children's weights child_w[child_off[i] .. child_off[i+1]) (kmax + 1 offsets
 * each).
 * For k = 0 .. kmax the first k cells are shared: phase 1 = LPT of the whole
 * cells k.. followed by the first k cells' slabs, phase 2 = LPT of their
 * children; the estimate is max phase-1 load + max phase-2 load.  A larger k
 * replaces the best one only when it is more than 2 % lower.  Optional outputs
 * (NULL: not wanted) for the best k: whole_owner[i] for cells i >= k (ncand
 * entries), slab_owner[q] for the slabs of cells < k and child_owner[q] for
 * their children (slab_off[kmax] / child_off[kmax] entries), and the phase-1 /
 * phase-2 load per rank (world entries each) -- the LPT of the two lists. */
int pcc_shard_plan_search(const double* whole_w, const uint64_t* slab_off, const double* slab_w,
                          const uint64_t* child_off, const double* child_w, uint32_t ncand, uint32_t kmax,
                          uint32_t world, uint32_t* best_k, double* best_t, uint32_t* whole_owner,
                          uint32_t* slab_owner, uint32_t* child_owner, double* load1, double* load2);

/* Points first .. first+n-1 of the synthetic stream of pcc_add_synthetic,
 * written to dst[0 .. n) in device memory (each rank generates its key range). */
int pcc_synth_device(pcc_point* dst, uint64_t first, uint64_t n, uint64_t seed, int kind, float lo, float extent,
                     int device);

/* Local bounding box of n device points (bounding-volume/src/lib.rs:23-52).
 * -EDOM when a coordinate is NaN or infinite: use pcc_shard_bbox_nonfinite. */
int pcc_shard_bbox(const pcc_point* dev_pts, uint64_t n, float bmin[3], float bmax[3], int device);
/* The same for an input with NaN / infinite coordinates, as 15 values to
 * all-reduce: parts[0..2] / [3..5] min / max over the non-NaN values (f32::min /
 * max skip NaN and keep infinities, bounding-volume/src/lib.rs:23-31);
 * parts[6..8] 1 where the axis has a non-NaN value (else the reference's box
 * stays NaN there); parts[9..11] / [12..14] min / max over the points without an
 * infinite coordinate, NaN taken as 0: the extent of the level-0 cells those
 * points enter (metadata.rs:100-102, `as i32` maps NaN to 0), i.e. the grid the
 * ownership plan needs.  A point with an infinite coordinate enters no grid
 * cell: the histograms and routes below count and send it with unit 0, so one
 * rank builds every such point (their cells meet no finite point's). */
int pcc_shard_bbox_nonfinite(const pcc_point* dev_pts, uint64_t n, float parts[15], int device);

/* Points per level-0 cell of the grid (dev_hist: dims.x*dims.y*dims.z u32). */
int pcc_shard_histogram(const pcc_point* dev_pts, uint64_t n, const pcc_shard_grid* g, uint32_t* dev_hist, int device);

/* Stable partition of this rank's points by owner rank (owner = dev_owner[cell]):
 * dev_send holds rank 0's points, then rank 1's, ... each in input order, and
 * dev_keys the global key (key0 + local index) of each; counts[r] = points for
 * rank r (host array of nranks, nranks <= 64). */
int pcc_shard_route(const pcc_point* dev_pts, uint64_t n, uint32_t key0, const pcc_shard_grid* g,
                    const uint32_t* dev_owner, uint32_t nranks, pcc_point* dev_send, uint32_t* dev_keys,
                    uint64_t* counts, int device);

/* Slab sharding of heavy level-0 cells: the unit is the level-0 slab (cell,
 * hex z-layer) -- unit id = cell id * PCC_SHARD_LAYERS + the layer's offset in
 * its cell, t - (2 * sub_grid_dimension * iz - 2) with t = trunc(z / r0)
 * (hex.rs:83; r0 = level-0 sub_cell_size / 2).  A slab's slots are resolved
 * on one rank (cell.rs:70-94 is per slot).  dev_hist / dev_owner hold
 * ncells * PCC_SHARD_LAYERS entries. */
#define PCC_SHARD_LAYERS 256
int pcc_shard_slab_histogram(const pcc_point* dev_pts, uint64_t n, const pcc_shard_grid* g, uint32_t sub_grid_dimension,
                             uint32_t* dev_hist, int device);
int pcc_shard_route_slabs(const pcc_point* dev_pts, uint64_t n, uint32_t key0, const pcc_shard_grid* g,
                          uint32_t sub_grid_dimension, const uint32_t* dev_owner, uint32_t nranks, pcc_point* dev_send,
                          uint32_t* dev_keys, uint64_t* counts, int device);

/* The local bounding box and the histogram (sub_grid_dimension > 0: per slab,
 * as pcc_shard_slab_histogram; 0: per cell) in ONE pass over the points, the
 * histogram taken over a grid guessed before the global box is known (e.g. from
 * pcc_shard_bbox_sample all-reduced, one cell of margin); *outside = local
 * points outside that grid (any on any rank: histogram again on the true grid).
 * Replaces pcc_shard_bbox + pcc_shard_(slab_)histogram on the sharded step's
 * critical path (converter.rs:96-104 box, converter.rs:32-47 grouping). */
int pcc_shard_bbox_histogram(const pcc_point* dev_pts, uint64_t n, const pcc_shard_grid* guess,
                             uint32_t sub_grid_dimension, uint32_t* dev_hist, float bmin[3], float bmax[3],
                             uint64_t* outside, int device);
/* -EDOM (pcc_shard_bbox_histogram, pcc_shard_bbox_sample): NaN or infinite
 * coordinates; the caller takes pcc_shard_bbox_nonfinite and histograms the
 * true grid (an infinite point is outside every guessed grid). */
/* Bounding box of a sample of the points (512 tiles of 3 072): the guess. */
int pcc_shard_bbox_sample(const pcc_point* dev_pts, uint64_t n, float bmin[3], float bmax[3], int device);

/* Exchange-lean form of pcc_shard_route / pcc_shard_route_slabs
 * (sub_grid_dimension 0: cell units, else slab units): no key per routed point;
 * instead dev_bitmaps[r * ceil(n/64) + w] bit b is set iff local point 64 w + b
 * goes to rank r (u64 words, written in full by the call).  A receiver gets row
 * r of every sender (4 B per routed point become 1 bit per sender point) and
 * rebuilds the keys with pcc_shard_keys_from_bitmaps. */
int pcc_shard_route_bitmaps(const pcc_point* dev_pts, uint64_t n, const pcc_shard_grid* g,
                            uint32_t sub_grid_dimension, const uint32_t* dev_owner, uint32_t nranks,
                            pcc_point* dev_send, uint64_t* dev_bitmaps, uint64_t* counts, int device);
/* One-pass form of pcc_shard_route_bitmaps (same outputs): dev_hist = this
 * rank's points per unit (pcc_shard_histogram for cell units,
 * pcc_shard_slab_histogram for slab units, over the same dev_pts), which gives
 * every destination's total before the points are read; the points are then
 * read once (decoupled look-back between 4096-point tiles) instead of twice.
 * -EBADMSG if the histogram does not match the points. */
int pcc_shard_route_bitmaps_hist(const pcc_point* dev_pts, uint64_t n, const pcc_shard_grid* g,
                                 uint32_t sub_grid_dimension, const uint32_t* dev_owner, uint32_t nranks,
                                 const uint32_t* dev_hist, pcc_point* dev_send, uint64_t* dev_bitmaps,
                                 uint64_t* counts, int device);
/* Keys of the points received from nsrc senders (sender order, each ascending):
 * dev_bitmaps = the senders' rows for this rank concatenated (nwords[s] words
 * each), key0[s] = sender s's first global key.  nkeys must equal the number of
 * set bits (= received points), else -EBADMSG. */
int pcc_shard_keys_from_bitmaps(const uint64_t* dev_bitmaps, const uint64_t* nwords, const uint64_t* key0,
                                uint32_t nsrc, uint32_t* dev_keys, uint64_t nkeys, int device);
/* The rank-local start of every global batch: local[b] = the received points
 * (the senders' rows of dev_bitmaps as in pcc_shard_keys_from_bitmaps) whose
 * global key is below gstarts[b] (host arrays of nb, gstarts ascending; global
 * keys are 64-bit here, so clouds of 2^32 points and more shard). */
int pcc_shard_batch_starts(const uint64_t* dev_bitmaps, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                           const uint64_t* gstarts, uint64_t nb, uint64_t* local, int device);

/* Writes one cell file h_{hierarchy}/c_x_y_z.bin under out_dir from a view
 * (Cell::write_to cell.rs:155-181): a cell assembled by the caller from the
 * pieces several ranks built. */
int pcc_write_cell_view(const char* out_dir, const pcc_cell_view* v);

/* Global file structure (points per input file, CLI order; lib.rs:31-52
 * batching) without points.  Switches the converter to keyed input. */
int pcc_declare_files(pcc_converter* c, const uint64_t* file_points, uint64_t nfiles);
/* Rank-local keys (a sharded rank's input of any global size, 2^32 points and
 * beyond): instead of global keys and the declared files, the event batch
 * (lib.rs:31-52: the get_batch counter, across files) of each input point i is
 * batches[k] for the last k with starts[k] <= i.  starts[0] = 0, starts and
 * batches strictly ascending (one entry per global batch holding some of this
 * rank's points); total_batches = the global batch count (empty ones included).
 * The input then comes from pcc_set_keyed_points_device with dev_keys = NULL
 * (the rank's points in global key order; keys are their indices).  The table
 * from the exchange bitmaps: pcc_shard_batch_starts. */
int pcc_set_event_table(pcc_converter* c, const uint64_t* starts, const uint32_t* batches, uint64_t n,
                        uint64_t total_batches);

/* This rank's points (device memory) with their global keys, ascending. */
int pcc_add_keyed_points_device(pcc_converter* c, const pcc_point* dev_pts, const uint32_t* dev_keys, uint64_t n);

/* Zero-copy form of the above: the build reads all of this rank's points and
 * keys straight from these device buffers (typically the exchange's receive
 * buffers), which must stay valid and unchanged until pcc_build returns.  Only
 * after pcc_declare_files and before any other input; no input may follow.
 * dev_keys may be NULL: the keys are then 0 .. n-1 (one rank holds the whole
 * input in key order, so routing is the identity). */
int pcc_set_keyed_points_device(pcc_converter* c, const pcc_point* dev_pts, const uint32_t* dev_keys, uint64_t n);

/* Points [first, last) of the borrowed input (pcc_set_keyed_points_device with
 * dev_keys = NULL after pcc_set_event_table; no merge) are in place, or will be
 * once the work queued so far on after_stream (a hipStream_t, NULL: none)
 * completes.  Level-0 pass 1 of the build then runs on every group of tiles
 * whose points have all landed, on the converter's stream, while the rest of
 * the input is still arriving (a sharded rank's exchange); the
 * build runs the groups left.  Ranges may come in any order and overlap.
 * Optional: without it the build is the same, all of pass 1 inside pcc_build.
 * The landed points must not change until pcc_build returns. */
int pcc_input_landed(pcc_converter* c, uint64_t first, uint64_t last, void* after_stream);

/* Level ranges: one heavy level-0 cell built by several ranks (SURVEY §8e/§8f-4;
 * converter.rs:114-139 recursion split at a level boundary, which is exact
 * because a level-h cell's build depends only on the points forwarded to it).
 * root_level h0: the input is the exported arrivals of level-h0 cells (keys =
 * their global event keys), with the parent buckets' spill batches from
 * pcc_set_root_spill_batches; cells are written as h_{h0}, h_{h0+1}, ...
 * max_levels m > 0: build levels h0 .. h0+m-1 only and keep the next level's
 * arrivals on the device for pcc_export_pending.  raw_buckets != 0: the last
 * built level keeps no overflow lists and forwards every emission (its cells
 * are partial: the caller resolves their buckets, cell.rs:108-153, from all
 * ranks' emissions and assembles the cell files).  Not for merges. */
int pcc_set_level_range(pcc_converter* c, uint32_t root_level, uint32_t max_levels, int raw_buckets);
int pcc_set_root_spill_batches(pcc_converter* c, const int32_t* cells_xyz, const uint32_t* spill_batch, uint64_t ncells);
/* After pcc_build with max_levels: the cells of the first level not built. */
int pcc_pending_cells(pcc_converter* c, uint64_t* ncells, uint64_t* npoints);
/* Their arrivals, cell after cell (cell_points[i] each; a cell's slabs in layer
 * order, each slab in key order) into device buffers of npoints; the cells'
 * (x, y, z) and spill batches into host arrays of ncells. */
int pcc_export_pending(pcc_converter* c, int32_t* cells_xyz, uint32_t* spill_batch, uint64_t* cell_points,
                       pcc_point* dev_pts, uint32_t* dev_keys);
/* After pcc_build: the grid points (cell.rs:70-94 slot winners) of the cells of
 * the first built level -- a raw build's partial level-0 cells -- compacted into
 * device memory, cell after cell in the order pcc_visit_cells walks them, each
 * cell's points in that walk's order; the cells' (x, y, z) and point counts into
 * host arrays of ncells.  pcc_grid_cells gives ncells and the total npoints. */
int pcc_grid_cells(pcc_converter* c, uint64_t* ncells, uint64_t* npoints);
int pcc_export_grid(pcc_converter* c, int32_t* cells_xyz, uint64_t* cell_points, pcc_point* dev_pts);

/* Owner side of shared level-0 cells' overflow buckets: cell.rs:108-153
 * add_points_in_overflow resolved over the emissions every rank's raw lead build
 * forwarded (the numpy statement: pcconv/dist.py resolve_bucket).  The emissions
 * are nseg segments of dev_pts/dev_keys rows (seg_n[s] rows each, contiguous in
 * order), segment s belonging to bucket seg_bucket[s] < nbuckets; a segment is
 * in key order and a bucket's keys are distinct.  file_points / batch_size: the
 * global file structure (lib.rs:31-52 batching); limit: the overflow limit.
 * Per bucket (host arrays of nbuckets): state 1 = Some (the list is kept) or
 * 2 = None (spilled at spill_batch), kept_n = its kept points (0 for None).
 * dev_kept: the Some buckets' lists, bucket after bucket, each in key order
 * (*nkept rows); dev_sub_pts/keys: the None buckets' emissions, bucket after
 * bucket, segments in order (*nsub rows).  Each output needs room for every row.
 * Host transfers are the tables and the states only. */
int pcc_shard_resolve_buckets(const uint64_t* seg_n, const uint32_t* seg_bucket, uint64_t nseg, uint32_t nbuckets,
                              const pcc_point* dev_pts, const uint32_t* dev_keys, const uint64_t* file_points,
                              uint64_t nfiles, uint32_t batch_size, uint32_t limit, uint32_t* state,
                              uint32_t* spill_batch, uint64_t* kept_n, pcc_point* dev_kept, pcc_point* dev_sub_pts,
                              uint32_t* dev_sub_keys, uint64_t* nkept, uint64_t* nsub, int device);

/* Global metadata values after the ranks' all-reduce (converter.rs:96-112,141-158). */
int pcc_set_summary(pcc_converter* c, uint64_t number_of_points, const float bmin[3], const float bmax[3],
                    uint32_t hierarchies);

/* converter.rs:218-225 save_cache only (this rank's cells) / save_metadata only. */
int pcc_write_cells(pcc_converter* c);
int pcc_write_metadata(pcc_converter* c);

/* Drop all added input (and build results) but keep device allocations. */
int pcc_clear_input(pcc_converter* c);

/* Thread-local message of the last failing call ("" if none). */
const char* pcc_last_error(void);

/* ABI version, bumped on any incompatible change. */
uint32_t pcc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PCCONV_H */
