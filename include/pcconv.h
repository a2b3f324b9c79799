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
 * Creates out_dir.  An existing metadata.json supplies the config; merging into
 * an existing non-empty cloud is not supported yet (-ENOTSUP). */
int pcc_open(const char* out_dir, const pcc_options* opt, pcc_converter** out);

/* converter.rs:106-112 add_points_batch over ceil(n/batch) consecutive slices
 * (lib.rs:31-52).  Host memory; copied to the device; caller keeps ownership. */
int pcc_add_points(pcc_converter* c, const pcc_point* pts, uint64_t n);

/* Same as pcc_add_points for points already resident in device memory. */
int pcc_add_points_device(pcc_converter* c, const pcc_point* dev_pts, uint64_t n);

/* One input file whose reader yields k empty batches (the reference's ASCII PLY
 * branch drops every point, ply.rs:43-51, but still counts batches). */
int pcc_add_empty_batches(pcc_converter* c, uint32_t k);

/* Deterministic synthetic file generated in HBM (kind 0 uniform in
 * [lo, lo+extent)^3, kind 1 clustered); used by bench.py and tests. */
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

/* Free without writing anything. */
int pcc_close(pcc_converter* c);

int pcc_get_stats(const pcc_converter* c, pcc_stats* out);

/* Enable per-stage HIP-event timing of subsequent builds (bench.py). */
int pcc_set_profiling(pcc_converter* c, int on);
int pcc_get_profile(const pcc_converter* c, pcc_profile* out);

/* Device pointer of the converter's resident input (n points), for timing. */
const pcc_point* pcc_device_input(const pcc_converter* c);

/* lib.rs:11-60 convert_from_paths: every file in order (".ply" supported;
 * ".las"/".laz"/".json" inputs are reported as unsupported), one converter,
 * then finish.  Logs like the reference CLI. */
int pcc_convert_files(const char* out_dir, const char* const* paths, size_t npaths, const pcc_options* opt);

/* Thread-local message of the last failing call ("" if none). */
const char* pcc_last_error(void);

/* ABI version, bumped on any incompatible change. */
uint32_t pcc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PCCONV_H */
