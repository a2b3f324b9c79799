// capi.cpp — extern "C" boundary (include/pcconv.h) over pcc::Engine.
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fstream>
#include <memory>
#include <sstream>
#include <thread>
#include <string>
#include <array>

#include "../../include/pcconv.h"
#include "engine.h"
#include "format.h"
#include "hip_check.h"
#include "pcc_math.h"

using namespace pcc;

static_assert(sizeof(pcc_point) == sizeof(Point), "pcc_point layout");

namespace {
thread_local std::string g_err;

int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// env_logger default format: [<rfc3339 utc> <LEVEL> <target>] msg  (main.rs:29)
void log_line(const char* level, const char* fmt, ...) {
    char ts[32];
    std::time_t t = std::time(nullptr);
    std::strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%SZ", std::gmtime(&t));
    char msg[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    fprintf(stderr, "[%s %-5s point_converter] %s\n", ts, level, msg);
}

bool mkdirs(const std::string& d) {
    if (d.empty()) return true;
    struct stat st;
    if (stat(d.c_str(), &st) == 0) return S_ISDIR(st.st_mode);
    size_t p = d.find_last_of('/');
    if (p != std::string::npos && p > 0 && !mkdirs(d.substr(0, p))) return false;
    return mkdir(d.c_str(), 0755) == 0 || errno == EEXIST;
}
}  // namespace

struct pcc_converter {
    std::string out_dir;
    pcc_options opt;
    Metadata meta;
    std::unique_ptr<Engine> eng;
    bool built = false;
    bool keyed = false;         // pcc_declare_files: sharded input
    bool streaming = false;     // a file opened by pcc_begin_file
    bool summary_set = false;   // pcc_set_summary: global metadata values
    double build_ms = 0;
    bool merge = false;         // out_dir held a non-empty cloud: incremental merge
    Metadata prior;             // its metadata.json
    // merge: the existing cloud's cells.  Only cells touched by new points are
    // rebuilt; the others stay as they are (converter.rs:160-207 loads a cell
    // only when a batch reaches it), so they are output from here.
    std::vector<CellFile> prior_cells;
    bool prior_on_disk = false;         // they are the files in out_dir (nothing to rewrite)
    std::vector<uint8_t> prior_touched; // per prior cell, after a build
    uint64_t untouched_grid = 0, untouched_kept = 0, untouched_cells = 0;
    // the merge state's host arrays (tens of GB at config 5), kept until the
    // converter closes: unmapping them takes about a second and blocks the
    // process's other memory mappings meanwhile
    std::unique_ptr<PriorState> prior_host;
};

namespace {
// pcc_cell_view of an existing cloud's cell as read from disk (header values
// recomputed exactly as Cell::new / Header::new do, cell.rs:43-49, 264-274)
void file_cell_view(const Config& cfg, const CellFile& f, pcc_cell_view& v) {
    v.hierarchy = f.h;
    v.x = f.idx[0]; v.y = f.idx[1]; v.z = f.idx[2];
    v.total_number_of_points = f.total;
    v.number_of_points = f.number;
    v.number_of_overflow_points = f.overflow;
    v.size = cell_size(cfg.max_cell_size, f.h);
    v.sub_cell_size = sub_cell_size(v.size, cfg.sub_grid_dimension);
    v.pos[0] = cell_pos1(f.idx[0], v.size); v.pos[1] = cell_pos1(f.idx[1], v.size); v.pos[2] = cell_pos1(f.idx[2], v.size);
    v.grid = reinterpret_cast<const pcc_point*>(f.grid.data());
    v.entries = (uint32_t)f.entries.size();
    for (uint32_t e = 0; e < v.entries; e++) {
        for (int a = 0; a < 3; a++) v.child[e][a] = f.entries[e].child[a];
        v.count[e] = f.entries[e].some ? (uint32_t)f.entries[e].pts.size() : 0u;
        v.list[e] = f.entries[e].some ? reinterpret_cast<const pcc_point*>(f.entries[e].pts.data()) : nullptr;
    }
}
// the merge's untouched existing cells after a build (touched = rebuilt)
void mark_touched(pcc_converter* c) {
    c->prior_touched.assign(c->prior_cells.size(), 0);
    c->untouched_grid = c->untouched_kept = c->untouched_cells = 0;
    std::vector<int32_t> hxyz;
    c->eng->built_cells(hxyz);
    std::vector<std::array<int32_t, 4>> built;
    for (size_t i = 0; i + 3 < hxyz.size(); i += 4) built.push_back({hxyz[i], hxyz[i + 1], hxyz[i + 2], hxyz[i + 3]});
    std::sort(built.begin(), built.end());
    for (size_t i = 0; i < c->prior_cells.size(); i++) {
        const CellFile& f = c->prior_cells[i];
        const std::array<int32_t, 4> k{(int32_t)f.h, f.idx[0], f.idx[1], f.idx[2]};
        c->prior_touched[i] = std::binary_search(built.begin(), built.end(), k) ? 1 : 0;
        if (!c->prior_touched[i]) {
            c->untouched_cells++;
            c->untouched_grid += f.number;
            c->untouched_kept += f.overflow;
        }
    }
}
}  // namespace

#define GUARD_BEGIN try {
#define GUARD_END                                            \
    }                                                        \
    catch (const std::exception& e) {                        \
        return set_err(-EIO, std::string("HIP/host error: ") + e.what()); \
    }

extern "C" {

uint32_t pcc_abi_version(void) { return 1; }

const char* pcc_last_error(void) { return g_err.c_str(); }

int pcc_options_default(pcc_options* o) {
    if (!o) return set_err(-EINVAL, "null options");
    o->batch_size = 10000;
    o->device = 0;
    o->cell_point_overflow_limit = 5000;
    o->sub_grid_dimension = 96;
    o->max_cell_size = 1000.0f;
    o->reserved = 0;
    return 0;
}

static bool any_cell_file(const std::string& dir) {
    for (uint32_t h = 0; h < 31; h++) {
        DIR* d = opendir((dir + "/h_" + std::to_string(h)).c_str());
        if (!d) continue;
        bool found = false;
        while (dirent* e = readdir(d)) {
            int x, y, z;
            char tail[8] = {0};
            if (sscanf(e->d_name, "c_%d_%d_%d.%3s", &x, &y, &z, tail) == 4 && strcmp(tail, "bin") == 0) { found = true; break; }
        }
        closedir(d);
        if (found) return true;
    }
    return false;
}

static int open_impl(const char* out_dir, const pcc_options* opt, const std::vector<int32_t>* subtrees,
                     pcc_converter** out) {
    if (!out_dir || !out) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    auto c = std::make_unique<pcc_converter>();
    c->out_dir = out_dir;
    if (opt) c->opt = *opt; else pcc_options_default(&c->opt);
    if (c->opt.batch_size == 0) return set_err(-EINVAL, "batch_size must be >= 1");
    c->meta.config.cell_point_overflow_limit = c->opt.cell_point_overflow_limit;
    c->meta.config.sub_grid_dimension = c->opt.sub_grid_dimension;
    c->meta.config.max_cell_size = c->opt.max_cell_size;
    // lib.rs:86-101 load_metadata
    const std::string mp = c->out_dir + "/metadata.json";
    std::ifstream f(mp);
    if (f) {
        std::stringstream ss;
        ss << f.rdbuf();
        std::string err;
        Metadata m;
        if (!parse_metadata_json(ss.str(), m, err)) return set_err(-EINVAL, err);
        c->meta.config = m.config;
        c->prior = m;
        c->merge = m.number_of_points > 0;
    }
    // converter.rs:187-207 opens a cell's existing file whenever the cell is
    // first touched, whatever metadata.json says: cell files left without
    // metadata.json (a run that never reached Drop) are merged as well, with
    // the counters starting from metadata.json or from zero
    if (!c->merge && any_cell_file(c->out_dir)) c->merge = true;
    // converter.rs:79-94 create_dir_all
    if (!mkdirs(c->out_dir)) return set_err(-EIO, "cannot create output directory " + c->out_dir);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_err(-ENODEV, "no HIP device available: the MI355X build needs a GPU (there is no CPU fallback)");
    if (c->opt.device < 0 || c->opt.device >= ndev) return set_err(-ENODEV, "invalid HIP device ordinal");
    c->eng = std::make_unique<Engine>(c->meta.config, c->opt.device);
    if (c->merge) {   // converter.rs:187-207: existing cells are the starting state
        std::string err;
        const auto t0 = std::chrono::steady_clock::now();
        int rc = read_cloud(c->out_dir, 31, c->prior_cells, err, subtrees);
        if (rc) return set_err(rc, err);
        const auto t1 = std::chrono::steady_clock::now();
        PriorState ps;
        rc = prior_from_cells(c->prior_cells, c->meta.config, ps, err);
        if (rc) return set_err(rc, err);
        const auto t2 = std::chrono::steady_clock::now();
        c->eng->set_prior(ps);
        c->prior_on_disk = true;
        c->prior_host = std::make_unique<PriorState>(std::move(ps));
        if (getenv("PCC_VERBOSE")) {
            const auto t3 = std::chrono::steady_clock::now();
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            fprintf(stderr, "[pcc] open: %zu cells read %.1f ms, merge state %.1f ms, upload %.1f ms\n",
                    c->prior_cells.size(), ms(t0, t1), ms(t1, t2), ms(t2, t3));
        }
    }
    *out = c.release();
    return 0;
    GUARD_END
}

int pcc_open(const char* out_dir, const pcc_options* opt, pcc_converter** out) {
    return open_impl(out_dir, opt, nullptr, out);
}

// Sharded merge: the existing cloud's state is read
// for the given level-0 subtrees only; cells of other subtrees are neither read
// nor rewritten by this converter.
int pcc_open_subtrees(const char* out_dir, const pcc_options* opt, const int32_t* l0_cells, uint64_t n,
                      pcc_converter** out) {
    if (!l0_cells && n) return set_err(-EINVAL, "null argument");
    const std::vector<int32_t> st(l0_cells, l0_cells + 3 * n);
    return open_impl(out_dir, opt, &st, out);
}

int pcc_add_points(pcc_converter* c, const pcc_point* pts, uint64_t n) {
    if (c && c->streaming) return set_err(-EINVAL, "a file opened by pcc_begin_file is still open");
    if (c && c->keyed) return set_err(-EINVAL, "converter takes keyed (sharded) input after pcc_declare_files");
    if (!c || (!pts && n)) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "points added after build");
    GUARD_BEGIN
    c->eng->add_file_host(reinterpret_cast<const Point*>(pts), n, c->opt.batch_size);
    return 0;
    GUARD_END
}

int pcc_add_points_device(pcc_converter* c, const pcc_point* pts, uint64_t n) {
    if (c && c->streaming) return set_err(-EINVAL, "a file opened by pcc_begin_file is still open");
    if (c && c->keyed) return set_err(-EINVAL, "converter takes keyed (sharded) input after pcc_declare_files");
    if (!c || (!pts && n)) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "points added after build");
    GUARD_BEGIN
    c->eng->add_file_device(reinterpret_cast<const Point*>(pts), n, c->opt.batch_size);
    return 0;
    GUARD_END
}

int pcc_begin_file(pcc_converter* c, uint64_t expected_points) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "points added after build");
    if (c->keyed) return set_err(-EINVAL, "keyed (sharded) input takes no files");
    if (c->streaming) return set_err(-EINVAL, "a file is already open");
    GUARD_BEGIN
    c->eng->stream_begin(expected_points);
    c->streaming = true;
    return 0;
    GUARD_END
}

int pcc_append_points(pcc_converter* c, const pcc_point* pts, uint64_t n) {
    if (!c || (!pts && n)) return set_err(-EINVAL, "null argument");
    if (!c->streaming) return set_err(-EINVAL, "pcc_begin_file must come first");
    GUARD_BEGIN
    c->eng->stream_push(reinterpret_cast<const Point*>(pts), n);
    return 0;
    GUARD_END
}

int pcc_end_file(pcc_converter* c, uint64_t keep_points) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (!c->streaming) return set_err(-EINVAL, "no file is open");
    GUARD_BEGIN
    c->eng->stream_end(keep_points, c->opt.batch_size);
    c->streaming = false;
    return 0;
    GUARD_END
}

int pcc_cancel_file(pcc_converter* c) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (!c->streaming) return set_err(-EINVAL, "no file is open");
    GUARD_BEGIN
    c->eng->stream_cancel();
    c->streaming = false;
    return 0;
    GUARD_END
}

int pcc_add_empty_batches(pcc_converter* c, uint32_t k) {
    if (c && c->streaming) return set_err(-EINVAL, "a file opened by pcc_begin_file is still open");
    if (!c) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "points added after build");
    c->eng->add_empty_batches(k);
    return 0;
}

int pcc_add_synthetic(pcc_converter* c, uint64_t seed, int kind, uint64_t n, float lo, float extent) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "points added after build");
    if (kind < 0 || kind > 2) return set_err(-EINVAL, "kind must be 0 (uniform), 1 (clustered blobs) or 2 (config-3 Gaussian mixture)");
    GUARD_BEGIN
    c->eng->add_file_synth(seed, kind, n, c->opt.batch_size, lo, extent);
    HIP_CHECK(hipStreamSynchronize(c->eng->stream()));
    return 0;
    GUARD_END
}

int pcc_build(pcc_converter* c) {
    if (c && c->streaming) return set_err(-EINVAL, "a file opened by pcc_begin_file is still open");
    if (!c) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = c->eng->build();
    HIP_CHECK(hipStreamSynchronize(c->eng->stream()));
    c->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc) return set_err(rc, c->eng->last_error());
    c->built = true;
    if (c->merge) mark_touched(c);
    if (c->summary_set) return 0;
    Metadata& m = c->meta;   // converter.rs:96-112 + 141-145
    m.number_of_points = c->eng->num_points();
    m.hierarchies = c->eng->hierarchies();
    if (m.number_of_points > 0)
        for (int a = 0; a < 3; a++) { m.bmin[a] = c->eng->bbox_min()[a]; m.bmax[a] = c->eng->bbox_max()[a]; }
    if (c->merge && c->prior.number_of_points == 0 && m.number_of_points > 0) {
        // stale cells, no counted cloud: the engine's box also spans the seeds,
        // the reference's (converter.rs:96-104) only the new points
        const int rc2 = shard_bbox(c->eng->input_points(), m.number_of_points, m.bmin, m.bmax, c->opt.device);
        if (rc2) return set_err(rc2, "bounding box of the new points failed");
    }
    if (c->merge) {   // lib.rs:86-101: counters continue from the loaded metadata; Aabb::extend_aabb
        const Metadata& p = c->prior;
        if (m.number_of_points == 0)
            for (int a = 0; a < 3; a++) { m.bmin[a] = p.bmin[a]; m.bmax[a] = p.bmax[a]; }
        else if (p.number_of_points > 0)   // converter.rs:96-104: the first batch assigns when the count is 0
            for (int a = 0; a < 3; a++) { m.bmin[a] = std::fmin(m.bmin[a], p.bmin[a]); m.bmax[a] = std::fmax(m.bmax[a], p.bmax[a]); }
        m.number_of_points += p.number_of_points;
        m.hierarchies = std::max(m.hierarchies, p.hierarchies);
    }
    return 0;
    GUARD_END
}

static int write_impl(pcc_converter* c, bool with_metadata) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (!c->built) {
        int rc = pcc_build(c);
        if (rc) return rc;
    }
    GUARD_BEGIN
    // Async output writer: level i's cell files are
    // written by a pool of host threads while level i+1 is compacted and copied
    // off the device.
    std::string err;
    int rc = make_output_dirs(c->out_dir, c->meta.hierarchies, err);
    if (rc) return set_err(rc, err);
    struct Slot { LevelHost H; HostPoints grid, kept; };
    Slot slot[2];
    int wrc = 0;
    std::string werr;
    const unsigned nt = writer_threads();
    std::thread writer;   // declared after everything it touches, joined before they go
    struct Join {         // a HIP error thrown below must not leave the writer joinable
        std::thread& t;
        ~Join() { if (t.joinable()) t.join(); }
    } join_writer{writer};
    const bool verbose = getenv("PCC_VERBOSE") != nullptr;
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    double wms[2] = {0, 0};
    for (uint32_t i = 0; i < c->eng->num_levels(); i++) {
        Slot& S = slot[i & 1];   // the writer of level i-1 holds the other slot
        const auto t0 = clk::now();
        rc = c->eng->download_level(i, S.H, S.grid, S.kept);
        if (rc) break;
        const auto t1 = clk::now();
        if (writer.joinable()) writer.join();
        if (wrc) break;
        if (verbose)
            fprintf(stderr, "[pcc] write: level %u download %.1f ms (%zu grid + %zu kept points), waited %.1f ms for level %u's files\n",
                    i, ms(t0, t1), S.grid.size(), S.kept.size(), ms(t1, clk::now()), i ? i - 1 : 0);
        writer = std::thread([&, sp = &S, slot_i = i & 1] {
            const auto w0 = clk::now();
            wrc = write_level_cells(c->out_dir, c->meta.config, sp->H, sp->grid.data(), sp->kept.data(), nt, werr);
            wms[slot_i] = ms(w0, clk::now());
        });
    }
    const auto tj = clk::now();
    if (writer.joinable()) writer.join();
    if (verbose) fprintf(stderr, "[pcc] write: last level's files %.1f ms after the last download\n", ms(tj, clk::now()));
    if (rc) return set_err(rc, c->eng->last_error());
    if (wrc) return set_err(wrc, werr);
    if (!c->eng->side_cells().empty()) {   // the cells of points with an infinite coordinate
        rc = write_cell_files(c->out_dir, c->meta.config, c->eng->side_cells(), nullptr, err);
        if (rc) return set_err(rc, err);
    }
    if (c->merge && !c->prior_on_disk) {   // adopted cloud: its untouched cells are not on disk here
        rc = write_cell_files(c->out_dir, c->meta.config, c->prior_cells, &c->prior_touched, err);
        if (rc) return set_err(rc, err);
    }
    if (with_metadata) {
        rc = write_metadata(c->out_dir, c->meta, err);
        if (rc) return set_err(rc, err);
    }
    return 0;
    GUARD_END
}

int pcc_visit_cells(pcc_converter* c, pcc_cell_visitor fn, void* user) {
    if (!c || !fn) return set_err(-EINVAL, "null argument");
    if (!c->built) {
        int rc = pcc_build(c);
        if (rc) return rc;
    }
    GUARD_BEGIN
    LevelHost H;
    HostPoints grid, kept;
    pcc_cell_view v;
    for (uint32_t i = 0; i < c->eng->num_levels(); i++) {
        const int rc = c->eng->download_level(i, H, grid, kept);
        if (rc) return set_err(rc, c->eng->last_error());
        const uint32_t ncells = (uint32_t)(H.cell_idx.size() / 3);
        for (uint32_t k = 0; k < ncells; k++) {
            level_cell_view(c->meta.config, H, k, grid.data(), kept.data(), v);
            const int r = fn(&v, user);
            if (r) return r;
        }
    }
    for (const CellFile& f : c->eng->side_cells()) {   // cells of points with an infinite coordinate
        file_cell_view(c->meta.config, f, v);
        const int r = fn(&v, user);
        if (r) return r;
    }
    for (size_t i = 0; i < c->prior_cells.size(); i++) {   // merge: the existing cells no new point reached
        if (i < c->prior_touched.size() && c->prior_touched[i]) continue;
        file_cell_view(c->meta.config, c->prior_cells[i], v);
        const int r = fn(&v, user);
        if (r) return r;
    }
    return 0;
    GUARD_END
}

int pcc_write(pcc_converter* c) { return write_impl(c, true); }
int pcc_write_cells(pcc_converter* c) { return write_impl(c, false); }

int pcc_write_metadata(pcc_converter* c) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (!c->built && !c->summary_set) return set_err(-EINVAL, "nothing built and no summary set");
    std::string err;
    if (!mkdirs(c->out_dir)) return set_err(-EIO, "cannot create output directory " + c->out_dir);
    for (uint32_t h = 0; h < c->meta.hierarchies; h++)   // converter.rs:141-158 (folders exist on every rank's disk view)
        if (!mkdirs(c->out_dir + "/h_" + std::to_string(h))) return set_err(-EIO, "cannot create hierarchy folder");
    const int rc = write_metadata(c->out_dir, c->meta, err);
    return rc ? set_err(rc, err) : 0;
}

int pcc_shard_grid_from_bbox(const float gmin[3], const float gmax[3], float max_cell_size, pcc_shard_grid* out) {
    if (!gmin || !gmax || !out) return set_err(-EINVAL, "null argument");
    const float cs = cell_size(max_cell_size, 0);
    uint64_t nc = 1;
    for (int a = 0; a < 3; a++) {
        if (!(gmin[a] <= gmax[a])) return set_err(-EINVAL, "empty or non-finite bounding box");
        out->lo[a] = cell_index1(gmin[a], cs);
        const int64_t d = (int64_t)cell_index1(gmax[a], cs) - out->lo[a] + 1;
        out->dims[a] = (uint32_t)d;
        nc *= (uint64_t)d;
    }
    out->cell_size = cs;
    if (nc > (1ull << 22)) return set_err(-EFBIG, "level-0 grid of the bounding box exceeds 2^22 cells");
    return 0;
}

// Least loaded rank, ties by rank, in log2(world) compares per placement: a
// tournament tree over the ranks (leaves padded to a power of two with +inf),
// each node holding the winner of its two children, the left one on ties.
struct LeastLoaded {
    uint32_t m = 1;
    std::vector<double> load;
    std::vector<uint32_t> node;   // node[1] = the overall winner
    explicit LeastLoaded(uint32_t world) {
        while (m < world) m <<= 1;
        load.assign(m, INFINITY);
        for (uint32_t r = 0; r < world; r++) load[r] = 0.0;
        node.assign(2 * m, 0);
        for (uint32_t r = 0; r < m; r++) node[m + r] = r;
        for (uint32_t v = m - 1; v >= 1; v--) node[v] = pick(node[2 * v], node[2 * v + 1]);
    }
    uint32_t pick(uint32_t a, uint32_t b) const { return load[b] < load[a] ? b : a; }
    // adds w to the least loaded rank and returns it
    uint32_t place(double w) {
        const uint32_t r = node[1];
        load[r] += w;
        for (uint32_t v = (m + r) >> 1; v >= 1; v >>= 1) node[v] = pick(node[2 * v], node[2 * v + 1]);
        return r;
    }
};

// largest first (ties by index) to the least loaded rank (ties by rank)
static void lpt(const double* w, uint64_t n, uint32_t world, uint32_t* owner, double* load) {
    std::vector<uint64_t> order(n);
    for (uint64_t i = 0; i < n; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return w[a] > w[b]; });
    LeastLoaded ll(world);
    for (uint64_t i : order) {
        const uint32_t best = ll.place(w[i]);
        if (owner) owner[i] = best;
    }
    for (uint32_t r = 0; r < world; r++) load[r] = ll.load[r];
}

int pcc_shard_lpt(const double* w, uint64_t n, uint32_t world, uint32_t* owner, double* load) {
    if ((n && (!w || !owner)) || !load || world == 0) return set_err(-EINVAL, "null argument or no ranks");
    GUARD_BEGIN
    lpt(w, n, world, owner, load);
    return 0;
    GUARD_END
}

int pcc_shard_plan_search(const double* whole_w, const uint64_t* slab_off, const double* slab_w,
                          const uint64_t* child_off, const double* child_w, uint32_t ncand, uint32_t kmax,
                          uint32_t world, uint32_t* best_k, double* best_t, uint32_t* whole_owner,
                          uint32_t* slab_owner, uint32_t* child_owner, double* load1, double* load2) {
    if (!best_k || !best_t || world == 0 || kmax > ncand || (ncand && (!whole_w || !slab_off || !child_off)))
        return set_err(-EINVAL, "null argument, no ranks or kmax > ncand");
    GUARD_BEGIN
    // Every k places a subset of one fixed item list in one fixed order: the
    // phase-1 list of k is [whole cells k..] + [slabs of cells ..k), so by
    // weight (descending), then whole cells before slabs, then position.  Sort
    // once, then each k is one filtered greedy pass.
    struct It { double w; uint32_t type, cell; uint64_t pos; };
    std::vector<It> p1, p2;
    // only the first kmax candidates can be shared: their slabs and children alone
    for (uint32_t i = 0; i < ncand; i++) {
        p1.push_back({whole_w[i], 0u, i, i});
        if (i >= kmax) continue;
        for (uint64_t q = slab_off[i]; q < slab_off[i + 1]; q++) p1.push_back({slab_w[q], 1u, i, q});
        for (uint64_t q = child_off[i]; q < child_off[i + 1]; q++) p2.push_back({child_w[q], 1u, i, q});
    }
    auto by = [](const It& a, const It& b) {
        if (a.w != b.w) return a.w > b.w;
        if (a.type != b.type) return a.type < b.type;
        return a.pos < b.pos;
    };
    std::sort(p1.begin(), p1.end(), by);
    std::sort(p2.begin(), p2.end(), by);
    auto in1 = [](const It& it, uint32_t k) { return (it.cell >= k) == (it.type == 0); };
    bool have = false;
    *best_k = 0;
    *best_t = 0.0;
    for (uint32_t k = 0; k <= kmax; k++) {
        LeastLoaded l1(world), l2(world);
        for (const It& it : p1)
            if (in1(it, k)) l1.place(it.w);
        bool any2 = false;
        for (const It& it : p2)
            if (it.cell < k) { l2.place(it.w); any2 = true; }
        const double t = *std::max_element(l1.load.begin(), l1.load.begin() + world) +
                         (any2 ? *std::max_element(l2.load.begin(), l2.load.begin() + world) : 0.0);
        if (!have || t < *best_t * 0.98) {
            have = true;
            *best_t = t;
            *best_k = k;
        }
    }
    // the best k's placement (= LPT of its two lists, the same order): owners
    // of the whole cells k.., of the slabs and children of the cells ..k
    if (whole_owner || slab_owner || child_owner || load1 || load2) {
        const uint32_t k = *best_k;
        LeastLoaded l1(world), l2(world);
        for (const It& it : p1) {
            if (!in1(it, k)) continue;
            const uint32_t r = l1.place(it.w);
            if (it.type == 0 && whole_owner) whole_owner[it.pos] = r;
            if (it.type == 1 && slab_owner) slab_owner[it.pos] = r;
        }
        for (const It& it : p2) {
            if (it.cell >= k) continue;
            const uint32_t r = l2.place(it.w);
            if (child_owner) child_owner[it.pos] = r;
        }
        for (uint32_t r = 0; r < world; r++) {
            if (load1) load1[r] = l1.load[r];
            if (load2) load2[r] = l2.load[r];
        }
    }
    return 0;
    GUARD_END
}

static ShardGrid to_grid(const pcc_shard_grid* g) {
    ShardGrid s;
    for (int a = 0; a < 3; a++) { s.lo[a] = g->lo[a]; s.dims[a] = g->dims[a]; }
    s.cs = g->cell_size;
    return s;
}

int pcc_synth_device(pcc_point* dst, uint64_t first, uint64_t n, uint64_t seed, int kind, float lo, float extent,
                     int device) {
    if (!dst && n) return set_err(-EINVAL, "null argument");
    if (kind < 0 || kind > 2) return set_err(-EINVAL, "kind must be 0 (uniform), 1 (clustered blobs) or 2 (config-3 Gaussian mixture)");
    GUARD_BEGIN
    return shard_synth(reinterpret_cast<Point*>(dst), first, n, seed, kind, lo, extent, device);
    GUARD_END
}

int pcc_shard_bbox(const pcc_point* d, uint64_t n, float bmin[3], float bmax[3], int device) {
    if ((!d && n) || !bmin || !bmax) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    const int rc = shard_bbox(reinterpret_cast<const Point*>(d), n, bmin, bmax, device);
    return rc ? set_err(rc, "input contains NaN or infinite coordinates (pcc_shard_bbox_nonfinite)") : 0;
    GUARD_END
}

int pcc_shard_batch_starts(const uint64_t* dbm, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                           const uint64_t* gstarts, uint64_t nb, uint64_t* local, int device) {
    if (!nwords || !key0 || ((!gstarts || !local) && nb)) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    const int rc = shard_batch_starts(dbm, nwords, key0, nsrc, gstarts, nb, local, device);
    return rc ? set_err(rc, "batch starts: 1..64 senders in key order, ascending batch starts") : 0;
    GUARD_END
}

int pcc_shard_bbox_nonfinite(const pcc_point* d, uint64_t n, float parts[15], int device) {
    if ((!d && n) || !parts) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    return shard_bbox_nonfinite(reinterpret_cast<const Point*>(d), n, parts, device);
    GUARD_END
}

int pcc_shard_histogram(const pcc_point* d, uint64_t n, const pcc_shard_grid* g, uint32_t* dhist, int device) {
    if ((!d && n) || !g || !dhist) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    const int rc = shard_histogram(reinterpret_cast<const Point*>(d), n, to_grid(g), dhist, device);
    return rc ? set_err(rc, "point outside the shard grid (grid not spanned by the global bbox?)") : 0;
    GUARD_END
}

int pcc_shard_route(const pcc_point* d, uint64_t n, uint32_t key0, const pcc_shard_grid* g, const uint32_t* downer,
                    uint32_t nranks, pcc_point* dsend, uint32_t* dkeys, uint64_t* counts, int device) {
    if ((!d || !dsend || !dkeys) && n) return set_err(-EINVAL, "null argument");
    if (!g || !downer || !counts) return set_err(-EINVAL, "null argument");
    if ((uint64_t)key0 + n > (1ull << 32)) return set_err(-EOVERFLOW, "global keys must fit in 32 bits");
    GUARD_BEGIN
    const int rc = shard_route(reinterpret_cast<const Point*>(d), n, key0, to_grid(g), downer, nranks,
                               reinterpret_cast<Point*>(dsend), dkeys, counts, device);
    return rc ? set_err(rc, "routing failed (nranks > 64, point outside grid, or owner >= nranks)") : 0;
    GUARD_END
}

int pcc_shard_slab_histogram(const pcc_point* d, uint64_t n, const pcc_shard_grid* g, uint32_t sub_grid_dimension,
                             uint32_t* dhist, int device) {
    if ((!d && n) || !g || !dhist) return set_err(-EINVAL, "null argument");
    if (sub_grid_dimension == 0 || 2 * sub_grid_dimension + 2 > PCC_SHARD_LAYERS)
        return set_err(-EINVAL, "sub_grid_dimension out of range for slab sharding");
    GUARD_BEGIN
    const int rc = shard_histogram(reinterpret_cast<const Point*>(d), n, to_grid(g), dhist, device, sub_grid_dimension);
    return rc ? set_err(rc, "point outside the shard grid (grid not spanned by the global bbox?)") : 0;
    GUARD_END
}

int pcc_shard_bbox_histogram(const pcc_point* d, uint64_t n, const pcc_shard_grid* g, uint32_t sub_grid_dimension,
                             uint32_t* dhist, float bmin[3], float bmax[3], uint64_t* outside, int device) {
    if ((!d && n) || !g || !dhist || !bmin || !bmax || !outside) return set_err(-EINVAL, "null argument");
    if (sub_grid_dimension && 2 * sub_grid_dimension + 2 > PCC_SHARD_LAYERS)
        return set_err(-EINVAL, "sub_grid_dimension out of range for slab sharding");
    GUARD_BEGIN
    const int rc = shard_bbox_histogram(reinterpret_cast<const Point*>(d), n, to_grid(g), sub_grid_dimension, dhist,
                                        bmin, bmax, outside, device);
    return rc ? set_err(rc, rc == -EDOM ? "input contains NaN or infinite coordinates (pcc_shard_bbox_nonfinite)"
                                        : "histogram grid too large") : 0;
    GUARD_END
}

int pcc_shard_bbox_sample(const pcc_point* d, uint64_t n, float bmin[3], float bmax[3], int device) {
    if ((!d && n) || !bmin || !bmax) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    const int rc = shard_bbox_sample(reinterpret_cast<const Point*>(d), n, bmin, bmax, device);
    return rc ? set_err(rc, "sample box not finite (NaN or infinite coordinates)") : 0;
    GUARD_END
}

int pcc_shard_route_slabs(const pcc_point* d, uint64_t n, uint32_t key0, const pcc_shard_grid* g,
                          uint32_t sub_grid_dimension, const uint32_t* downer, uint32_t nranks, pcc_point* dsend,
                          uint32_t* dkeys, uint64_t* counts, int device) {
    if ((!d || !dsend || !dkeys) && n) return set_err(-EINVAL, "null argument");
    if (!g || !downer || !counts) return set_err(-EINVAL, "null argument");
    if (sub_grid_dimension == 0 || 2 * sub_grid_dimension + 2 > PCC_SHARD_LAYERS)
        return set_err(-EINVAL, "sub_grid_dimension out of range for slab sharding");
    if ((uint64_t)key0 + n > (1ull << 32)) return set_err(-EOVERFLOW, "global keys must fit in 32 bits");
    GUARD_BEGIN
    const int rc = shard_route(reinterpret_cast<const Point*>(d), n, key0, to_grid(g), downer, nranks,
                               reinterpret_cast<Point*>(dsend), dkeys, counts, device, sub_grid_dimension);
    return rc ? set_err(rc, "routing failed (nranks > 64, point outside grid, or owner >= nranks)") : 0;
    GUARD_END
}

int pcc_shard_route_bitmaps(const pcc_point* d, uint64_t n, const pcc_shard_grid* g, uint32_t sub_grid_dimension,
                            const uint32_t* downer, uint32_t nranks, pcc_point* dsend, uint64_t* dbitmaps,
                            uint64_t* counts, int device) {
    if ((!d || !dsend || !dbitmaps) && n) return set_err(-EINVAL, "null argument");
    if (!g || !downer || !counts) return set_err(-EINVAL, "null argument");
    if (sub_grid_dimension != 0 && 2 * sub_grid_dimension + 2 > PCC_SHARD_LAYERS)
        return set_err(-EINVAL, "sub_grid_dimension out of range for slab sharding");
    GUARD_BEGIN
    const int rc = shard_route(reinterpret_cast<const Point*>(d), n, 0, to_grid(g), downer, nranks,
                               reinterpret_cast<Point*>(dsend), nullptr, counts, device, sub_grid_dimension, dbitmaps);
    return rc ? set_err(rc, "routing failed (nranks > 64, point outside grid, or owner >= nranks)") : 0;
    GUARD_END
}

int pcc_shard_route_bitmaps_hist(const pcc_point* d, uint64_t n, const pcc_shard_grid* g, uint32_t sub_grid_dimension,
                                 const uint32_t* downer, uint32_t nranks, const uint32_t* dhist, pcc_point* dsend,
                                 uint64_t* dbitmaps, uint64_t* counts, int device) {
    if ((!d || !dsend || !dbitmaps) && n) return set_err(-EINVAL, "null argument");
    if (!g || !downer || !dhist || !counts) return set_err(-EINVAL, "null argument");
    if (sub_grid_dimension != 0 && 2 * sub_grid_dimension + 2 > PCC_SHARD_LAYERS)
        return set_err(-EINVAL, "sub_grid_dimension out of range for slab sharding");
    GUARD_BEGIN
    const int rc = shard_route_hist(reinterpret_cast<const Point*>(d), n, to_grid(g), downer, nranks, dhist,
                                    reinterpret_cast<Point*>(dsend), dbitmaps, counts, device, sub_grid_dimension);
    if (rc == -EBADMSG) return set_err(rc, "the unit histogram does not match the points");
    return rc ? set_err(rc, "routing failed (nranks > 64, point outside grid, or owner >= nranks)") : 0;
    GUARD_END
}

int pcc_shard_keys_from_bitmaps(const uint64_t* dbitmaps, const uint64_t* nwords, const uint64_t* key0, uint32_t nsrc,
                                uint32_t* dkeys, uint64_t nkeys, int device) {
    if (!nwords || !key0 || (nkeys && (!dkeys || !dbitmaps))) return set_err(-EINVAL, "null argument");
    for (uint32_t s = 0; s < nsrc; s++)
        if (key0[s] + 64 * nwords[s] > (1ull << 32) + 63) return set_err(-EOVERFLOW, "global keys must fit in 32 bits");
    GUARD_BEGIN
    const int rc = shard_keys_from_bitmaps(dbitmaps, nwords, key0, nsrc, dkeys, nkeys, device);
    if (rc == -EBADMSG) return set_err(rc, "bitmaps do not match the number of received points");
    return rc ? set_err(rc, "key rebuild failed (nsrc outside 1..64 or too many words)") : 0;
    GUARD_END
}

int pcc_shard_resolve_buckets(const uint64_t* seg_n, const uint32_t* seg_bucket, uint64_t nseg, uint32_t nbuckets,
                              const pcc_point* dev_pts, const uint32_t* dev_keys, const uint64_t* file_points,
                              uint64_t nfiles, uint32_t batch_size, uint32_t limit, uint32_t* state,
                              uint32_t* spill_batch, uint64_t* kept_n, pcc_point* dev_kept, pcc_point* dev_sub_pts,
                              uint32_t* dev_sub_keys, uint64_t* nkept, uint64_t* nsub, int device) {
    if (!nkept || !nsub || (nseg && (!seg_n || !seg_bucket)) || (nbuckets && (!state || !spill_batch || !kept_n)) ||
        (nfiles && !file_points))
        return set_err(-EINVAL, "null argument");
    uint64_t rows = 0;
    for (uint64_t s = 0; s < nseg; s++) rows += seg_n[s];
    if (rows && (!dev_pts || !dev_keys || !dev_kept || !dev_sub_pts || !dev_sub_keys))
        return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    const int rc = shard_resolve_buckets(seg_n, seg_bucket, nseg, nbuckets, reinterpret_cast<const Point*>(dev_pts),
                                         dev_keys, file_points, nfiles, batch_size, limit, state, spill_batch, kept_n,
                                         reinterpret_cast<Point*>(dev_kept), reinterpret_cast<Point*>(dev_sub_pts),
                                         dev_sub_keys, nkept, nsub, device);
    return rc ? set_err(rc, "bucket resolution failed (no files, no segments, or a segment's bucket out of range)") : 0;
    GUARD_END
}

int pcc_write_cell_view(const char* out_dir, const pcc_cell_view* v) {
    if (!out_dir || !v) return set_err(-EINVAL, "null argument");
    if (v->entries > 8) return set_err(-EINVAL, "a cell has at most 8 overflow entries");
    GUARD_BEGIN
    std::string err;
    const int rc = write_view_file(out_dir, *v, err);
    return rc ? set_err(rc, err) : 0;
    GUARD_END
}

int pcc_declare_files(pcc_converter* c, const uint64_t* file_points, uint64_t nfiles) {
    if (!c || (!file_points && nfiles)) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "files declared after build");
    uint64_t tot = 0;
    for (uint64_t f = 0; f < nfiles; f++) tot += file_points[f];
    if (tot > (1ull << 32)) return set_err(-EOVERFLOW, "global keys must fit in 32 bits");
    GUARD_BEGIN
    c->eng->declare_files(file_points, nfiles, c->opt.batch_size);
    c->keyed = true;
    return 0;
    GUARD_END
}

int pcc_set_event_table(pcc_converter* c, const uint64_t* starts, const uint32_t* batches, uint64_t n,
                        uint64_t total_batches) {
    if (!c || ((!starts || !batches) && n)) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "event table after build");
    if (total_batches > 0xFFFFFFFFull) return set_err(-EOVERFLOW, "more than 2^32-1 batches");
    GUARD_BEGIN
    c->eng->set_event_table(starts, batches, n, total_batches);
    c->keyed = true;
    return 0;
    GUARD_END
}

int pcc_add_keyed_points_device(pcc_converter* c, const pcc_point* d, const uint32_t* keys, uint64_t n) {
    if (!c || ((!d || !keys) && n)) return set_err(-EINVAL, "null argument");
    if (!c->keyed) return set_err(-EINVAL, "pcc_declare_files must come first");
    if (c->built) return set_err(-EINVAL, "points added after build");
    GUARD_BEGIN
    c->eng->add_keyed_device(reinterpret_cast<const Point*>(d), keys, n);
    return 0;
    GUARD_END
}

int pcc_set_keyed_points_device(pcc_converter* c, const pcc_point* d, const uint32_t* keys, uint64_t n) {
    if (!c || (!d && n)) return set_err(-EINVAL, "null argument");
    if (!c->keyed) return set_err(-EINVAL, "pcc_declare_files must come first");
    if (c->built) return set_err(-EINVAL, "points added after build");
    GUARD_BEGIN
    c->eng->set_keyed_external(reinterpret_cast<const Point*>(d), keys, n);
    return 0;
    GUARD_END
}

int pcc_input_landed(pcc_converter* c, uint64_t first, uint64_t last, void* after_stream) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (c->built) return set_err(-EINVAL, "input landed after build");
    if (c->merge) return set_err(-EINVAL, "input_landed: not for a merge");
    GUARD_BEGIN
    const int rc = c->eng->input_landed(first, last, static_cast<hipStream_t>(after_stream));
    if (rc) return set_err(rc, c->eng->last_error());
    return 0;
    GUARD_END
}

int pcc_set_level_range(pcc_converter* c, uint32_t root_level, uint32_t max_levels, int raw_buckets) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (c->merge) return set_err(-EINVAL, "a merge cannot be split into level ranges");
    if (root_level >= 31) return set_err(-EINVAL, "root level must be < 31");
    c->eng->set_root_level(root_level);
    c->eng->set_max_levels(max_levels, raw_buckets != 0);
    return 0;
}

int pcc_set_root_spill_batches(pcc_converter* c, const int32_t* cells_xyz, const uint32_t* spill_batch, uint64_t n) {
    if (!c || ((!cells_xyz || !spill_batch) && n)) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    c->eng->set_root_spill_batches(cells_xyz, spill_batch, n);
    return 0;
    GUARD_END
}

int pcc_pending_cells(pcc_converter* c, uint64_t* ncells, uint64_t* npoints) {
    if (!c || !ncells || !npoints) return set_err(-EINVAL, "null argument");
    if (!c->built) return set_err(-EINVAL, "nothing built");
    return c->eng->pending_info(*ncells, *npoints);
}

int pcc_export_pending(pcc_converter* c, int32_t* cells_xyz, uint32_t* spill_batch, uint64_t* cell_points,
                       pcc_point* dev_pts, uint32_t* dev_keys) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (!c->built) return set_err(-EINVAL, "nothing built");
    uint64_t nc = 0, np = 0;
    c->eng->pending_info(nc, np);
    if (nc && (!cells_xyz || !spill_batch || !cell_points)) return set_err(-EINVAL, "null argument");
    if (np && (!dev_pts || !dev_keys)) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    return c->eng->export_pending(cells_xyz, spill_batch, cell_points, reinterpret_cast<Point*>(dev_pts), dev_keys);
    GUARD_END
}

int pcc_grid_cells(pcc_converter* c, uint64_t* ncells, uint64_t* npoints) {
    if (!c || !ncells || !npoints) return set_err(-EINVAL, "null argument");
    if (!c->built) return set_err(-EINVAL, "nothing built");
    *ncells = *npoints = 0;
    if (!c->eng->num_levels()) return 0;
    GUARD_BEGIN
    return c->eng->grid_cells(0, *ncells, *npoints);
    GUARD_END
}

int pcc_export_grid(pcc_converter* c, int32_t* cells_xyz, uint64_t* cell_points, pcc_point* dev_pts) {
    if (!c) return set_err(-EINVAL, "null argument");
    if (!c->built) return set_err(-EINVAL, "nothing built");
    if (!c->eng->num_levels()) return 0;
    GUARD_BEGIN
    uint64_t nc = 0, np = 0;
    int rc = c->eng->grid_cells(0, nc, np);
    if (rc) return set_err(rc, c->eng->last_error());
    if ((nc && (!cells_xyz || !cell_points)) || (np && !dev_pts)) return set_err(-EINVAL, "null argument");
    rc = c->eng->export_grid(0, cells_xyz, cell_points, reinterpret_cast<Point*>(dev_pts));
    return rc ? set_err(rc, c->eng->last_error()) : 0;
    GUARD_END
}

int pcc_set_summary(pcc_converter* c, uint64_t number_of_points, const float bmin[3], const float bmax[3],
                    uint32_t hierarchies) {
    if (!c || !bmin || !bmax) return set_err(-EINVAL, "null argument");
    Metadata& m = c->meta;
    m.number_of_points = number_of_points;
    m.hierarchies = hierarchies;
    for (int a = 0; a < 3; a++) {
        m.bmin[a] = number_of_points ? bmin[a] : 0.0f;
        m.bmax[a] = number_of_points ? bmax[a] : 0.0f;
    }
    c->summary_set = true;
    return 0;
}

int pcc_clear_input(pcc_converter* c) {
    if (!c) return set_err(-EINVAL, "null argument");
    GUARD_BEGIN
    c->eng->clear_input();
    c->built = false;
    c->keyed = false;
    c->summary_set = false;
    return 0;
    GUARD_END
}

// The built cloud of `src` as the merge state of `dst` (in memory, no files):
// the same state pcc_open would load from src's output directory.
int pcc_adopt_prior(pcc_converter* dst, pcc_converter* src) {
    if (!dst || !src) return set_err(-EINVAL, "null argument");
    if (dst->built || dst->eng->num_points() || dst->merge) return set_err(-EINVAL, "destination must be freshly opened");
    const Config& a = dst->meta.config;
    const Config& b = src->meta.config;
    if (a.cell_point_overflow_limit != b.cell_point_overflow_limit || a.sub_grid_dimension != b.sub_grid_dimension ||
        a.max_cell_size != b.max_cell_size)
        return set_err(-EINVAL, "configs differ");
    if (!src->built) {
        const int rc = pcc_build(src);
        if (rc) return rc;
    }
    if (!src->eng->side_cells().empty())
        return set_err(-22, "a cloud with infinite coordinates cannot be merged into (merges reject them)");
    GUARD_BEGIN
    std::vector<LevelHost> levels;
    std::vector<Point> grid, kept;
    int rc = src->eng->download(levels, grid, kept);
    if (rc) return set_err(rc, src->eng->last_error());
    std::vector<CellFile> cells;
    for (size_t i = 0; i < src->prior_cells.size(); i++)   // src is itself a merge: its untouched cells
        if (i >= src->prior_touched.size() || !src->prior_touched[i]) cells.push_back(src->prior_cells[i]);
    for (const LevelHost& L : levels) {   // cell.rs:155-181 contents without the file round trip
        const uint32_t ncells = (uint32_t)(L.cell_idx.size() / 3);
        for (uint32_t c = 0; c < ncells; c++) {
            CellFile f;
            f.h = L.h;
            for (int q = 0; q < 3; q++) f.idx[q] = L.cell_idx[3 * c + q];
            for (uint32_t s = L.cell_slab0[c]; s < L.cell_slab0[c + 1]; s++)
                f.grid.insert(f.grid.end(), grid.begin() + L.grid_base + L.slab_grid_off[s],
                              grid.begin() + L.grid_base + L.slab_grid_off[s] + L.slab_grid_n[s]);
            for (int o = 0; o < 8; o++) {
                const uint32_t st = L.bkt_state[8 * c + o];
                if (!st) continue;
                CellFile::Entry e;
                e.child[0] = 2 * f.idx[0] + (o & 1);
                e.child[1] = 2 * f.idx[1] + ((o >> 1) & 1);
                e.child[2] = 2 * f.idx[2] + ((o >> 2) & 1);
                e.some = st == 1;
                if (e.some)
                    e.pts.assign(kept.begin() + L.kept_base + L.bkt_off[8 * c + o],
                                 kept.begin() + L.kept_base + L.bkt_off[8 * c + o] + L.bkt_n[8 * c + o]);
                f.entries.push_back(std::move(e));
            }
            cells.push_back(std::move(f));
        }
    }
    PriorState ps;
    std::string err;
    rc = prior_from_cells(cells, dst->meta.config, ps, err);
    if (rc) return set_err(rc, err);
    dst->eng->set_prior(ps);
    dst->merge = true;
    dst->prior = src->meta;
    dst->prior_cells = std::move(cells);
    dst->prior_on_disk = false;
    return 0;
    GUARD_END
}

int pcc_finish(pcc_converter* c) {
    if (!c) return set_err(-EINVAL, "null argument");
    const int rc = pcc_write(c);
    delete c;
    return rc;
}

int pcc_close(pcc_converter* c) {
    delete c;
    return 0;
}

uint64_t pcc_release_device_cache(void) {
    try {
        return (uint64_t)pcc::release_device_cache();
    } catch (...) {
        return 0;
    }
}

int pcc_get_stats(const pcc_converter* c, pcc_stats* s) {
    if (!c || !s) return set_err(-EINVAL, "null argument");
    memset(s, 0, sizeof *s);
    const BuildStats& b = c->eng->stats();
    s->number_of_points = c->eng->num_points();
    s->hierarchies = c->eng->hierarchies();
    if (c->merge && c->built) {   // merged cloud: metadata values (existing + new)
        s->number_of_points = c->meta.number_of_points;
        s->hierarchies = c->meta.hierarchies;
    }
    s->levels = b.levels;
    s->cells = b.cells;
    s->slabs = b.slabs;
    s->arrivals = b.arrivals;
    s->grid_points = b.grid_points + c->untouched_grid;   // merge: + the existing cells left as they are
    s->kept_points = b.kept_points + c->untouched_kept;
    s->cells += c->untouched_cells;
    s->build_ms = c->build_ms;
    s->level0_early_tiles = b.pre0_tiles;
    s->level0_fold = b.l0_fold;
    s->sequential_replay = b.seq_replay;
    for (int a = 0; a < 3; a++) { s->bbox_min[a] = c->meta.bmin[a]; s->bbox_max[a] = c->meta.bmax[a]; }
    return 0;
}

int pcc_set_profiling(pcc_converter* c, int on) {
    if (!c) return set_err(-EINVAL, "null argument");
    c->eng->set_profiling(on != 0);
    return 0;
}

int pcc_get_profile(const pcc_converter* c, pcc_profile* out) {
    if (!c || !out) return set_err(-EINVAL, "null argument");
    const StageProfile& p = c->eng->profile();
    out->level0_ms = p.level0_ms;
    out->dense_ms = p.dense_ms;
    out->small_ms = p.small_ms;
    out->bucket_ms = p.bucket_ms;
    out->next_ms = p.next_ms;
    out->dense_arrivals = p.dense_arrivals;
    out->small_arrivals = p.small_arrivals;
    out->dense_launches = p.dense_launches;
    out->small_launches = p.small_launches;
    return 0;
}

const pcc_point* pcc_device_input(const pcc_converter* c) {
    return c ? reinterpret_cast<const pcc_point*>(c->eng->device_input()) : nullptr;
}

// lib.rs:11-60 convert_from_paths
int pcc_convert_files(const char* out_dir, const char* const* paths, size_t npaths, const pcc_options* opt) {
    pcc_converter* c = nullptr;
    {
        std::ifstream f(std::string(out_dir) + "/metadata.json");
        if (f) log_line("INFO", "Found an existing metadata file.");
        else log_line("INFO", "Found no metadata file. A new one will be created.");
    }
    int rc = pcc_open(out_dir, opt, &c);
    if (rc) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < npaths; i++) {
        const std::string p = paths[i];
        log_line("INFO", "Converting file %zu/%zu, \"%s\"", i + 1, npaths, p.c_str());
        const size_t dot = p.find_last_of('.');
        const size_t slash = p.find_last_of('/');
        std::string ext = (dot == std::string::npos || (slash != std::string::npos && dot < slash)) ? "" : p.substr(dot + 1);
        // lib.rs:31-52: a get_batch error is logged and ends that file; the batches
        // read before it stay, the failing batch is lost, the next file follows.
        // So a file whose data ends early contributes its complete batches only.
        const uint64_t B = c->opt.batch_size;
        if (ext == "ply") {
            // streamed: the reader's pieces go through the pinned ring to the
            // device while the next piece is read (HIP-stream upload scheduler)
            PlyResult r;
            std::string err;
            bool open = false, logged = false;
            uint64_t pushed = 0;
            int src = 0;
            const PointSink sink = [&](const Point* pts, uint64_t m) -> bool {
                if (!logged) { log_line("INFO", "Converting %llu points", (unsigned long long)r.vertex_count); logged = true; }
                if (!open) { if ((src = pcc_begin_file(c, r.vertex_count))) return false; open = true; }
                if ((src = pcc_append_points(c, reinterpret_cast<const pcc_point*>(pts), m))) return false;
                pushed += m;
                return true;
            };
            const bool ok = read_ply(p, r, err, sink);
            if (!ok || src) {
                if (open) pcc_cancel_file(c);
                pcc_close(c);
                return src ? src : set_err(-EIO, err);   // the reference unwraps header parsing (ply.rs:20-24)
            }
            if (!logged) log_line("INFO", "Converting %llu points", (unsigned long long)r.vertex_count);
            if (r.ascii) {
                const uint64_t nb = r.data_error.empty() ? std::max<uint64_t>(1, (r.vertex_count + B - 1) / B)
                                                         : r.ascii_lines / B;
                if (nb) rc = pcc_add_empty_batches(c, (uint32_t)nb);
            } else {
                // lib.rs:31-52: a truncated file keeps its complete batches; none at all: no batch
                const uint64_t keep = r.data_error.empty() ? pushed : (pushed / B) * B;
                if (open) rc = (r.data_error.empty() || keep) ? pcc_end_file(c, keep) : pcc_cancel_file(c);
                else if (r.data_error.empty()) rc = pcc_add_points(c, nullptr, 0);   // an empty file: one empty batch
            }
            if (rc) { pcc_close(c); return rc; }
            if (!r.data_error.empty()) log_line("ERROR", "%s", r.data_error.c_str());
        } else if (ext == "las" || ext == "laz") {   // converter/las.rs:14-46, streamed like PLY
            LasResult r;
            std::string err;
            bool open = false, logged = false;
            uint64_t pushed = 0;
            int src = 0;
            const PointSink sink = [&](const Point* pts, uint64_t m) -> bool {
                if (!logged) { log_line("INFO", "Converting %llu points", (unsigned long long)r.count); logged = true; }
                if (!open) { if ((src = pcc_begin_file(c, r.count))) return false; open = true; }
                if ((src = pcc_append_points(c, reinterpret_cast<const pcc_point*>(pts), m))) return false;
                pushed += m;
                return true;
            };
            const bool ok = read_las(p, r, err, sink);
            if (!ok || src) {
                if (open) pcc_cancel_file(c);
                pcc_close(c);
                return src ? src : set_err(-EIO, err);   // the reference unwraps Reader::from_path (las.rs:16)
            }
            if (!r.laz_error.empty()) {
                log_line("ERROR", "%s", r.laz_error.c_str());
                continue;
            }
            if (!logged) log_line("INFO", "Converting %llu points", (unsigned long long)r.count);
            const uint64_t keep = r.data_error.empty() ? pushed : (pushed / B) * B;
            if (open) rc = (r.data_error.empty() || keep) ? pcc_end_file(c, keep) : pcc_cancel_file(c);
            else if (r.data_error.empty()) rc = pcc_add_points(c, nullptr, 0);   // no points: one empty batch
            if (rc) { pcc_close(c); return rc; }
            if (!r.data_error.empty()) log_line("ERROR", "%s", r.data_error.c_str());
        } else if (ext == "json") {   // converter/own.rs: another converted cloud as input, streamed
            uint64_t total = 0, pushed = 0;
            std::string err;
            bool open = false, logged = false;
            int src = 0;
            const PointSink sink = [&](const Point* pts, uint64_t m) -> bool {
                if (!logged) { log_line("INFO", "Converting %llu points", (unsigned long long)total); logged = true; }
                if (!open) { if ((src = pcc_begin_file(c, total))) return false; open = true; }
                if ((src = pcc_append_points(c, reinterpret_cast<const pcc_point*>(pts), m))) return false;
                pushed += m;
                return true;
            };
            const int r = read_cloud_points(p, total, sink, err);
            if (src) {   // the converter refused a piece
                if (open) pcc_cancel_file(c);
                pcc_close(c);
                return src;
            }
            if (r) {   // lib.rs:75-77 unwraps; reported instead, the file contributes nothing
                if (open) pcc_cancel_file(c);
                log_line("ERROR", "%s", err.c_str());
                continue;
            }
            if (!logged) log_line("INFO", "Converting %llu points", (unsigned long long)total);
            rc = open ? pcc_end_file(c, pushed) : pcc_add_points(c, nullptr, 0);   // an empty cloud: one empty batch
            if (rc) { pcc_close(c); return rc; }
        } else {
            log_line("WARN", "Unsupported file format '%s'", ext.c_str());   // lib.rs:78-81
        }
    }
    rc = pcc_build(c);
    if (rc) { pcc_close(c); return rc; }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    log_line("INFO", "Finished converting after %llu ms", (unsigned long long)ms);   // lib.rs:56-59
    return pcc_finish(c);
}

}  // extern "C"
