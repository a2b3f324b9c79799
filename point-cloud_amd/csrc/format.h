// format.h — the reference's on-disk formats and input readers (host C++17).
//   cell files     point-converter/src/cell.rs:155-229, 280-335; point.rs:26-54
//   metadata.json  point-converter/src/metadata.rs:9-57 (serde_json pretty)
//   PLY input      point-converter/src/converter/ply.rs:19-73 + point.rs:56-130
#pragma once
#include <stdint.h>
#include <functional>
#include <string>
#include <vector>

#include "../../include/pcconv.h"
#include "engine.h"

namespace pcc {

struct Metadata {                  // metadata.rs:9-41
    std::string version = "1.0";
    std::string name = "Unknown";
    uint64_t number_of_points = 0;
    uint32_t hierarchies = 0;
    float bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
    Config config;
};

std::string format_f32(float v);                       // ryu-style shortest round trip
std::string metadata_json(const Metadata& m);           // serde_json::to_writer_pretty layout
bool parse_metadata_json(const std::string& text, Metadata& m, std::string& err);

// Writes h_{h}/c_{x}_{y}_{z}.bin for every cell of every level, then metadata.json
// (converter.rs:218-238 order: cells first, metadata last).
// with_metadata=false writes the cells only (sharded build: rank 0 writes the
// global metadata.json once all ranks' cells are on disk).
int make_output_dirs(const std::string& dir, uint32_t hierarchies, std::string& err);
// Cell c of a downloaded level as the C ABI's view (header values as
// Cell::write_to stores them, cell.rs:155-181; pointers into grid / kept).
void level_cell_view(const Config& cfg, const LevelHost& L, uint32_t c, const Point* grid, const Point* kept,
                     pcc_cell_view& v);
// Cell files of one level, split over nthreads host threads.
// One cell file from a view (h_{h}/c_x_y_z.bin under dir; folders created).
void serialize_view(const pcc_cell_view& v, std::string& buf);
int write_view_file(const std::string& dir, const pcc_cell_view& v, std::string& err);
int write_level_cells(const std::string& dir, const Config& cfg, const LevelHost& L, const Point* grid,
                      const Point* kept, unsigned nthreads, std::string& err);
unsigned writer_threads();   // PCC_WRITE_THREADS, else min(16, hardware threads)
// cells as read from disk, written back unchanged (skip[i] != 0: not written)
int write_cell_files(const std::string& dir, const Config& cfg, const std::vector<CellFile>& cells,
                     const std::vector<uint8_t>* skip, std::string& err);
int write_output(const std::string& dir, const Metadata& meta, const std::vector<LevelHost>& levels,
                 const std::vector<Point>& grid, const std::vector<Point>& kept, std::string& err,
                 bool with_metadata = true);
int write_metadata(const std::string& dir, const Metadata& meta, std::string& err);

// (CellFile: engine.h)
bool read_cell_file(const std::string& path, CellFile& out, std::string& err);
// Every h_{h}/c_{x}_{y}_{z}.bin with h < hierarchies (the layout own.rs:16-62 and
// converter.rs:187-207 read; the order of the returned cells is unspecified).
// subtrees (optional): level-0 cell triples; only cells below them are read
int read_cloud(const std::string& dir, uint32_t hierarchies, std::vector<CellFile>& cells, std::string& err,
               const std::vector<int32_t>* subtrees = nullptr);
// The existing cloud as the engine's merge state (engine.h PriorState).
int prior_from_cells(const std::vector<CellFile>& cells, const Config& cfg, PriorState& out, std::string& err);

// PLY reader.  Returns points of the `vertex` element.  `ascii` is set when the
// file is ASCII-encoded: the reference's ASCII branch parses but never stores
// the points (ply.rs:43-51), so callers must feed empty batches instead.
struct PlyResult {
    std::vector<Point> points;
    uint64_t vertex_count = 0;
    bool ascii = false;
    uint64_t ascii_lines = 0;   // ASCII: vertex lines present (a short file ends the reader early)
    std::string data_error;     // set when the vertex data ends early or is unreadable:
                                // `points` then holds the records read before the error
};
// sink: when set, the points are handed over in pieces (file order) instead of
// being collected in out.points; returning false stops the reader.
using PointSink = std::function<bool(const Point*, uint64_t)>;
bool read_ply(const std::string& path, PlyResult& out, std::string& err, const PointSink& sink = nullptr);

// LAS reader (converter/las.rs:23-46 over las 0.8.4 [dep]): uncompressed LAS
// 1.0-1.4, point formats 0-10.  x = (scale * X + offset) in f64 (las
// Transform::direct), then `as f32`; colour = u16 `as u8` (low byte), alpha 255;
// formats without colour give (0, 0, 0, 255) (Color::default).  Compressed
// point data (LAZ, `laz` = true) is decoded by laz.h for point formats 0-3;
// other LAZ variants set `laz_error` and give no points.
struct LasResult {
    std::vector<Point> points;
    uint64_t count = 0;   // header number_of_points
    bool laz = false;
    std::string laz_error;   // a LAZ variant this build does not decode
    std::string data_error;   // truncated point data: `points` holds the records read before it
};
bool read_las(const std::string& path, LasResult& out, std::string& err, const PointSink& sink = nullptr);

// Points of a converted cloud used as an input file (converter/own.rs:16-78):
// h_0 .. h_{H-1}, every cell's grid points then its Some lists.  The reference
// enumerates directories and FxHashMaps in unspecified order; this reader fixes
// the order (file names sorted, grid and overflow entries in file order), so
// parity for this input is defined relative to that enumeration.
// converter/own.rs: another cloud (its metadata.json) as an input file, its
// points handed to `sink` cell after cell (grid, then kept lists), streamed
// through windows of cell files; -ECANCELED when the sink stops it
int read_cloud_points(const std::string& metadata_path, uint64_t& number_of_points, const PointSink& sink,
                      std::string& err);

}  // namespace pcc
