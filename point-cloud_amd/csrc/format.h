// format.h — the reference's on-disk formats and input readers (host C++17).
//   cell files     point-converter/src/cell.rs:155-229, 280-335; point.rs:26-54
//   metadata.json  point-converter/src/metadata.rs:9-57 (serde_json pretty)
//   PLY input      point-converter/src/converter/ply.rs:19-73 + point.rs:56-130
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

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
int write_output(const std::string& dir, const Metadata& meta, const std::vector<LevelHost>& levels,
                 const std::vector<Point>& grid, const std::vector<Point>& kept, std::string& err,
                 bool with_metadata = true);
int write_metadata(const std::string& dir, const Metadata& meta, std::string& err);

// PLY reader.  Returns points of the `vertex` element.  `ascii` is set when the
// file is ASCII-encoded: the reference's ASCII branch parses but never stores
// the points (ply.rs:43-51), so callers must feed empty batches instead.
struct PlyResult {
    std::vector<Point> points;
    uint64_t vertex_count = 0;
    bool ascii = false;
};
bool read_ply(const std::string& path, PlyResult& out, std::string& err);

}  // namespace pcc
