// laz.h — LAZ (LASzip) point-data decompression for the LAS reader
// (converter/las.rs:14-46 reads .laz through las 0.8.4 + laz 0.9.1 [dep]).
//
// Restated from the published LASzip format (the format of laz-perf / laszip /
// laz-rs): an adaptive binary arithmetic coder (Amir Said's FastAC model as
// LASzip uses it), integer compressors with k-bit correctors, and
//   point formats 0-5: "pointwise chunked" compression with the version-2
//     item compressors POINT10, GPSTIME11, RGB12 and BYTE, and WAVEPACKET13
//     version 1 (formats 4 / 5: LASzip has no other version of it);
//   point formats 6-10: LASzip 3 "layered chunked" compression with the
//     version-3 items POINT14, RGB14, RGBNIR14, WAVEPACKET14 and BYTE14 (one
//     arithmetic stream per field group, models per scanner channel).
//
// The encoder half exists for tests and the laz_tool utility (LAS -> LAZ),
// never for the converter.  Parity unpinned: no .laz fixture ships with the
// reference and no LASzip implementation is available here, so round trips
// through this codec are all that the tests check.  The layered coder's
// context tables (return map, first-point flags) are restated from memory of
// the LASzip 3 design and are the least certain part.
#pragma once
#include <stdint.h>
#include <stdio.h>

#include <memory>
#include <string>
#include <vector>

namespace pcc {
namespace laz {

enum ItemType : uint16_t {
    BYTE = 0, POINT10 = 6, GPSTIME11 = 7, RGB12 = 8, WAVEPACKET13 = 9, POINT14 = 10, RGB14 = 11, RGBNIR14 = 12,
    WAVEPACKET14 = 13, BYTE14 = 14
};
struct Item { uint16_t type, size, version; };

// The LASzip VLR (user id "laszip encoded", record id 22204)
struct Vlr {
    uint16_t compressor = 0;   // 1 pointwise, 2 pointwise chunked, 3 layered chunked
    uint16_t coder = 0;        // 0 arithmetic
    uint8_t version_major = 0, version_minor = 0;
    uint16_t version_revision = 0;
    uint32_t options = 0;
    uint32_t chunk_size = 0;   // points per chunk (0xFFFFFFFF: variable, counts in the chunk table)
    int64_t number_of_special_evlrs = -1, offset_to_special_evlrs = -1;
    std::vector<Item> items;
};
bool parse_vlr(const uint8_t* d, size_t n, Vlr& v, std::string& err);
std::vector<uint8_t> write_vlr(const Vlr& v);
// Items of a LAS point format 0-10 record of `rec` bytes (extra bytes as
// BYTE / BYTE14); compressor 2 for formats 0-5, 3 (layered) for 6-10
uint16_t compressor_for_format(uint8_t format);
bool items_for_format(uint8_t format, uint16_t rec, std::vector<Item>& items, std::string& err);

class PointDecoder;
// Sequential reader of the compressed point records of one file.
class Reader {
public:
    Reader();
    ~Reader();
    // f positioned anywhere; data_off = offset to point data (LAS header)
    bool open(FILE* f, uint64_t data_off, uint64_t npoints, uint16_t rec, const Vlr& v, std::string& err);
    // decodes up to m records (m * rec bytes) into out; returns the count decoded
    // (fewer than m only at the end of the data or on an error, then err is set)
    uint64_t read(uint8_t* out, uint64_t m, std::string& err);

private:
    bool load_chunk(std::string& err);
    FILE* f_ = nullptr;
    uint16_t rec_ = 0;
    uint64_t left_ = 0;                         // points not yet returned
    Vlr v_;
    std::vector<uint64_t> chunk_start_, chunk_pts_;
    size_t chunk_ = 0;
    uint64_t in_chunk_ = 0, chunk_n_ = 0;        // points read from / in the current chunk
    std::vector<uint8_t> buf_;                  // the current chunk's bytes
    std::unique_ptr<PointDecoder> dec_;
};

// LAS point records (formats 0-10, `rec` bytes each) -> LASzip point
// data: the 8-byte chunk-table offset, the chunks, the chunk table.
std::vector<uint8_t> compress(const uint8_t* recs, uint64_t n, uint16_t rec, const std::vector<Item>& items,
                              uint32_t chunk_size);

}  // namespace laz
}  // namespace pcc
