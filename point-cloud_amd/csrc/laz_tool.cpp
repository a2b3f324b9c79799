// laz_tool — LAS <-> LAZ utility over laz.h (tests and manual checks; not part
// of the converter).
//   laz_tool compress   IN.las OUT.laz [chunk_size]   formats 0-3 (pointwise chunked), 6-8 (layered chunked)
//   laz_tool decompress IN.laz OUT.las
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "laz.h"

using namespace pcc;

static bool read_file(const char* path, std::vector<uint8_t>& d) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    d.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    const bool ok = fread(d.data(), 1, d.size(), f) == d.size();
    fclose(f);
    return ok;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: laz_tool compress IN.las OUT.laz [chunk_size] | decompress IN.laz OUT.las\n");
        return 2;
    }
    const std::string mode = argv[1];
    std::vector<uint8_t> in;
    if (!read_file(argv[2], in) || in.size() < 227 || memcmp(in.data(), "LASF", 4) != 0) {
        fprintf(stderr, "cannot read LAS file %s\n", argv[2]);
        return 1;
    }
    auto u16 = [&](size_t o) { uint16_t v; memcpy(&v, in.data() + o, 2); return v; };
    auto u32 = [&](size_t o) { uint32_t v; memcpy(&v, in.data() + o, 4); return v; };
    auto u64 = [&](size_t o) { uint64_t v; memcpy(&v, in.data() + o, 8); return v; };
    const uint16_t hsize = u16(94);
    const uint32_t data_off = u32(96), nvlr = u32(100);
    const uint8_t fmt_raw = in[104];
    const uint16_t rec = u16(105);
    uint64_t n = u32(107);
    if (in[25] >= 4 && hsize >= 375) n = u64(247);
    if (mode == "compress") {
        if (fmt_raw & 0x80) { fprintf(stderr, "already compressed\n"); return 1; }
        const uint32_t chunk = argc > 4 ? (uint32_t)strtoul(argv[4], nullptr, 10) : 50000u;
        laz::Vlr v;
        v.compressor = laz::compressor_for_format(fmt_raw & 0x3F);
        v.coder = 0;
        v.version_major = v.compressor == 3 ? 3 : 2;
        v.version_minor = v.compressor == 3 ? 4 : 2;
        v.chunk_size = chunk;
        std::string err;
        if (!laz::items_for_format(fmt_raw & 0x3F, rec, v.items, err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
        const std::vector<uint8_t> vd = laz::write_vlr(v);
        const std::vector<uint8_t> data = laz::compress(in.data() + data_off, n, rec, v.items, chunk);
        // header + existing VLRs (up to the point data) + the LASzip VLR
        std::vector<uint8_t> out(in.begin(), in.begin() + data_off);
        std::vector<uint8_t> vh(54, 0);
        memcpy(vh.data() + 2, "laszip encoded", 14);
        const uint16_t rid = 22204, len = (uint16_t)vd.size();
        memcpy(vh.data() + 18, &rid, 2);
        memcpy(vh.data() + 20, &len, 2);
        out.insert(out.end(), vh.begin(), vh.end());
        out.insert(out.end(), vd.begin(), vd.end());
        const uint32_t new_off = (uint32_t)out.size(), new_nvlr = nvlr + 1;
        memcpy(out.data() + 96, &new_off, 4);
        memcpy(out.data() + 100, &new_nvlr, 4);
        out[104] = fmt_raw | 0x80;
        // the chunk table offset is relative to the file: shift it by the point data's start
        std::vector<uint8_t> d2 = data;
        int64_t tab;
        memcpy(&tab, d2.data(), 8);
        tab += new_off;
        memcpy(d2.data(), &tab, 8);
        out.insert(out.end(), d2.begin(), d2.end());
        FILE* f = fopen(argv[3], "wb");
        if (!f || fwrite(out.data(), 1, out.size(), f) != out.size()) { fprintf(stderr, "cannot write %s\n", argv[3]); return 1; }
        fclose(f);
        return 0;
    }
    if (mode == "decompress") {
        if (!(fmt_raw & 0x80)) { fprintf(stderr, "not compressed\n"); return 1; }
        laz::Vlr v;
        bool found = false;
        size_t pos = hsize;
        std::vector<uint8_t> vlrs;   // the other VLRs, kept
        uint32_t kept = 0;
        for (uint32_t i = 0; i < nvlr; i++) {
            uint16_t rid, len;
            memcpy(&rid, in.data() + pos + 18, 2);
            memcpy(&len, in.data() + pos + 20, 2);
            std::string err;
            if (memcmp(in.data() + pos + 2, "laszip encoded", 14) == 0 && rid == 22204) {
                found = laz::parse_vlr(in.data() + pos + 54, len, v, err);
            } else {
                vlrs.insert(vlrs.end(), in.begin() + pos, in.begin() + pos + 54 + len);
                kept++;
            }
            pos += 54 + len;
        }
        if (!found) { fprintf(stderr, "no LASzip VLR\n"); return 1; }
        FILE* f = fopen(argv[2], "rb");
        laz::Reader r;
        std::string err;
        if (!r.open(f, data_off, n, rec, v, err)) { fprintf(stderr, "%s\n", err.c_str()); return 1; }
        std::vector<uint8_t> recs(n * rec);
        const uint64_t got = r.read(recs.data(), n, err);
        fclose(f);
        if (got != n) { fprintf(stderr, "decoded %llu of %llu points: %s\n", (unsigned long long)got, (unsigned long long)n, err.c_str()); return 1; }
        std::vector<uint8_t> out(in.begin(), in.begin() + hsize);
        out.insert(out.end(), vlrs.begin(), vlrs.end());
        const uint32_t off = (uint32_t)out.size();
        memcpy(out.data() + 96, &off, 4);
        memcpy(out.data() + 100, &kept, 4);
        out[104] = fmt_raw & 0x3F;
        out.insert(out.end(), recs.begin(), recs.end());
        FILE* o = fopen(argv[3], "wb");
        if (!o || fwrite(out.data(), 1, out.size(), o) != out.size()) { fprintf(stderr, "cannot write %s\n", argv[3]); return 1; }
        fclose(o);
        return 0;
    }
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
}
