// format.cpp — cell / metadata writers and the PLY reader (see format.h).
#include "format.h"
#include "laz.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <thread>

#include "pcc_math.h"

namespace pcc {

// ------------------------------------------------------------------ floats
// Shortest round-trip digits (std::to_chars) laid out like ryu::Buffer::format
// for f32 (serde_json 1.0.114 -> ryu 1.0.17 [dep]).  Byte parity unpinned:
// tests compare parsed values.
std::string format_f32(float v) {
    if (v == 0.0f) return std::signbit(v) ? "-0.0" : "0.0";
    // serde_json serializes a non-finite f32 as null (the bounding box of an
    // input with infinite coordinates, bounding-volume/src/lib.rs:23-31)
    if (!std::isfinite(v)) return "null";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
    std::string s(buf, r.ptr);   // [-]d[.ddd]e[+-]xx
    bool neg = false;
    size_t i = 0;
    if (s[0] == '-') { neg = true; i = 1; }
    std::string digits;
    for (; i < s.size() && s[i] != 'e'; i++)
        if (s[i] != '.') digits += s[i];
    int ex = std::atoi(s.c_str() + i + 1);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const int nd = (int)digits.size();
    const int k = ex - (nd - 1), kk = nd + k;
    std::string o = neg ? "-" : "";
    if (0 <= k && kk <= 13) {
        o += digits + std::string(k, '0') + ".0";
    } else if (0 < kk && kk <= 13) {
        o += digits.substr(0, kk) + "." + digits.substr(kk);
    } else if (-6 < kk && kk <= 0) {
        o += "0." + std::string(-kk, '0') + digits;
    } else if (nd == 1) {
        o += digits + "e" + std::to_string(kk - 1);
    } else {
        o += digits.substr(0, 1) + "." + digits.substr(1) + "e" + std::to_string(kk - 1);
    }
    return o;
}

std::string metadata_json(const Metadata& m) {
    std::ostringstream o;
    o << "{\n  \"version\": \"" << m.version << "\",\n  \"name\": \"" << m.name << "\",\n"
      << "  \"number_of_points\": " << m.number_of_points << ",\n  \"hierarchies\": " << m.hierarchies << ",\n"
      << "  \"bounding_box\": {\n    \"min\": [\n      " << format_f32(m.bmin[0]) << ",\n      " << format_f32(m.bmin[1])
      << ",\n      " << format_f32(m.bmin[2]) << "\n    ],\n    \"max\": [\n      " << format_f32(m.bmax[0]) << ",\n      "
      << format_f32(m.bmax[1]) << ",\n      " << format_f32(m.bmax[2]) << "\n    ]\n  },\n  \"config\": {\n"
      << "    \"cell_point_overflow_limit\": " << m.config.cell_point_overflow_limit << ",\n"
      << "    \"sub_grid_dimension\": " << m.config.sub_grid_dimension << ",\n"
      << "    \"max_cell_size\": " << format_f32(m.config.max_cell_size) << "\n  }\n}";
    return o.str();
}

// Minimal JSON reader for the metadata schema (metadata.rs:9-28).
namespace {
struct J {
    const std::string& s;
    size_t i = 0;
    std::string err;
    explicit J(const std::string& t) : s(t) {}
    void ws() { while (i < s.size() && isspace((unsigned char)s[i])) i++; }
    bool eat(char c) { ws(); if (i < s.size() && s[i] == c) { i++; return true; } return false; }
    bool str(std::string& out) {
        ws();
        if (i >= s.size() || s[i] != '"') return false;
        i++;
        out.clear();
        while (i < s.size() && s[i] != '"') {
            if (s[i] == '\\' && i + 1 < s.size()) i++;
            out += s[i++];
        }
        if (i >= s.size()) return false;
        i++;
        return true;
    }
    bool num(double& v) {
        ws();
        size_t j = i;
        while (j < s.size() && (isdigit((unsigned char)s[j]) || strchr("+-.eE", s[j]))) j++;
        if (j == i) return false;
        v = strtod(s.substr(i, j - i).c_str(), nullptr);
        i = j;
        return true;
    }
    bool f32num(float& v) {   // parse as f32 directly (serde_json parses f32 fields via f64 then `as f32`)
        double d;
        if (!num(d)) return false;
        v = (float)d;
        return true;
    }
    bool null_seen = false;   // a `null` component (serde_json's non-finite f32)
    bool vec3(float* v) {
        if (!eat('[')) return false;
        for (int a = 0; a < 3; a++) {
            ws();
            if (s.compare(i, 4, "null") == 0) {   // kept as NaN; the caller reports it
                i += 4;
                v[a] = NAN;
                null_seen = true;
            } else if (!f32num(v[a])) {
                return false;
            }
            if (a < 2 && !eat(',')) return false;
        }
        return eat(']');
    }
    bool skip() {   // skip any value
        ws();
        if (i >= s.size()) return false;
        if (s[i] == '"') { std::string t; return str(t); }
        if (s[i] == '{' || s[i] == '[') {
            char open = s[i], close = open == '{' ? '}' : ']';
            int depth = 0;
            bool instr = false;
            for (; i < s.size(); i++) {
                if (instr) { if (s[i] == '\\') i++; else if (s[i] == '"') instr = false; continue; }
                if (s[i] == '"') instr = true;
                else if (s[i] == open) depth++;
                else if (s[i] == close && --depth == 0) { i++; return true; }
            }
            return false;
        }
        double d;
        if (num(d)) return true;
        for (const char* w : {"true", "false", "null"})
            if (s.compare(i, strlen(w), w) == 0) { i += strlen(w); return true; }
        return false;
    }
};
}  // namespace

bool parse_metadata_json(const std::string& text, Metadata& m, std::string& err) {
    J j(text);
    if (!j.eat('{')) { err = "metadata.json: expected object"; return false; }
    bool first = true;
    while (!j.eat('}')) {
        if (!first && !j.eat(',')) { err = "metadata.json: expected ,"; return false; }
        first = false;
        std::string key;
        if (!j.str(key) || !j.eat(':')) { err = "metadata.json: bad key"; return false; }
        double d;
        bool ok = true;
        if (key == "version") ok = j.str(m.version);
        else if (key == "name") ok = j.str(m.name);
        else if (key == "number_of_points") { ok = j.num(d); m.number_of_points = (uint64_t)d; }
        else if (key == "hierarchies") { ok = j.num(d); m.hierarchies = (uint32_t)d; }
        else if (key == "bounding_box") {
            ok = j.eat('{');
            bool f2 = true;
            while (ok && !j.eat('}')) {
                if (!f2 && !j.eat(',')) { ok = false; break; }
                f2 = false;
                std::string k2;
                ok = j.str(k2) && j.eat(':');
                if (!ok) break;
                if (k2 == "min") ok = j.vec3(m.bmin);
                else if (k2 == "max") ok = j.vec3(m.bmax);
                else ok = j.skip();
            }
        } else if (key == "config") {
            ok = j.eat('{');
            bool f2 = true;
            while (ok && !j.eat('}')) {
                if (!f2 && !j.eat(',')) { ok = false; break; }
                f2 = false;
                std::string k2;
                ok = j.str(k2) && j.eat(':');
                if (!ok) break;
                if (k2 == "cell_point_overflow_limit") { ok = j.num(d); m.config.cell_point_overflow_limit = (uint32_t)d; }
                else if (k2 == "sub_grid_dimension") { ok = j.num(d); m.config.sub_grid_dimension = (uint32_t)d; }
                else if (k2 == "max_cell_size") ok = j.f32num(m.config.max_cell_size);
                else ok = j.skip();
            }
        } else ok = j.skip();
        if (!ok) { err = "metadata.json: bad value for " + key; return false; }
    }
    if (j.null_seen) {
        // lib.rs:86-101 reads the file with serde_json, which refuses `null` for
        // an f32 (the reference panics there): a cloud with infinite coordinates,
        // or an axis of NaN only, cannot be merged into
        err = "metadata.json: the existing cloud's bounding box is not finite (null), so it cannot be merged into "
              "(the reference's serde_json cannot read it back either)";
        return false;
    }
    return true;
}

// ------------------------------------------------------------------ cells
static void put32(std::string& b, uint32_t v) { b.append(reinterpret_cast<const char*>(&v), 4); }
static void putf(std::string& b, float v) { b.append(reinterpret_cast<const char*>(&v), 4); }

int make_output_dirs(const std::string& dir, uint32_t hierarchies, std::string& err) {
    if (mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST) { err = "cannot create " + dir; return -errno; }
    for (uint32_t h = 0; h < hierarchies; h++) {   // converter.rs:141-158
        std::string hd = dir + "/h_" + std::to_string(h);
        if (mkdir(hd.c_str(), 0755) != 0 && errno != EEXIST) { err = "cannot create " + hd; return -errno; }
    }
    return 0;
}

// Header values of a new cell (converter.rs:197-199, cell.rs:43-49, 264-274) and
// its contents after the build.  A cell's slabs are consecutive and the
// downloaded winners are compacted in slab order, so its grid points are one
// contiguous run.
void level_cell_view(const Config& cfg, const LevelHost& L, uint32_t c, const Point* grid, const Point* kept,
                     pcc_cell_view& v) {
    const float size = cell_size(cfg.max_cell_size, L.h);
    v.hierarchy = L.h;
    v.x = L.cell_idx[3 * c];
    v.y = L.cell_idx[3 * c + 1];
    v.z = L.cell_idx[3 * c + 2];
    uint32_t number = 0, overflow = 0, nb = 0;
    for (uint32_t s = L.cell_slab0[c]; s < L.cell_slab0[c + 1]; s++) number += L.slab_grid_n[s];
    const uint32_t s0 = L.cell_slab0[c];
    v.grid = reinterpret_cast<const pcc_point*>(grid + L.grid_base + (s0 < L.slab_grid_off.size() ? L.slab_grid_off[s0] : 0));
    for (int o = 0; o < 8; o++) {
        const uint32_t st = L.bkt_state[8 * c + o];
        if (!st) continue;
        v.child[nb][0] = 2 * v.x + (o & 1);
        v.child[nb][1] = 2 * v.y + ((o >> 1) & 1);
        v.child[nb][2] = 2 * v.z + ((o >> 2) & 1);
        if (st == 1) {
            v.count[nb] = L.bkt_n[8 * c + o];
            v.list[nb] = reinterpret_cast<const pcc_point*>(kept + L.kept_base + L.bkt_off[8 * c + o]);
            overflow += v.count[nb];
        } else {
            v.count[nb] = 0;
            v.list[nb] = nullptr;
        }
        nb++;
    }
    v.entries = nb;
    v.total_number_of_points = number + overflow;
    v.number_of_points = number;
    v.number_of_overflow_points = overflow;
    v.size = size;
    v.sub_cell_size = sub_cell_size(size, cfg.sub_grid_dimension);
    v.pos[0] = cell_pos1(v.x, size);
    v.pos[1] = cell_pos1(v.y, size);
    v.pos[2] = cell_pos1(v.z, size);
}

// Cell::write_to cell.rs:155-181 with Header::write_to :280-298, from a view.
void serialize_view(const pcc_cell_view& v, std::string& buf) {
    buf.clear();
    buf.reserve(48 + 16ull * v.total_number_of_points + 1 + 16 * v.entries);
    put32(buf, v.hierarchy);
    put32(buf, (uint32_t)v.x); put32(buf, (uint32_t)v.y); put32(buf, (uint32_t)v.z);
    put32(buf, v.total_number_of_points);
    put32(buf, v.number_of_points);
    put32(buf, v.number_of_overflow_points);
    putf(buf, v.size);
    putf(buf, v.sub_cell_size);
    putf(buf, v.pos[0]); putf(buf, v.pos[1]); putf(buf, v.pos[2]);
    // grid points (cell.rs:158-160; order free)
    buf.append(reinterpret_cast<const char*>(v.grid), 16ull * v.number_of_points);
    buf.push_back((char)(uint8_t)v.entries);   // cell.rs:162
    for (uint32_t e = 0; e < v.entries; e++) {
        put32(buf, (uint32_t)v.child[e][0]);
        put32(buf, (uint32_t)v.child[e][1]);
        put32(buf, (uint32_t)v.child[e][2]);
        put32(buf, v.count[e]);
        if (v.count[e]) buf.append(reinterpret_cast<const char*>(v.list[e]), 16ull * v.count[e]);
    }
}

int write_view_file(const std::string& dir, const pcc_cell_view& v, std::string& err) {
    const std::string hd = dir + "/h_" + std::to_string(v.hierarchy);
    if (mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST) { err = "cannot create " + dir; return -EIO; }
    if (mkdir(hd.c_str(), 0755) != 0 && errno != EEXIST) { err = "cannot create " + hd; return -EIO; }
    std::string buf;
    serialize_view(v, buf);
    char name[96];
    snprintf(name, sizeof name, "/c_%d_%d_%d.bin", v.x, v.y, v.z);
    const std::string path = hd + name;
    FILE* fp = fopen(path.c_str(), "wb");
    bool ok = fp != nullptr;
    if (ok) { ok = fwrite(buf.data(), 1, buf.size(), fp) == buf.size(); ok = (fclose(fp) == 0) && ok; }
    if (!ok) { err = "cannot write " + path; return -EIO; }
    return 0;
}

// Cell files of one level (Cell::write_to cell.rs:155-181, Header::write_to
// :280-298), cells split over `nthreads` host threads (files are independent).
int write_level_cells(const std::string& dir, const Config& cfg, const LevelHost& L, const Point* grid,
                      const Point* kept, unsigned nthreads, std::string& err) {
    const uint32_t h = L.h;
    const uint32_t ncells = (uint32_t)(L.cell_idx.size() / 3);
    std::atomic<uint32_t> next{0};
    std::atomic<int> rc{0};
    std::mutex emu;
    auto work = [&]() {
        std::string buf;
        pcc_cell_view v;
        for (;;) {
            const uint32_t c = next.fetch_add(1);
            if (c >= ncells || rc.load() != 0) return;
            level_cell_view(cfg, L, c, grid, kept, v);
            serialize_view(v, buf);
            const int32_t ix = v.x, iy = v.y, iz = v.z;
            char name[96];
            snprintf(name, sizeof name, "/h_%u/c_%d_%d_%d.bin", h, ix, iy, iz);
            const std::string path = dir + name;
            FILE* f = fopen(path.c_str(), "wb");
            bool ok = f != nullptr;
            if (ok) {
                ok = fwrite(buf.data(), 1, buf.size(), f) == buf.size();
                ok = (fclose(f) == 0) && ok;
            }
            if (!ok) {
                std::lock_guard<std::mutex> g(emu);
                if (rc.load() == 0) { err = "cannot write " + path; rc.store(-EIO); }
                return;
            }
        }
    };
    const unsigned nt = std::max(1u, std::min<unsigned>(nthreads, ncells));
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    return rc.load();
}

int write_cell_files(const std::string& dir, const Config& cfg, const std::vector<CellFile>& cells,
                     const std::vector<uint8_t>* skip, std::string& err) {
    std::string buf;
    for (size_t i = 0; i < cells.size(); i++) {
        if (skip && i < skip->size() && (*skip)[i]) continue;
        const CellFile& f = cells[i];
        const float size = cell_size(cfg.max_cell_size, f.h);
        buf.clear();
        put32(buf, f.h);
        put32(buf, (uint32_t)f.idx[0]); put32(buf, (uint32_t)f.idx[1]); put32(buf, (uint32_t)f.idx[2]);
        put32(buf, f.total); put32(buf, f.number); put32(buf, f.overflow);
        putf(buf, size);
        putf(buf, sub_cell_size(size, cfg.sub_grid_dimension));
        putf(buf, cell_pos1(f.idx[0], size)); putf(buf, cell_pos1(f.idx[1], size)); putf(buf, cell_pos1(f.idx[2], size));
        buf.append(reinterpret_cast<const char*>(f.grid.data()), 16ull * f.grid.size());
        buf.push_back((char)(uint8_t)f.entries.size());
        for (const CellFile::Entry& e : f.entries) {
            put32(buf, (uint32_t)e.child[0]); put32(buf, (uint32_t)e.child[1]); put32(buf, (uint32_t)e.child[2]);
            put32(buf, e.some ? (uint32_t)e.pts.size() : 0u);
            if (e.some) buf.append(reinterpret_cast<const char*>(e.pts.data()), 16ull * e.pts.size());
        }
        const std::string hd = dir + "/h_" + std::to_string(f.h);
        if (mkdir(hd.c_str(), 0755) != 0 && errno != EEXIST) { err = "cannot create " + hd; return -EIO; }
        char name[96];
        snprintf(name, sizeof name, "/c_%d_%d_%d.bin", f.idx[0], f.idx[1], f.idx[2]);
        const std::string path = hd + name;
        FILE* fp = fopen(path.c_str(), "wb");
        bool ok = fp != nullptr;
        if (ok) { ok = fwrite(buf.data(), 1, buf.size(), fp) == buf.size(); ok = (fclose(fp) == 0) && ok; }
        if (!ok) { err = "cannot write " + path; return -EIO; }
    }
    return 0;
}

unsigned writer_threads() {
    const char* e = getenv("PCC_WRITE_THREADS");
    if (e && atoi(e) > 0) return (unsigned)atoi(e);
    return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

int write_output(const std::string& dir, const Metadata& meta, const std::vector<LevelHost>& levels,
                 const std::vector<Point>& grid, const std::vector<Point>& kept, std::string& err, bool with_metadata) {
    int rc = make_output_dirs(dir, meta.hierarchies, err);
    if (rc) return rc;
    for (const LevelHost& L : levels) {
        rc = write_level_cells(dir, meta.config, L, grid.data(), kept.data(), writer_threads(), err);
        if (rc) return rc;
    }
    return with_metadata ? write_metadata(dir, meta, err) : 0;
}

int write_metadata(const std::string& dir, const Metadata& meta, std::string& err) {
    const std::string mp = dir + "/metadata.json";
    FILE* f = fopen(mp.c_str(), "wb");
    if (!f) { err = "cannot write " + mp; return -errno; }
    const std::string js = metadata_json(meta);
    const bool ok = fwrite(js.data(), 1, js.size(), f) == js.size();
    if (fclose(f) != 0 || !ok) { err = "write failed: " + mp; return -EIO; }
    return 0;
}

// ------------------------------------------------------------------ existing cloud
bool read_cell_file(const std::string& path, CellFile& out, std::string& err) {
    // header, grid points straight into the cell's array, then the overflow
    // entries (cell.rs:183-229): no zero fill, no intermediate copy
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) { err = "cannot open " + path; return false; }
    struct stat sb;
    if (fstat(fd, &sb) != 0) { close(fd); err = "cannot stat " + path; return false; }
    const uint64_t size = (uint64_t)sb.st_size;
    auto rd = [&](void* dst, uint64_t n) {
        uint64_t got = 0;
        while (got < n) {
            const ssize_t r = read(fd, static_cast<char*>(dst) + got, n - got);
            if (r <= 0) return false;
            got += (uint64_t)r;
        }
        return true;
    };
    auto bad = [&](const char* what) { close(fd); err = path + ": " + what; return false; };
    char hb[48];
    if (size < 49 || !rd(hb, 48)) return bad("truncated header");
    auto u32 = [](const char* q) { uint32_t v; memcpy(&v, q, 4); return v; };
    auto i32 = [](const char* q) { int32_t v; memcpy(&v, q, 4); return v; };
    out.h = u32(hb);
    out.idx[0] = i32(hb + 4); out.idx[1] = i32(hb + 8); out.idx[2] = i32(hb + 12);
    out.total = u32(hb + 16); out.number = u32(hb + 20); out.overflow = u32(hb + 24);
    if (48 + 16ull * out.number + 1 > size) return bad("truncated grid");
    out.grid.resize(out.number);
    if (out.number && !rd(out.grid.data(), 16ull * out.number)) return bad("truncated grid");
    HostVec<char> tb(size - 48 - 16ull * out.number);
    if (!rd(tb.data(), tb.size())) return bad("truncated overflow entries");
    close(fd);
    const char* p = tb.data();
    const uint64_t len = tb.size();
    auto bad2 = [&](const char* what) { err = path + ": " + what; return false; };
    uint64_t off = 0;
    const uint32_t nb = (uint8_t)p[off++];
    if (nb > 8) return bad2("more than 8 overflow entries");
    out.entries.clear();
    for (uint32_t j = 0; j < nb; j++) {
        if (off + 16 > len) return bad2("truncated overflow entry");
        CellFile::Entry e;
        e.child[0] = i32(p + off); e.child[1] = i32(p + off + 4); e.child[2] = i32(p + off + 8);
        const uint32_t n = u32(p + off + 12);
        off += 16;
        e.some = n != 0;
        if (off + 16ull * n > len) return bad2("truncated overflow list");
        e.pts.resize(n);
        if (n) memcpy(e.pts.data(), p + off, 16ull * n);
        off += 16ull * n;
        out.entries.push_back(std::move(e));
    }
    if (off != len) return bad2("trailing bytes");
    return true;
}

namespace {
struct CloudFile { std::string path; uint32_t h; int32_t x, y, z; };
// The cell files of a cloud in a fixed order: hierarchy by hierarchy, names
// sorted; optionally only those below the given level-0 cells.
std::vector<CloudFile> list_cloud(const std::string& dir, uint32_t hierarchies, const std::vector<int32_t>* subtrees) {
    // level-0 subtrees to keep (sorted triples); a level-h cell's level-0
    // ancestor is its index >> h (arithmetic: child = 2 * parent + bit)
    std::vector<std::array<int32_t, 3>> keep;
    if (subtrees) {
        for (size_t i = 0; i + 2 < subtrees->size(); i += 3)
            keep.push_back({(*subtrees)[i], (*subtrees)[i + 1], (*subtrees)[i + 2]});
        std::sort(keep.begin(), keep.end());
    }
    std::vector<CloudFile> want;
    for (uint32_t h = 0; h < hierarchies; h++) {
        const std::string hd = dir + "/h_" + std::to_string(h);
        DIR* d = opendir(hd.c_str());
        if (!d) continue;   // converter.rs:187-207: a missing file is a new cell
        std::vector<std::string> names;
        while (dirent* e = readdir(d)) names.push_back(e->d_name);
        closedir(d);
        std::sort(names.begin(), names.end());
        for (const std::string& nm : names) {
            int x, y, z;
            char tail[8] = {0};
            if (sscanf(nm.c_str(), "c_%d_%d_%d.%3s", &x, &y, &z, tail) != 4 || strcmp(tail, "bin") != 0) continue;
            if (subtrees && !std::binary_search(keep.begin(), keep.end(), std::array<int32_t, 3>{x >> h, y >> h, z >> h}))
                continue;
            want.push_back({hd + "/" + nm, h, x, y, z});
        }
    }
    return want;
}
// files want[i0 .. i1) into cells[0 .. i1 - i0), in parallel (the writer's pool size)
bool read_cloud_files(const std::vector<CloudFile>& want, size_t i0, size_t i1, std::vector<CellFile>& cells,
                      std::string& err) {
    cells.resize(i1 - i0);
    std::atomic<size_t> next{i0};
    std::atomic<bool> failed{false};
    std::mutex em;
    auto work = [&]() {
        std::string e;
        for (;;) {
            const size_t i = next.fetch_add(1);
            if (i >= i1 || failed.load()) return;
            const CloudFile& w = want[i];
            CellFile& c = cells[i - i0];
            bool ok = read_cell_file(w.path, c, e);
            if (ok && (c.h != w.h || c.idx[0] != w.x || c.idx[1] != w.y || c.idx[2] != w.z)) {
                e = w.path + ": header does not match the file name";
                ok = false;
            }
            if (!ok) {
                std::lock_guard<std::mutex> g(em);
                if (!failed.exchange(true)) err = e;
                return;
            }
        }
    };
    const unsigned nt = std::max(1u, std::min<unsigned>(writer_threads(), (unsigned)(i1 - i0)));
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    return !failed.load();
}
}  // namespace

int read_cloud(const std::string& dir, uint32_t hierarchies, std::vector<CellFile>& cells, std::string& err,
               const std::vector<int32_t>* subtrees) {
    cells.clear();
    const std::vector<CloudFile> want = list_cloud(dir, hierarchies, subtrees);
    if (!read_cloud_files(want, 0, want.size(), cells, err)) {
        cells.clear();
        return -EINVAL;
    }
    return 0;
}

// The existing cloud as the engine's merge state (engine.h PriorState).  Keys
// follow the reference's order of precedence (all existing points before any
// new one); per level h: every cell's grid points, then every kept list in
// stored order.  Cells are taken in (x, y, z) order.  The per-slab grouping of
// levels >= 1 (hex layer trunc(z / r_h), hex.rs:83) and each seed's child slab
// at h+1 (metadata.rs:100-102, hex.rs:83) use the build's own f32 formulas.
int prior_from_cells(const std::vector<CellFile>& cells, const Config& cfg, PriorState& out, std::string& err) {
    uint32_t levels = 0;
    for (const CellFile& c : cells) levels = std::max(levels, c.h + 1);
    out = PriorState();
    out.forced_lo.assign(levels, 0);
    out.levels.assign(levels, PriorLevel());
    std::vector<std::vector<const CellFile*>> by(levels);
    for (const CellFile& c : cells) by[c.h].push_back(&c);
    for (auto& v : by)
        std::sort(v.begin(), v.end(), [](const CellFile* a, const CellFile* b) {
            return a->idx[0] != b->idx[0] ? a->idx[0] < b->idx[0] : (a->idx[1] != b->idx[1] ? a->idx[1] < b->idx[1] : a->idx[2] < b->idx[2]);
        });
    // keys and per-cell offsets
    struct CellPlan { uint64_t gkey = 0, kkey = 0, inj_off = 0; std::vector<int32_t> layers; std::vector<PriorSlabRec> recs; };
    std::vector<std::vector<CellPlan>> plan(levels);
    uint64_t key = 0, inj = 0;
    for (uint32_t h = 0; h < levels; h++) {
        plan[h].resize(by[h].size());
        for (size_t i = 0; i < by[h].size(); i++) { plan[h][i].gkey = key; key += by[h][i]->grid.size(); }
        out.forced_lo[h] = key;
        for (size_t i = 0; i < by[h].size(); i++) {
            plan[h][i].kkey = key;
            for (const CellFile::Entry& e : by[h][i]->entries) {
                const int32_t bx = e.child[0] - 2 * by[h][i]->idx[0], by_ = e.child[1] - 2 * by[h][i]->idx[1],
                              bz = e.child[2] - 2 * by[h][i]->idx[2];
                if (((bx | by_ | bz) & ~1) != 0) { err = "overflow entry that is not a child of its cell"; return -EINVAL; }
                if (e.some) key += e.pts.size();
            }
            if (h > 0) { plan[h][i].inj_off = inj; inj += key - plan[h][i].kkey + by[h][i]->grid.size(); }
        }
    }
    if (key >= 0xFFFFFFFFull) { err = "existing cloud has more than 2^32-1 points"; return -EOVERFLOW; }
    out.nseeds = key;
    out.inj.resize(inj);
    out.inj_keys.resize(inj);
    const unsigned nt = std::max(1u, std::min<unsigned>(16, std::thread::hardware_concurrency()));
    auto parallel = [&](auto&& work) {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
    };
    // level-0 seeds in key order (every grid, then every kept list), copied in parallel
    {
        std::vector<std::pair<const Point*, size_t>> parts;
        if (!by.empty()) {
            for (const CellFile* c : by[0]) parts.push_back({c->grid.data(), c->grid.size()});
            for (const CellFile* c : by[0])
                for (const CellFile::Entry& e : c->entries)
                    if (e.some) parts.push_back({e.pts.data(), e.pts.size()});
        }
        std::vector<size_t> at(parts.size() + 1, 0);
        for (size_t i = 0; i < parts.size(); i++) at[i + 1] = at[i] + parts[i].second;
        out.seeds0.resize(at.back());
        std::atomic<size_t> nx{0};
        parallel([&]() {
            for (size_t i; (i = nx.fetch_add(1)) < parts.size();)
                if (parts[i].second) memcpy(out.seeds0.data() + at[i], parts[i].first, parts[i].second * sizeof(Point));
        });
    }
    // per cell (threads): slabs by hex layer, seeds grouped by slab, their child slabs
    std::atomic<int> bad{0};
    std::atomic<bool> any_nan{false};
    std::mutex mx_mu;
    float mx_abs = 0.f;
    for (uint32_t h = 0; h < levels; h++) {
        const float cs = cell_size(cfg.max_cell_size, h), cr = hex_radius(sub_cell_size(cs, cfg.sub_grid_dimension));
        const float csc = cell_size(cfg.max_cell_size, h + 1), crc = hex_radius(sub_cell_size(csc, cfg.sub_grid_dimension));
        std::atomic<size_t> next{0};
        // Per cell: pass 1 takes every seed's hex layer (hex.rs:83) in key order
        // (grid, then the kept lists), pass 2 scatters the seeds into their
        // slab's run of inj (a stable counting sort by layer: both passes read
        // the cell's points in order) and counts each slab's child slabs.
        auto work = [&]() {
            std::vector<int32_t> tl;
            std::vector<uint32_t> cnt, cur;
            std::vector<int32_t> sid;
            for (;;) {
                const size_t i = next.fetch_add(1);
                if (i >= by[h].size()) return;
                const CellFile* c = by[h][i];
                CellPlan& P = plan[h][i];
                std::vector<std::pair<const Point*, size_t>> parts;   // grid, then the kept (Some) lists
                parts.push_back({c->grid.data(), c->grid.size()});
                for (const CellFile::Entry& e : c->entries)
                    if (e.some) parts.push_back({e.pts.data(), e.pts.size()});
                size_t n = 0;
                for (const auto& q : parts) n += q.second;
                tl.resize(n);
                int32_t tmin = INT32_MAX, tmax = INT32_MIN;
                {
                    // also: NaN seeds (the slab kernels' NaN rules) and the largest
                    // finite magnitude (fmax skips NaN; an infinity fails `< inf`)
                    bool nan = false;
                    float m = 0.f;
                    size_t j = 0;
                    for (const auto& q : parts)
                        for (size_t k = 0; k < q.second; k++, j++) {
                            const Point& pt = q.first[k];
                            tl[j] = sat_i32(pt.z / cr);   // hex.rs:83
                            tmin = std::min(tmin, tl[j]);
                            tmax = std::max(tmax, tl[j]);
                            nan |= (pt.x != pt.x) | (pt.y != pt.y) | (pt.z != pt.z);
                            const float a = std::fmax(std::fmax(std::fabs(pt.x), std::fabs(pt.y)), std::fabs(pt.z));
                            m = a < INFINITY ? std::fmax(m, a) : m;
                        }
                    if (nan) any_nan.store(true);
                    if (n) {
                        std::lock_guard<std::mutex> lk(mx_mu);
                        mx_abs = std::max(mx_abs, m);
                    }
                }
                if (n == 0) continue;
                if ((int64_t)tmax - tmin >= (1 << 20)) { bad.store(2); continue; }   // not one cell's layers
                const size_t nt_ = (size_t)(tmax - tmin) + 1;
                cnt.assign(nt_, 0);
                for (size_t j = 0; j < n; j++) cnt[(size_t)(tl[j] - tmin)]++;
                // one record per occupied layer, in layer order; seeds at w0 + exclusive scan
                sid.assign(nt_, -1);
                cur.assign(nt_, 0);
                uint64_t w = P.inj_off;
                for (size_t t = 0; t < nt_; t++) {
                    if (!cnt[t]) continue;
                    PriorSlabRec R;
                    R.seed_off = (uint32_t)w;
                    R.nseed = cnt[t];
                    R.ngrid = 0;
                    R.pad = 0;
                    for (int d = 0; d < 24; d++) { R.child[d] = kNoPriorSlab; R.dcap[d] = 0; }
                    sid[t] = (int32_t)P.recs.size();
                    cur[t] = (uint32_t)(w - P.inj_off);
                    P.layers.push_back(tmin + (int32_t)t);
                    P.recs.push_back(R);
                    w += cnt[t];
                }
                size_t j = 0;
                uint64_t key = P.gkey;
                for (size_t pi = 0; pi < parts.size(); pi++) {
                    if (pi == 1) key = P.kkey;   // kept seeds follow every grid seed of the level
                    for (size_t k = 0; k < parts[pi].second; k++, j++, key++) {
                        const Point* q = &parts[pi].first[k];
                        const size_t tt = (size_t)(tl[j] - tmin);
                        const int32_t t = tl[j];
                        PriorSlabRec& R = P.recs[(size_t)sid[tt]];
                        if (pi == 0) R.ngrid++;   // grid seeds precede the kept ones in every slab (key order)
                        const int32_t bx = cell_index1(q->x, csc) - 2 * c->idx[0], by_ = cell_index1(q->y, csc) - 2 * c->idx[1],
                                      bz = cell_index1(q->z, csc) - 2 * c->idx[2];
                        const int32_t sel = sat_i32(q->z / crc) - 2 * t + 1;
                        if (((bx | by_ | bz) & ~1) != 0 || sel < 0 || sel > 2) {
                            if (h + 1 < 31) bad.store(1);   // routes only matter if the child level can exist
                        } else {
                            R.dcap[(bx | (by_ << 1) | (bz << 2)) * 3 + sel]++;
                        }
                        if (h > 0) {
                            const uint64_t o = P.inj_off + cur[tt]++;
                            out.inj[o] = *q;
                            out.inj_keys[o] = (uint32_t)key;
                        }
                    }
                }
            }
        };
        parallel(work);
        PriorLevel& L = out.levels[h];
        L.cell_slab0.push_back(0);
        for (size_t i = 0; i < by[h].size(); i++) {
            const CellFile* c = by[h][i];
            PriorCell pc{c->idx[0], c->idx[1], c->idx[2], 0u};
            for (const CellFile::Entry& e : c->entries) {
                const int oct = (e.child[0] - 2 * c->idx[0]) | ((e.child[1] - 2 * c->idx[1]) << 1) | ((e.child[2] - 2 * c->idx[2]) << 2);
                pc.st |= (e.some ? 1u : 2u) << (2 * oct);
            }
            L.cells.push_back(pc);
            L.slab_layer.insert(L.slab_layer.end(), plan[h][i].layers.begin(), plan[h][i].layers.end());
            L.slabs.insert(L.slabs.end(), plan[h][i].recs.begin(), plan[h][i].recs.end());
            L.cell_slab0.push_back((uint32_t)L.slabs.size());
            std::vector<int32_t>().swap(plan[h][i].layers);
            std::vector<PriorSlabRec>().swap(plan[h][i].recs);
        }
    }
    out.has_nan = any_nan.load();
    out.max_abs = mx_abs;
    if (bad.load() == 2) { err = "existing cloud: a cell's points span more hex layers than a cell has"; return -EINVAL; }
    if (bad.load()) { err = "existing cloud: a point lies outside its cell's child slabs"; return -EINVAL; }
    // child links: slab (c, t), destination (octant, sel) -> record of (2c + octant bits, 2t - 1 + sel) at h+1
    for (uint32_t h = 0; h + 1 < levels; h++) {
        const PriorLevel& N = out.levels[h + 1];
        PriorLevel& L = out.levels[h];
        for (size_t i = 0; i < L.cells.size(); i++) {
            const PriorCell& c = L.cells[i];
            for (uint32_t s = L.cell_slab0[i]; s < L.cell_slab0[i + 1]; s++) {
                const int32_t t = L.slab_layer[s];
                for (int oct = 0; oct < 8; oct++) {
                    if (((c.st >> (2 * oct)) & 3u) != 2u) continue;   // only a None bucket has a child cell
                    const PriorCell key{2 * c.x + (oct & 1), 2 * c.y + ((oct >> 1) & 1), 2 * c.z + ((oct >> 2) & 1), 0};
                    auto it = std::lower_bound(N.cells.begin(), N.cells.end(), key, [](const PriorCell& a, const PriorCell& b) {
                        return a.x != b.x ? a.x < b.x : (a.y != b.y ? a.y < b.y : a.z < b.z);
                    });
                    if (it == N.cells.end() || it->x != key.x || it->y != key.y || it->z != key.z) continue;
                    const size_t ci = (size_t)(it - N.cells.begin());
                    for (int sel = 0; sel < 3; sel++) {
                        const int32_t u = 2 * t - 1 + sel;
                        if (u / 2 != t) continue;   // a child layer has one parent layer
                        const auto b0 = N.slab_layer.begin() + N.cell_slab0[ci], b1 = N.slab_layer.begin() + N.cell_slab0[ci + 1];
                        const auto jt = std::lower_bound(b0, b1, u);
                        if (jt != b1 && *jt == u) L.slabs[s].child[oct * 3 + sel] = (uint32_t)(jt - N.slab_layer.begin());
                    }
                }
            }
        }
    }
    return 0;
}

// ------------------------------------------------------------------ LAS
bool read_las(const std::string& path, LasResult& out, std::string& err, const PointSink& sink) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    uint8_t h[375] = {0};
    const size_t got = fread(h, 1, sizeof h, f);
    auto bad = [&](const std::string& what) { err = path + ": " + what; fclose(f); return false; };
    if (got < 227 || memcmp(h, "LASF", 4) != 0) return bad("not a LAS file");
    auto u16 = [&](size_t o) { uint16_t v; memcpy(&v, h + o, 2); return v; };
    auto u32 = [&](size_t o) { uint32_t v; memcpy(&v, h + o, 4); return v; };
    auto u64 = [&](size_t o) { uint64_t v; memcpy(&v, h + o, 8); return v; };
    auto f64 = [&](size_t o) { double v; memcpy(&v, h + o, 8); return v; };
    const uint8_t minor = h[25];
    const uint16_t hsize = u16(94);
    const uint32_t data_off = u32(96);
    const uint8_t fmt_raw = h[104];
    const uint16_t rec = u16(105);
    uint64_t n = u32(107);
    if (minor >= 4 && hsize >= 375 && got >= 255) n = u64(247);   // LAS 1.4 64-bit count
    out.count = n;
    out.points.clear();
    const uint8_t fmt = fmt_raw & 0x3F;
    // LAZ (las.rs:14-46 through las + laz [dep]): bit 7 of the format marks
    // compressed point data, described by the LASzip VLR
    laz::Reader lz;
    const bool compressed = (fmt_raw & 0x80) != 0;
    if (compressed) {
        out.laz = true;
        const uint32_t nvlr = u32(100);
        laz::Vlr lv;
        bool found = false;
        long pos = hsize;
        for (uint32_t i = 0; i < nvlr && !found; i++) {
            uint8_t vh[54];
            if (fseek(f, pos, SEEK_SET) != 0 || fread(vh, 1, 54, f) != 54) return bad("truncated VLR");
            uint16_t rid, len;
            memcpy(&rid, vh + 18, 2);
            memcpy(&len, vh + 20, 2);
            if (memcmp(vh + 2, "laszip encoded", 14) == 0 && rid == 22204) {
                std::vector<uint8_t> d(len);
                if (fread(d.data(), 1, len, f) != len) return bad("truncated LASzip VLR");
                std::string e;
                if (!laz::parse_vlr(d.data(), d.size(), lv, e)) return bad(e);
                found = true;
            }
            pos += 54 + len;
        }
        if (!found) return bad("compressed point data without a LASzip VLR");
        std::string e;
        const bool supported = fmt <= 10;
        if (!supported || !lz.open(f, data_off, n, rec, lv, e)) {
            out.laz_error = path + ": " + (!supported ? "LAZ point format " + std::to_string(fmt) +
                                                            " is not supported" : e);
            fclose(f);
            return true;
        }
    }
    if (fmt > 10) return bad("unsupported point data format " + std::to_string(fmt));
    static const int kColorOff[11] = {-1, -1, 20, 28, -1, 28, -1, 30, 30, -1, 30};
    static const int kMinLen[11] = {20, 28, 26, 34, 57, 63, 30, 36, 38, 59, 67};
    if (rec < kMinLen[fmt]) return bad("point record shorter than its format");
    const double sx = f64(131), sy = f64(139), sz = f64(147);
    const double ox = f64(155), oy = f64(163), oz = f64(171);
    const int co = kColorOff[fmt];
    if (!compressed && fseek(f, (long)data_off, SEEK_SET) != 0) return bad("bad offset to point data");
    if (!sink) out.points.resize(n);
    std::vector<uint8_t> buf;
    const uint64_t chunk = 1 << 18;
    buf.resize(chunk * rec);
    std::vector<Point> piece(sink ? chunk : 0);
    for (uint64_t base = 0; base < n; base += chunk) {
        uint64_t m = std::min<uint64_t>(chunk, n - base);
        std::string lerr;
        const uint64_t got_m = compressed ? lz.read(buf.data(), m, lerr) : fread(buf.data(), rec, m, f);
        if (got_m != m) {   // las Reader::read_n fails on the missing records (las.rs:23-46)
            out.data_error = path + ": " + (compressed ? lerr : std::string("truncated point data"));
            m = got_m;
            if (!sink) out.points.resize(base + m);
        }
        Point* dst = sink ? piece.data() : out.points.data() + base;
        for (uint64_t i = 0; i < m; i++) {
            const uint8_t* r = buf.data() + i * rec;
            int32_t X, Y, Z;
            memcpy(&X, r, 4); memcpy(&Y, r + 4, 4); memcpy(&Z, r + 8, 4);
            Point& p = dst[i];
            // las Transform::direct: scale * n + offset in f64 (no FMA), then `as f32`
            p.x = (float)((sx * (double)X) + ox);
            p.y = (float)((sy * (double)Y) + oy);
            p.z = (float)((sz * (double)Z) + oz);
            uint16_t c[3] = {0, 0, 0};
            if (co >= 0) memcpy(c, r + co, 6);
            p.rgba[0] = (uint8_t)c[0];   // las.rs:40 `color.red as u8`
            p.rgba[1] = (uint8_t)c[1];
            p.rgba[2] = (uint8_t)c[2];
            p.rgba[3] = 255;
        }
        if (sink && m && !sink(piece.data(), m)) break;
        if (!out.data_error.empty()) break;
    }
    fclose(f);
    return true;
}

int read_cloud_points(const std::string& metadata_path, uint64_t& number_of_points, const PointSink& sink,
                      std::string& err) {
    std::ifstream f(metadata_path);
    if (!f) { err = "cannot open " + metadata_path; return -ENOENT; }
    std::stringstream ss;
    ss << f.rdbuf();
    Metadata m;
    if (!parse_metadata_json(ss.str(), m, err)) return -EINVAL;   // own.rs:57-60
    number_of_points = m.number_of_points;
    const size_t slash = metadata_path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? "." : metadata_path.substr(0, slash);
    // own.rs:16-78 hands out the cloud's points cell by cell; here windows of
    // cell files are read in parallel and their points handed to the sink in
    // the fixed order (Cell::all_points cell.rs:66-68: grid, then the kept
    // lists), so at most one window is in host memory
    const std::vector<CloudFile> want = list_cloud(dir, m.hierarchies, nullptr);
    constexpr size_t kWindow = 64;
    std::vector<CellFile> cells;
    for (size_t i0 = 0; i0 < want.size(); i0 += kWindow) {
        const size_t i1 = std::min(want.size(), i0 + kWindow);
        if (!read_cloud_files(want, i0, i1, cells, err)) return -EINVAL;
        for (const CellFile& c : cells) {
            if (!c.grid.empty() && !sink(c.grid.data(), c.grid.size())) return -ECANCELED;
            for (const CellFile::Entry& e : c.entries)
                if (e.some && !e.pts.empty() && !sink(e.pts.data(), e.pts.size())) return -ECANCELED;
        }
    }
    return 0;
}

// ------------------------------------------------------------------ PLY
namespace {
enum PType { P_I8, P_U8, P_I16, P_U16, P_I32, P_U32, P_F32, P_F64, P_BAD };
PType ptype(const std::string& t) {
    if (t == "char" || t == "int8") return P_I8;
    if (t == "uchar" || t == "uint8") return P_U8;
    if (t == "short" || t == "int16") return P_I16;
    if (t == "ushort" || t == "uint16") return P_U16;
    if (t == "int" || t == "int32") return P_I32;
    if (t == "uint" || t == "uint32") return P_U32;
    if (t == "float" || t == "float32") return P_F32;
    if (t == "double" || t == "float64") return P_F64;
    return P_BAD;
}
int psize(PType t) {
    static const int s[] = {1, 1, 2, 2, 4, 4, 4, 8, 0};
    return s[t];
}
struct Prop {
    std::string name;
    PType type;
    bool list = false;
    PType count_type = P_U8;
};
template <class T>
T rd(const uint8_t* p, bool swap) {
    T v;
    uint8_t b[sizeof(T)];
    memcpy(b, p, sizeof(T));
    if (swap) std::reverse(b, b + sizeof(T));
    memcpy(&v, b, sizeof(T));
    return v;
}
double rdnum(const uint8_t* p, PType t, bool sw) {
    switch (t) {
        case P_I8: return (double)(int8_t)p[0];
        case P_U8: return (double)p[0];
        case P_I16: return rd<int16_t>(p, sw);
        case P_U16: return rd<uint16_t>(p, sw);
        case P_I32: return rd<int32_t>(p, sw);
        case P_U32: return rd<uint32_t>(p, sw);
        case P_F32: return rd<float>(p, sw);
        case P_F64: return rd<double>(p, sw);
        default: return 0;
    }
}
// Rust `f32 as u8`: saturating, NaN -> 0
uint8_t sat_u8(float v) {
    if (!(v == v)) return 0;
    if (v <= 0.0f) return 0;
    if (v >= 255.0f) return 255;
    return (uint8_t)v;
}
}  // namespace

bool read_ply(const std::string& path, PlyResult& out, std::string& err, const PointSink& sink) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { err = "cannot open " + path; return false; }
    std::string line;
    if (!std::getline(f, line) || line.rfind("ply", 0) != 0) { err = path + ": not a PLY file"; return false; }
    enum { ASCII, LE, BE } enc = LE;
    std::vector<Prop> vprops;
    // ply.rs:36-73 reads `vertex` records straight after the header, whatever
    // elements the header declares before it (their bytes are read as vertices)
    bool in_vertex = false, seen_vertex = false;
    uint64_t nvert = 0;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ls(line);
        std::string kw;
        ls >> kw;
        if (kw == "format") {
            std::string e;
            ls >> e;
            enc = e == "ascii" ? ASCII : e == "binary_big_endian" ? BE : LE;
            if (e != "ascii" && e != "binary_big_endian" && e != "binary_little_endian") { err = "bad PLY format " + e; return false; }
        } else if (kw == "element") {
            std::string name;
            uint64_t cnt;
            ls >> name >> cnt;
            in_vertex = name == "vertex";
            if (in_vertex) { nvert = cnt; seen_vertex = true; }
        } else if (kw == "property" && in_vertex) {
            std::string t;
            ls >> t;
            Prop p;
            if (t == "list") {
                std::string ct, it;
                ls >> ct >> it >> p.name;
                p.list = true;
                p.count_type = ptype(ct);
                p.type = ptype(it);
            } else {
                ls >> p.name;
                p.type = ptype(t);
            }
            if (p.type == P_BAD || p.count_type == P_BAD) { err = "unsupported PLY property type in " + line; return false; }
            vprops.push_back(p);
        } else if (kw == "end_header") {
            break;
        }
    }
    if (!seen_vertex) { err = path + ": no vertex element"; return false; }   // ply.rs:37 unwraps this
    out.vertex_count = nvert;
    out.points.clear();
    if (enc == ASCII) {   // ply.rs:43-51: lines are parsed but never pushed into the batch
        out.ascii = true;
        // a missing line makes read_ascii_element fail (ply.rs:46-47): count the lines present
        uint64_t lines = 0;
        while (lines < nvert && std::getline(f, line)) lines++;
        out.ascii_lines = lines;
        if (lines < nvert) out.data_error = path + ": truncated ASCII vertex data";
        return true;
    }
    const bool sw = enc == BE;
    // fixed-size records: each property compiled once to (target, type, offset)
    bool fixed = true;
    int rec = 0;
    for (auto& p : vprops) { if (p.list) fixed = false; rec += psize(p.type); }
    // point.rs:61-130 property names -> target: 0..2 x/y/z, 3..6 red/green/blue/alpha, -1 ignored
    auto target = [](const std::string& nm) {
        if (nm == "x") return 0;
        if (nm == "y") return 1;
        if (nm == "z") return 2;
        if (nm == "red" || nm == "r") return 3;
        if (nm == "green" || nm == "g") return 4;
        if (nm == "blue" || nm == "b") return 5;
        if (nm == "alpha" || nm == "a") return 6;
        return -1;
    };
    auto apply = [&](Point& pt, int tg, PType ty, const uint8_t* q) {
        if (tg < 0) return;
        if (tg < 3) {
            float v;
            if (ty == P_F32) v = rd<float>(q, sw);
            else if (ty == P_F64) v = (float)rd<double>(q, sw);
            else return;
            (tg == 0 ? pt.x : tg == 1 ? pt.y : pt.z) = v;
        } else {
            if (ty == P_U8) pt.rgba[tg - 3] = q[0];
            else if (ty == P_F32) pt.rgba[tg - 3] = sat_u8(rd<float>(q, sw) / 255.0f);
        }
    };
    const uint64_t chunk = 1 << 18;
    std::vector<Point> piece;
    auto emit = [&](const Point* pts, uint64_t m, uint64_t base) -> bool {
        if (sink) return sink(pts, m);
        std::memcpy(out.points.data() + base, pts, m * sizeof(Point));
        return true;
    };
    if (!sink) out.points.resize(nvert);
    if (fixed) {
        struct Op { int tg; PType ty; int off; };
        std::vector<Op> ops;
        int off = 0;
        for (auto& p : vprops) { ops.push_back({target(p.name), p.type, off}); off += psize(p.type); }
        // the on-disk Point itself (float x, y, z; uchar red, green, blue, alpha; LE): a plain copy
        const bool raw = !sw && rec == 16 && ops.size() == 7 && ops[0].tg == 0 && ops[0].ty == P_F32 &&
                         ops[1].tg == 1 && ops[1].ty == P_F32 && ops[2].tg == 2 && ops[2].ty == P_F32 &&
                         ops[3].tg == 3 && ops[3].ty == P_U8 && ops[4].tg == 4 && ops[4].ty == P_U8 &&
                         ops[5].tg == 5 && ops[5].ty == P_U8 && ops[6].tg == 6 && ops[6].ty == P_U8;
        std::vector<uint8_t> buf(chunk * rec);
        piece.resize(chunk);
        for (uint64_t base = 0; base < nvert; base += chunk) {
            const uint64_t m = std::min(chunk, nvert - base);
            f.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(m * rec));
            const uint64_t got_m = (uint64_t)f.gcount() / rec;
            const bool short_read = got_m != m;
            if (short_read) {   // read_*_endian_element fails on the first missing record (ply.rs:54-70)
                out.data_error = path + ": truncated vertex data";
                if (!sink) out.points.resize(base + got_m);
            }
            if (raw) {
                if (!emit(reinterpret_cast<const Point*>(buf.data()), got_m, base)) return true;
            } else {
                for (uint64_t i = 0; i < got_m; i++) {
                    Point& pt = piece[i];
                    pt.x = pt.y = pt.z = 0;
                    pt.rgba[0] = pt.rgba[1] = pt.rgba[2] = 0;
                    pt.rgba[3] = 255;   // point.rs:16-23
                    const uint8_t* q = buf.data() + i * rec;
                    for (const Op& op : ops) apply(pt, op.tg, op.ty, q + op.off);
                }
                if (!emit(piece.data(), got_m, base)) return true;
            }
            if (short_read) break;
        }
    } else {   // list properties: record by record
        std::vector<int> tgs;
        for (auto& p : vprops) tgs.push_back(target(p.name));
        piece.resize(chunk);
        uint64_t k = 0, base = 0;
        for (uint64_t i = 0; i < nvert; i++) {
            Point& pt = piece[k];
            pt.x = pt.y = pt.z = 0;
            pt.rgba[0] = pt.rgba[1] = pt.rgba[2] = 0;
            pt.rgba[3] = 255;
            for (size_t pi = 0; pi < vprops.size(); pi++) {
                const Prop& p = vprops[pi];
                uint8_t tmp[8];
                if (p.list) {
                    f.read(reinterpret_cast<char*>(tmp), psize(p.count_type));
                    const uint64_t cnt = (uint64_t)rdnum(tmp, p.count_type, sw);
                    f.seekg((std::streamoff)(cnt * psize(p.type)), std::ios::cur);
                } else {
                    f.read(reinterpret_cast<char*>(tmp), psize(p.type));
                    apply(pt, tgs[pi], p.type, tmp);
                }
                if (!f) {
                    out.data_error = path + ": truncated vertex data";
                    if (!sink) out.points.resize(base + k);
                    if (k) emit(piece.data(), k, base);
                    return true;
                }
            }
            if (++k == chunk) {
                if (!emit(piece.data(), k, base)) return true;
                base += k;
                k = 0;
            }
        }
        if (k) emit(piece.data(), k, base);
    }
    return true;
}

}  // namespace pcc
