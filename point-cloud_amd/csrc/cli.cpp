// cli.cpp — `point_converter` command line, same flags as the reference
// (point-converter/src/main.rs:11-50, clap derive): -o/--output DIR,
// -d/--directories DIRS (repeatable), -f/--files FILES (repeatable).
#include <dirent.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "../../include/pcconv.h"

static void usage(FILE* f) {
    fprintf(f,
            "Point converter will convert your points to a format that the point cloud renderer can use.\n"
            "Currently supported file formats are las/laz and ply and the generated metadata.json.\n\n"
            "Usage: point_converter [OPTIONS]\n\n"
            "Options:\n"
            "  -o, --output <DIR>         Output directory of the converted format.\n"
            "                             Will be created if it doesn't exist.\n"
            "  -d, --directories <DIRS>   Directories with input files to convert.\n"
            "  -f, --files <FILES>        Input files with the points to convert.\n"
            "  -h, --help                 Print help\n"
            "  -V, --version              Print version\n");
}

int main(int argc, char** argv) {
    std::string out;
    std::vector<std::string> dirs, files;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&](const char* name) -> std::string {
            size_t eq = a.find('=');
            if (a.rfind("--", 0) == 0 && eq != std::string::npos) return a.substr(eq + 1);
            if (i + 1 >= argc) {
                fprintf(stderr, "error: a value is required for '%s' but none was supplied\n", name);
                exit(2);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") { usage(stdout); return 0; }
        if (a == "-V" || a == "--version") { printf("point-converter 0.1.0\n"); return 0; }
        if (a == "-o" || a.rfind("--output", 0) == 0) out = val("--output <DIR>");
        else if (a == "-d" || a.rfind("--directories", 0) == 0) dirs.push_back(val("--directories <DIRS>"));
        else if (a == "-f" || a.rfind("--files", 0) == 0) files.push_back(val("--files <FILES>"));
        else {
            fprintf(stderr, "error: unexpected argument '%s' found\n\n", a.c_str());
            usage(stderr);
            return 2;
        }
    }
    // main.rs:32-38: files first, then directory entries (read_dir order)
    for (const auto& d : dirs) {
        DIR* dp = opendir(d.c_str());
        if (!dp) {
            fprintf(stderr, "cannot read directory %s\n", d.c_str());
            return 101;   // the reference unwraps read_dir (panic exit code)
        }
        while (dirent* e = readdir(dp)) {
            if (!strcmp(e->d_name, ".") || !strcmp(e->d_name, "..")) continue;
            files.push_back(d + "/" + e->d_name);
        }
        closedir(dp);
    }
    if (files.empty()) {
        char ts[32];
        std::time_t t = std::time(nullptr);
        std::strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%SZ", std::gmtime(&t));
        fprintf(stderr, "[%s WARN  point_converter] Please provide some files or directories\n", ts);
        return 0;
    }
    if (out.empty()) {
        char cwd[4096];
        out = getcwd(cwd, sizeof cwd) ? cwd : ".";
    }
    std::vector<const char*> p;
    for (auto& f : files) p.push_back(f.c_str());
    pcc_options opt;
    pcc_options_default(&opt);
    int rc = pcc_convert_files(out.c_str(), p.data(), p.size(), &opt);
    if (rc) {
        fprintf(stderr, "point_converter: error %d: %s\n", rc, pcc_last_error());
        return 1;
    }
    return 0;
}
