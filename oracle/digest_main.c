/*
 * digest_main.c — TEST INFRASTRUCTURE ONLY.  Runs the sequential oracle
 * (pcc_oracle.c) over one part of a full-size synthetic configuration and
 * prints canonical per-level-0-subtree digests (digest.c) as JSON lines; driven
 * by tests/golden/make_large_digests.py, which commits the results as fixtures.
 *
 * Level-0 subtrees are independent (every level-h cell has a unique level-0
 * ancestor, converter.rs:32-47, 114-139), so a part converts only the points of
 * its own level-0 cells, keeping the GLOBAL batch structure (lib.rs:31-52): each
 * 10 000-point batch of the stream is filtered to the part's cells and added as
 * one batch (an empty filtered batch leaves these cells untouched, as in the
 * reference where that batch's points go to other cells).
 *
 *   orc_digest PART PARTS SEED KIND N [SEED2 KIND2 N2]
 * Stream 1 = N points of synthetic kind KIND (seed SEED) in [-1000,1000)^3, one
 * file; optional stream 2 = a second file converted afterwards (incremental
 * merge, config 5: converting A then B into one directory == one run over A, B).
 * After each stream: one JSON line per subtree of this part, then a summary line.
 */
#include <inttypes.h>
#include <math.h>
#include <time.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "digest.h"

typedef struct { float x, y, z; uint8_t rgba[4]; } pt;
typedef struct { uint32_t cell_point_overflow_limit, sub_grid_dimension; float max_cell_size; } cfg_t;
typedef struct orc_conv orc_conv;
orc_conv* orc_new(const cfg_t* cfg);
void orc_free(orc_conv* c);
void orc_add_batch(orc_conv* c, const pt* p, uint64_t n);
void orc_synth(uint64_t seed, int kind, uint64_t first, uint64_t n, float lo, float ext, pt* out);
void orc_digest(const orc_conv* c, dg_acc* acc);
int orc_error(const orc_conv* c);
uint64_t orc_arrivals(const orc_conv* c);
uint32_t orc_hierarchies(const orc_conv* c);

static int part_of(const pt* p, int parts) {   /* metadata.rs:100-102 at h = 0 (cell size 1000) */
    const int32_t ix = (int32_t)floorf(p->x / 1000.0f), iy = (int32_t)floorf(p->y / 1000.0f),
                  iz = (int32_t)floorf(p->z / 1000.0f);
    return ((ix & 1) | ((iy & 1) << 1) | ((iz & 1) << 2)) % parts;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
static double g_convert_s = 0;   /* time inside orc_add_batch only (the generator is not timed) */

static void report(orc_conv* c, int phase, const float bb[6], uint64_t npts) {
    dg_acc* acc = dg_new();
    orc_digest(c, acc);
    const uint64_t n = dg_count(acc);
    for (uint64_t i = 0; i < n; i++) {
        int64_t a[4];
        uint64_t u[4];
        dg_get(acc, i, a, u);
        printf("{\"phase\": %d, \"subtree\": [%" PRId64 ", %" PRId64 ", %" PRId64 "], \"levels\": %" PRId64
               ", \"cells\": %" PRIu64 ", \"points\": %" PRIu64 ", \"W\": %" PRIu64 ", \"digest\": \"%016" PRIx64 "\"}\n",
               phase, a[0], a[1], a[2], a[3], u[0], u[1], u[2], u[3]);
    }
    uint64_t t[2];
    dg_totals(acc, t);
    uint32_t b[6];
    memcpy(b, bb, sizeof b);
    printf("{\"phase\": %d, \"summary\": true, \"input_points\": %" PRIu64 ", \"arrivals\": %" PRIu64
           ", \"grid_points\": %" PRIu64 ", \"kept_points\": %" PRIu64 ", \"error\": %d, \"bbox_bits\": [%u, %u, %u, %u, %u, %u]"
           ", \"convert_seconds\": %.3f}\n",
           phase, npts, orc_arrivals(c), t[0], t[1], orc_error(c), b[0], b[1], b[2], b[3], b[4], b[5], g_convert_s);
    fflush(stdout);
    dg_free(acc);
}

int main(int argc, char** argv) {
    if (argc != 6 && argc != 9) {
        fprintf(stderr, "usage: %s PART PARTS SEED KIND N [SEED2 KIND2 N2]\n", argv[0]);
        return 2;
    }
    const int part = atoi(argv[1]), parts = atoi(argv[2]);
    const cfg_t cfg = {5000, 96, 1000.0f};   /* MetadataConfig::default, metadata.rs:80-88 */
    orc_conv* c = orc_new(&cfg);
    const uint32_t B = 10000;                /* lib.rs:32 */
    pt* buf = (pt*)malloc(B * sizeof(pt));
    pt* sel = (pt*)malloc(B * sizeof(pt));
    float bb[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    uint64_t total = 0;
    const int streams = argc == 9 ? 2 : 1;
    for (int s = 0; s < streams; s++) {
        const uint64_t seed = strtoull(argv[3 + 3 * s], NULL, 10);
        const int kind = atoi(argv[4 + 3 * s]);
        const uint64_t n = strtoull(argv[5 + 3 * s], NULL, 10);
        for (uint64_t off = 0; off < n; off += B) {
            const uint64_t m = n - off < B ? n - off : B;
            orc_synth(seed, kind, off, m, -1000.0f, 2000.0f, buf);
            uint64_t k = 0;
            for (uint64_t i = 0; i < m; i++) {
                const float v[3] = {buf[i].x, buf[i].y, buf[i].z};
                for (int a = 0; a < 3; a++) { bb[a] = fminf(bb[a], v[a]); bb[3 + a] = fmaxf(bb[3 + a], v[a]); }
                if (part_of(&buf[i], parts) == part) sel[k++] = buf[i];
            }
            const double t0 = now_s();
            orc_add_batch(c, sel, k);
            g_convert_s += now_s() - t0;
        }
        total += n;
        report(c, s + 1, bb, total);
    }
    free(buf);
    free(sel);
    orc_free(c);
    return 0;
}
