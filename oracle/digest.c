/*
 * digest.c — TEST INFRASTRUCTURE ONLY.  Canonical digests of converted clouds
 * (SURVEY.md Appendix B.3, §4.4 "sampled digests for >= 100M inputs"), used to
 * compare the HIP build with the oracle at sizes where comparing files is
 * impractical (configs 3-5).  Nothing in the product links or calls this.
 *
 * Canonical form of one cell (what the reference's output determines, cell.rs:
 * 155-181): the header values (h, index, total/number/overflow counts, size,
 * sub_cell_size, pos bits), the MULTISET of grid points (their order inside a
 * file is FxHashMap order, cell.rs:158-160, so it is not part of parity), and the
 * overflow entries sorted by child index, each Some list in STORED order (that
 * order is deterministic: emission order, cell.rs:108-153).
 *
 * Digest of a level-0 subtree = sum mod 2^64 of mix(cell digest) over its cells
 * (order independent), plus its cell count, point count and W = sum over cells of
 * (h + 1) * total_number_of_points.  A level-h cell's level-0
 * ancestor is its index >> h (child index = 2 * parent + bit, converter.rs:32-47).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "digest.h"

uint64_t dg_view_size(void) { return sizeof(dg_view); }

static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t point_hash(const dg_point* p) {
    uint64_t lo, hi;
    memcpy(&lo, p, 8);
    memcpy(&hi, (const char*)p + 8, 8);
    return mix64(mix64(lo ^ 0x5851F42D4C957F2Dull) ^ hi);
}
static uint64_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
#define SEQ(acc, v) ((acc) = mix64((acc) ^ (uint64_t)(v)))

uint64_t dg_cell(const dg_view* v) {
    uint64_t a = 0x243F6A8885A308D3ull;
    SEQ(a, v->hierarchy); SEQ(a, (uint32_t)v->x); SEQ(a, (uint32_t)v->y); SEQ(a, (uint32_t)v->z);
    SEQ(a, v->total); SEQ(a, v->number); SEQ(a, v->overflow);
    SEQ(a, f2u(v->size)); SEQ(a, f2u(v->sub));
    SEQ(a, f2u(v->pos[0])); SEQ(a, f2u(v->pos[1])); SEQ(a, f2u(v->pos[2]));
    uint64_t gsum = 0;   /* multiset of grid points */
    for (uint32_t i = 0; i < v->number; i++) gsum += point_hash(&v->grid[i]);
    SEQ(a, gsum);
    SEQ(a, v->entries);
    int ord[8];
    for (uint32_t e = 0; e < v->entries; e++) ord[e] = (int)e;
    for (uint32_t i = 1; i < v->entries; i++)   /* entries by child index (x, y, z) */
        for (uint32_t j = i; j > 0; j--) {
            const int32_t* p = v->child[ord[j - 1]];
            const int32_t* q = v->child[ord[j]];
            int gt = p[0] != q[0] ? p[0] > q[0] : (p[1] != q[1] ? p[1] > q[1] : p[2] > q[2]);
            if (!gt) break;
            int t = ord[j - 1]; ord[j - 1] = ord[j]; ord[j] = t;
        }
    for (uint32_t k = 0; k < v->entries; k++) {
        const int e = ord[k];
        SEQ(a, (uint32_t)v->child[e][0]); SEQ(a, (uint32_t)v->child[e][1]); SEQ(a, (uint32_t)v->child[e][2]);
        SEQ(a, v->count[e]);
        for (uint32_t i = 0; i < v->count[e]; i++) SEQ(a, point_hash(&v->list[e][i]));
    }
    return a;
}

/* ------------------------------------------------------------------ per-subtree accumulator */
typedef struct { int32_t x, y, z; uint32_t levels; uint64_t cells, points, W, sum; } dg_sub;
struct dg_acc { dg_sub* s; size_t n, cap; uint64_t grid_points, kept_points; };

dg_acc* dg_new(void) { return (dg_acc*)calloc(1, sizeof(dg_acc)); }
void dg_free(dg_acc* a) { if (a) { free(a->s); free(a); } }

static dg_sub* sub_of(dg_acc* a, int32_t x, int32_t y, int32_t z) {
    for (size_t i = 0; i < a->n; i++)
        if (a->s[i].x == x && a->s[i].y == y && a->s[i].z == z) return &a->s[i];
    if (a->n == a->cap) {
        a->cap = a->cap ? 2 * a->cap : 16;
        a->s = (dg_sub*)realloc(a->s, a->cap * sizeof(dg_sub));
    }
    dg_sub* s = &a->s[a->n++];
    memset(s, 0, sizeof *s);
    s->x = x; s->y = y; s->z = z;
    return s;
}

void dg_add_view(dg_acc* a, const dg_view* v) {
    const uint32_t h = v->hierarchy;
    dg_sub* s = sub_of(a, h < 32 ? v->x >> h : 0, h < 32 ? v->y >> h : 0, h < 32 ? v->z >> h : 0);
    s->cells += 1;
    s->points += v->total;
    s->W += (uint64_t)(h + 1) * v->total;
    s->sum += mix64(dg_cell(v) ^ 0xD6E8FEB86659FD93ull);
    if (h + 1 > s->levels) s->levels = h + 1;
    a->grid_points += v->number;
    a->kept_points += v->overflow;
}

static int sub_cmp(const void* p, const void* q) {
    const dg_sub* a = (const dg_sub*)p;
    const dg_sub* b = (const dg_sub*)q;
    if (a->x != b->x) return a->x < b->x ? -1 : 1;
    if (a->y != b->y) return a->y < b->y ? -1 : 1;
    if (a->z != b->z) return a->z < b->z ? -1 : 1;
    return 0;
}
/* subtrees sorted by level-0 index; returns the count */
uint64_t dg_count(dg_acc* a) {
    qsort(a->s, a->n, sizeof(dg_sub), sub_cmp);
    return a->n;
}
/* out: x, y, z, levels as int64, then cells, points, W, digest */
void dg_get(const dg_acc* a, uint64_t i, int64_t out_i[4], uint64_t out_u[4]) {
    const dg_sub* s = &a->s[i];
    out_i[0] = s->x; out_i[1] = s->y; out_i[2] = s->z; out_i[3] = s->levels;
    out_u[0] = s->cells; out_u[1] = s->points; out_u[2] = s->W; out_u[3] = s->sum;
}
void dg_totals(const dg_acc* a, uint64_t out[2]) { out[0] = a->grid_points; out[1] = a->kept_points; }
