/* digest.h — TEST INFRASTRUCTURE ONLY (see digest.c). */
#ifndef ORC_DIGEST_H
#define ORC_DIGEST_H
#include <stdint.h>

typedef struct { float x, y, z; uint8_t rgba[4]; } dg_point;

/* Same layout as the C ABI's pcc_cell_view (include/pcconv.h); restated here so
 * the checker does not include product headers.  tests/ assert the size. */
typedef struct {
    uint32_t hierarchy;
    int32_t x, y, z;
    uint32_t total, number, overflow;
    float size, sub, pos[3];
    const dg_point* grid;
    uint32_t entries;
    int32_t child[8][3];
    uint32_t count[8];
    const dg_point* list[8];
} dg_view;

typedef struct dg_acc dg_acc;
dg_acc* dg_new(void);
void dg_free(dg_acc* a);
void dg_add_view(dg_acc* a, const dg_view* v);
uint64_t dg_count(dg_acc* a);
void dg_get(const dg_acc* a, uint64_t i, int64_t out_i[4], uint64_t out_u[4]);
void dg_totals(const dg_acc* a, uint64_t out[2]);
#endif
