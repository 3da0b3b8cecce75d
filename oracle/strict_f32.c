/*
 * strict_f32.c -- TEST INFRASTRUCTURE ONLY.  Neighbor-set oracle for md::neighbor_searcher
 * (stage_interphase/contact_map.cpp:60-62): every pair (i < j) of points closer than `distance`.
 *
 * The predicate is evaluated exactly as the device kernels evaluate it, so the pair sets are comparable bit
 * for bit.  fp32 engine (gcso_search_neighbors): p = (float)x;  d = p_i - p_j (per axis, fp32);
 * r2 = (dx*dx + dy*dy) + dz*dz (fp32, no contraction);  pair iff r2 < (float)distance * (float)distance.
 * fp64 engine (gcso_search_neighbors64): the same expression in fp64 on x itself, pair iff
 * r2 < distance * distance -- what md::neighbor_searcher's double arithmetic computes (INFERRED: the reference's
 * squared-distance form; -funsafe-math-optimizations there may contract it, which moves only pairs at the cutoff).
 * This file is compiled with -ffp-contract=off and without -funsafe-math-optimizations (oracle/Makefile).
 * Candidate pairs come from a cell grid built in fp64 with a 1e-3 relative margin, so the grid never
 * decides membership; the predicate does.
 */
#include "gcs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static int cmp_pair(const void* a, const void* b)
{
    const uint32_t* p = (const uint32_t*)a;
    const uint32_t* q = (const uint32_t*)b;
    if (p[0] != q[0]) return p[0] < q[0] ? -1 : 1;
    if (p[1] != q[1]) return p[1] < q[1] ? -1 : 1;
    return 0;
}

static inline int strict_pair(const float* p, int64_t i, int64_t j, float rc2)
{
    float dx = p[3 * i] - p[3 * j];
    float dy = p[3 * i + 1] - p[3 * j + 1];
    float dz = p[3 * i + 2] - p[3 * j + 2];
    float xx = dx * dx;
    float yy = dy * dy;
    float zz = dz * dz;
    float r2 = (xx + yy) + zz;
    return r2 < rc2;
}

static inline int strict_pair64(const double* p, int64_t i, int64_t j, double rc2)
{
    double dx = p[3 * i] - p[3 * j];
    double dy = p[3 * i + 1] - p[3 * j + 1];
    double dz = p[3 * i + 2] - p[3 * j + 2];
    double xx = dx * dx;
    double yy = dy * dy;
    double zz = dz * dz;
    double r2 = (xx + yy) + zz;
    return r2 < rc2;
}

static int64_t search(const double* xyz, int64_t n, double distance, uint32_t* pairs, int64_t capacity, int f64)
{
    if (n < 2) return 0;
    float* p = (float*)malloc((size_t)(3 * n) * sizeof(float));
    for (int64_t k = 0; k < 3 * n; k++) p[k] = (float)xyz[k];
    float rcf = (float)distance;
    float rc2 = rcf * rcf;
    double rc2_64 = distance * distance;
    double cell = (double)rcf * 1.001 + 1e-30;
    double lo[3], hi[3];
    for (int k = 0; k < 3; k++) lo[k] = hi[k] = p[k];
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            double v = p[3 * i + k];
            if (v < lo[k]) lo[k] = v;
            if (v > hi[k]) hi[k] = v;
        }
    int64_t nc[3], total = 1;
    for (int k = 0; k < 3; k++) {
        int64_t m = (int64_t)floor((hi[k] - lo[k]) / cell);
        if (m < 1) m = 1;
        if (m > 512) m = 512;
        nc[k] = m;
        total *= m;
    }
    while (total > 8 * n + 64) {
        int kk = 0;
        for (int k = 1; k < 3; k++)
            if (nc[k] > nc[kk]) kk = k;
        total /= nc[kk];
        nc[kk] = nc[kk] > 1 ? nc[kk] / 2 : 1;
        total *= nc[kk];
    }
    double inv[3];
    for (int k = 0; k < 3; k++) inv[k] = (hi[k] > lo[k]) ? (double)nc[k] / (hi[k] - lo[k]) : 0.0;
    int64_t* start = (int64_t*)calloc((size_t)(total + 1), sizeof(int64_t));
    int64_t* cellof = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* items = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        int64_t c[3];
        for (int k = 0; k < 3; k++) {
            int64_t v = (int64_t)(((double)p[3 * i + k] - lo[k]) * inv[k]);
            if (v < 0) v = 0;
            if (v >= nc[k]) v = nc[k] - 1;
            c[k] = v;
        }
        cellof[i] = c[0] + nc[0] * (c[1] + nc[1] * c[2]);
        start[cellof[i] + 1]++;
    }
    for (int64_t c = 0; c < total; c++) start[c + 1] += start[c];
    int64_t* fill = (int64_t*)malloc((size_t)(total + 1) * sizeof(int64_t));
    memcpy(fill, start, (size_t)(total + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) items[fill[cellof[i]]++] = i;
    free(fill);

    int64_t count = 0;
    for (int64_t cz = 0; cz < nc[2]; cz++)
        for (int64_t cy = 0; cy < nc[1]; cy++)
            for (int64_t cx = 0; cx < nc[0]; cx++) {
                int64_t c = cx + nc[0] * (cy + nc[1] * cz);
                for (int64_t a = start[c]; a < start[c + 1]; a++) {
                    int64_t i = items[a];
                    for (int64_t dz = -1; dz <= 1; dz++)
                        for (int64_t dy = -1; dy <= 1; dy++)
                            for (int64_t dx = -1; dx <= 1; dx++) {
                                int64_t x2 = cx + dx, y2 = cy + dy, z2 = cz + dz;
                                if (x2 < 0 || y2 < 0 || z2 < 0 || x2 >= nc[0] || y2 >= nc[1] || z2 >= nc[2]) continue;
                                int64_t c2 = x2 + nc[0] * (y2 + nc[1] * z2);
                                for (int64_t b = start[c2]; b < start[c2 + 1]; b++) {
                                    int64_t j = items[b];
                                    if (j <= i) continue;
                                    if (f64 ? !strict_pair64(xyz, i, j, rc2_64) : !strict_pair(p, i, j, rc2)) continue;
                                    if (count < capacity) {
                                        pairs[2 * count] = (uint32_t)i;
                                        pairs[2 * count + 1] = (uint32_t)j;
                                    }
                                    count++;
                                }
                            }
                }
            }
    if (count <= capacity) qsort(pairs, (size_t)count, 2 * sizeof(uint32_t), cmp_pair);
    free(start);
    free(cellof);
    free(items);
    free(p);
    return count;
}

int64_t gcso_search_neighbors(const double* xyz, int64_t n, double distance, uint32_t* pairs, int64_t capacity)
{
    return search(xyz, n, distance, pairs, capacity, 0);
}

int64_t gcso_search_neighbors64(const double* xyz, int64_t n, double distance, uint32_t* pairs, int64_t capacity)
{
    return search(xyz, n, distance, pairs, capacity, 1);
}
