/*
 * gcs_oracle.c -- TEST INFRASTRUCTURE ONLY: the checker and the CPU baseline, never the product path.
 *
 * fp64 single-threaded restatement of the reference hot path (see gcs_oracle.h for the parity status).
 * Reference paths are relative to /root/reference/src/simulation/.  Choices for micromd semantics that
 * the reference does not pin are marked INFERRED and listed in DESIGN.md ("Oracle").
 */
#include "gcs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

enum {
    K_SOFTCORE = 1,
    K_SOFTWELL,
    K_BONDED,
    K_BENDING,
    K_WALL_IN,
    K_WALL_OUT,
    K_POINT,
    K_KFIBER,
};

/* per_kind energy slots (same order as gcs_engine_compute_energy) */
enum { E_PAIR, E_SOFTWELL, E_BONDS, E_BENDING, E_WALL_IN, E_WALL_OUT, E_POINT, E_KFIBER, E_COUNT };

typedef struct ofield {
    int kind, handle;
    gcs_softcore_params sc;
    gcs_softwell_params sw;
    gcs_bond_params bond;
    gcs_wall_params wall;
    gcs_point_source_params point;
    double spring, center[3], pole[3], energy;
    int64_t* idx; /* bonded: pairs [n][2]; bending: triple starts [n]; softwell: targets [n] */
    int64_t n;
    gcs_kinetochore_spec* specs;
} ofield;

struct gcso_system {
    int64_t n;
    double *x, *mu, *ab, *F;
    ofield* fields;
    int nfields, cap, next_handle;
    gcs_context ctx;
    gcs_schedule sched;
    double* noise;
    int64_t noise_steps, noise_cursor;
    /* cell-list scratch */
    int64_t *cell_start, *cell_items;
    int64_t cell_cap;
    int64_t* cell_of;
    /* domain decomposition (C5): integrate / count reactions of the particles inside the box [dom_lo, dom_hi) only */
    int dom_on;
    double dom_lo[3], dom_hi[3];
    unsigned char* dom_own;
};

/* ------------------------------------------------------------------------------------------------ */
/* system                                                                                           */

gcso_system* gcso_create(const gcs_system_desc* d)
{
    gcso_system* s = (gcso_system*)calloc(1, sizeof(*s));
    int64_t n = d->particle_count;
    s->n = n;
    s->x = (double*)calloc((size_t)(3 * n + 3), sizeof(double));
    s->F = (double*)calloc((size_t)(3 * n + 3), sizeof(double));
    s->mu = (double*)malloc((size_t)(n + 1) * sizeof(double));
    s->ab = (double*)calloc((size_t)(2 * n + 2), sizeof(double));
    s->cell_of = (int64_t*)malloc((size_t)(n + 1) * sizeof(int64_t));
    s->cell_items = (int64_t*)malloc((size_t)(n + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        s->mu[i] = d->mobilities ? d->mobilities[i] : 1.0;
        if (d->ab_factors) {
            s->ab[2 * i] = d->ab_factors[2 * i];
            s->ab[2 * i + 1] = d->ab_factors[2 * i + 1];
        }
    }
    s->ctx.core_scale = 1;
    s->ctx.bond_scale = 1;
    s->next_handle = 1;
    return s;
}

void gcso_destroy(gcso_system* s)
{
    if (!s) return;
    for (int k = 0; k < s->nfields; k++) {
        free(s->fields[k].idx);
        free(s->fields[k].specs);
    }
    free(s->fields);
    free(s->x);
    free(s->F);
    free(s->mu);
    free(s->ab);
    free(s->noise);
    free(s->cell_start);
    free(s->cell_items);
    free(s->cell_of);
    free(s);
}

static ofield* new_field(gcso_system* s, int kind)
{
    if (s->nfields == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 8;
        s->fields = (ofield*)realloc(s->fields, (size_t)s->cap * sizeof(ofield));
    }
    ofield* f = &s->fields[s->nfields++];
    memset(f, 0, sizeof(*f));
    f->kind = kind;
    f->handle = s->next_handle++;
    return f;
}

int gcso_add_neighbor_softcore(gcso_system* s, const gcs_softcore_params* p)
{
    ofield* f = new_field(s, K_SOFTCORE);
    f->sc = *p;
    return f->handle;
}

int gcso_add_neighbor_softwell(gcso_system* s, const gcs_softwell_params* p, const int64_t* targets, int64_t n)
{
    ofield* f = new_field(s, K_SOFTWELL);
    f->sw = *p;
    f->n = n;
    f->idx = (int64_t*)malloc((size_t)(n + 1) * sizeof(int64_t));
    memcpy(f->idx, targets, (size_t)n * sizeof(int64_t));
    return f->handle;
}

/* add_bonded_range(b, e) = pairs (k, k+1) for k in [b, e-1) (micromd, INFERRED; used at
 * simulation_driver_forcefield.cpp:93-95); the loop field adds (i, i+2) pairs explicitly (:131-135). */
int gcso_add_bonded_pairwise(gcso_system* s, const gcs_bond_params* p, const int64_t* ranges, int64_t n_ranges,
                             int32_t stride, const int64_t* pairs, int64_t n_pairs)
{
    ofield* f = new_field(s, K_BONDED);
    f->bond = *p;
    int64_t total = n_pairs;
    for (int64_t r = 0; r < n_ranges; r++) {
        int64_t len = ranges[2 * r + 1] - ranges[2 * r] - stride;
        if (len > 0) total += len;
    }
    f->idx = (int64_t*)malloc((size_t)(2 * total + 2) * sizeof(int64_t));
    int64_t m = 0;
    for (int64_t r = 0; r < n_ranges; r++)
        for (int64_t k = ranges[2 * r]; k + stride < ranges[2 * r + 1]; k++) {
            f->idx[2 * m] = k;
            f->idx[2 * m + 1] = k + stride;
            m++;
        }
    for (int64_t q = 0; q < n_pairs; q++) {
        f->idx[2 * m] = pairs[2 * q];
        f->idx[2 * m + 1] = pairs[2 * q + 1];
        m++;
    }
    f->n = m;
    return f->handle;
}

/* triplewise add_bonded_range(b, e) = triples (k, k+1, k+2), k in [b, e-2) (INFERRED;
 * stage_anatelophase/simulation_driver.cpp:171-178). */
int gcso_add_bonded_triplewise(gcso_system* s, double energy, const int64_t* ranges, int64_t n_ranges)
{
    ofield* f = new_field(s, K_BENDING);
    f->energy = energy;
    int64_t total = 0;
    for (int64_t r = 0; r < n_ranges; r++) {
        int64_t len = ranges[2 * r + 1] - ranges[2 * r] - 2;
        if (len > 0) total += len;
    }
    f->idx = (int64_t*)malloc((size_t)(total + 1) * sizeof(int64_t));
    int64_t m = 0;
    for (int64_t r = 0; r < n_ranges; r++)
        for (int64_t k = ranges[2 * r]; k + 2 < ranges[2 * r + 1]; k++) f->idx[m++] = k;
    f->n = m;
    return f->handle;
}

int gcso_add_ellipsoid_inward(gcso_system* s, const gcs_wall_params* p)
{
    ofield* f = new_field(s, K_WALL_IN);
    f->wall = *p;
    return f->handle;
}

int gcso_add_ellipsoid_outward(gcso_system* s, double spring, const double center[3])
{
    ofield* f = new_field(s, K_WALL_OUT);
    f->spring = spring;
    for (int k = 0; k < 3; k++) f->center[k] = center ? center[k] : 0.0;
    return f->handle;
}

int gcso_add_point_source(gcso_system* s, const gcs_point_source_params* p)
{
    ofield* f = new_field(s, K_POINT);
    f->point = *p;
    return f->handle;
}

int gcso_add_kinetochore_fiber(gcso_system* s, const double pole[3], const gcs_kinetochore_spec* specs, int64_t n)
{
    ofield* f = new_field(s, K_KFIBER);
    for (int k = 0; k < 3; k++) f->pole[k] = pole[k];
    f->n = n;
    f->specs = (gcs_kinetochore_spec*)malloc((size_t)(n + 1) * sizeof(gcs_kinetochore_spec));
    memcpy(f->specs, specs, (size_t)n * sizeof(gcs_kinetochore_spec));
    return f->handle;
}

int gcso_remove_forcefield(gcso_system* s, int handle)
{
    for (int k = 0; k < s->nfields; k++) {
        if (s->fields[k].handle == handle) {
            free(s->fields[k].idx);
            free(s->fields[k].specs);
            memmove(&s->fields[k], &s->fields[k + 1], (size_t)(s->nfields - k - 1) * sizeof(ofield));
            s->nfields--;
            return 0;
        }
    }
    return -1;
}

void gcso_set_positions(gcso_system* s, const double* xyz) { memcpy(s->x, xyz, (size_t)(3 * s->n) * sizeof(double)); }
void gcso_get_positions(const gcso_system* s, double* xyz) { memcpy(xyz, s->x, (size_t)(3 * s->n) * sizeof(double)); }
void gcso_set_context(gcso_system* s, const gcs_context* c) { s->ctx = *c; }
void gcso_get_context(const gcso_system* s, gcs_context* c) { *c = s->ctx; }
void gcso_set_schedule(gcso_system* s, const gcs_schedule* sc) { s->sched = *sc; }

int gcso_set_noise(gcso_system* s, const double* normals, int64_t steps)
{
    free(s->noise);
    s->noise = (double*)malloc((size_t)(steps * s->n * 3 + 1) * sizeof(double));
    memcpy(s->noise, normals, (size_t)(steps * s->n * 3) * sizeof(double));
    s->noise_steps = steps;
    s->noise_cursor = 0;
    return 0;
}

/* The interphase callback's state updates, in the reference order:
 * time (simulation_driver_interphase.cpp:17), update_core_scale (:67-76), update_wall_semiaxes (:79-90).
 * The reaction is the sum of both walls' stats.axial_reaction (simulation_driver_forcefield.cpp:239-243)
 * from the latest force evaluation (Appendix C #8 of SURVEY.md: the engine defines it that way). */
void gcso_apply_schedule(gcso_system* s, int64_t step)
{
    const gcs_schedule* sc = &s->sched;
    gcs_context* c = &s->ctx;
    c->step = step;
    if (sc->update_time) c->time = (double)step * sc->timestep;
    if (sc->update_scales) {
        double t_bead = c->time / sc->core_scale_tau;
        double t_bond = c->time / sc->bond_scale_tau;
        c->core_scale = 1 - (1 - sc->core_scale_init) * exp(-t_bead);
        c->bond_scale = 1 - (1 - sc->bond_scale_init) * exp(-t_bond);
    }
    if (sc->update_wall) {
        for (int k = 0; k < 3; k++) {
            double net = 0;
            net += c->inward_reaction[k] + c->outward_reaction[k];
            net -= sc->wall_semiaxes_spring[k] * c->wall_semiaxes[k];
            c->wall_semiaxes[k] += sc->timestep * sc->wall_mobility * net;
        }
    }
}

/* ------------------------------------------------------------------------------------------------ */
/* potentials (micromd forms, INFERRED)                                              */

/* softcore_potential<2,3>{eps, sigma}: U = eps (1 - r^2/sigma^2)^3; returns U, *coef with F = coef * r */
static inline double sc23(double r2, double eps, double sigma, double* coef)
{
    double k2 = 1.0 / (sigma * sigma);
    double u2 = r2 * k2;
    if (u2 >= 1.0) {
        *coef = 0;
        return 0;
    }
    double g = 1.0 - u2;
    *coef = 6.0 * eps * k2 * g * g;
    return eps * g * g * g;
}

/* softcore_potential<8,3>{eps, sigma}: U = eps (1 - (r/sigma)^8)^3 */
static inline double sc83(double r2, double eps, double sigma, double* coef)
{
    double k2 = 1.0 / (sigma * sigma);
    double u2 = r2 * k2;
    if (u2 >= 1.0) {
        *coef = 0;
        return 0;
    }
    double u4 = u2 * u2;
    double u6 = u4 * u2;
    double g = 1.0 - u4 * u4;
    *coef = 24.0 * eps * k2 * g * g * u6;
    return eps * g * g * g;
}

/* spring-type potentials evaluated at vector r: returns U, *coef with F = coef * r */
static inline double spring_like(int pot, double K, double l, double r2, double* coef)
{
    if (pot == GCS_POT_HARMONIC) {
        *coef = -K;
        return 0.5 * K * r2;
    }
    double d = sqrt(r2);
    if (pot == GCS_POT_SEMISPRING && d <= l) {
        *coef = 0;
        return 0;
    }
    if (d <= 0) {
        *coef = 0;
        return 0.5 * K * l * l;
    }
    double dl = d - l;
    *coef = -K * dl / d;
    return 0.5 * K * dl * dl;
}

/* force_flux_potential (common/potentials/force_flux_potential.hpp:24-37, in-repo, PINNED) */
static inline double force_flux(double f, double b, double r2, double* coef)
{
    double r1 = sqrt(r2);
    double r3 = r1 * r2;
    double b2 = b * b;
    *coef = (r1 > 0) ? f * b2 / (b2 * r1 + r3) : 0;
    return f * b * atan2(b, r1);
}

/* ------------------------------------------------------------------------------------------------ */
/* neighbor pairs (fp64 cell list, half stencil, Newton's third law: the CPU-natural form)          */

typedef void (*pair_fn)(gcso_system* s, const ofield* f, int64_t i, int64_t j, double r2, const double* r,
                        double* energy, int want_force);

static void pair_softcore(gcso_system* s, const ofield* f, int64_t i, int64_t j, double r2, const double* r,
                          double* energy, int want_force)
{
    /* simulation_driver_forcefield.cpp:32-47 (interphase, mix) and
     * stage_anatelophase/simulation_driver.cpp:128-136 (mitotic, plain softcore<2,3>) */
    const gcs_softcore_params* p = &f->sc;
    double scale = p->scaled ? s->ctx.core_scale : 1.0;
    double a = 1.0, b = 0.0;
    if (p->mix) {
        a = 0.5 * (s->ab[2 * i] + s->ab[2 * j]);
        b = 0.5 * (s->ab[2 * i + 1] + s->ab[2 * j + 1]);
    }
    double ca = 0, cb = 0, u = 0;
    u += a * sc23(r2, p->a_energy, p->a_diameter * scale, &ca);
    if (p->b_energy != 0 || p->mix) u += b * sc83(r2, p->b_energy, p->b_diameter * scale, &cb);
    *energy += u;
    if (want_force) {
        double c = a * ca + b * cb;
        for (int k = 0; k < 3; k++) {
            s->F[3 * i + k] += c * r[k];
            s->F[3 * j + k] -= c * r[k];
        }
    }
}

static void ensure_cells(gcso_system* s, int64_t ncell)
{
    if (ncell + 1 > s->cell_cap) {
        free(s->cell_start);
        s->cell_cap = ncell + 1;
        s->cell_start = (int64_t*)malloc((size_t)s->cell_cap * sizeof(int64_t));
    }
}

/* Enumerate every unordered pair closer than rc exactly once. */
static void for_each_pair(gcso_system* s, const ofield* f, double rc, pair_fn fn, double* energy, int want_force)
{
    int64_t n = s->n;
    if (n < 2) return;
    double lo[3], hi[3];
    for (int k = 0; k < 3; k++) lo[k] = hi[k] = s->x[k];
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            double v = s->x[3 * i + k];
            if (v < lo[k]) lo[k] = v;
            if (v > hi[k]) hi[k] = v;
        }
    int64_t nc[3];
    double inv[3];
    int64_t total = 1;
    for (int k = 0; k < 3; k++) {
        double ext = hi[k] - lo[k];
        int64_t m = (int64_t)floor(ext / (rc * (1 + 1e-9)));
        if (m < 1) m = 1;
        if (m > 256) m = 256;
        nc[k] = m;
        inv[k] = ext > 0 ? (double)m / ext : 0;
        total *= m;
    }
    while (total > 4 * n + 64) { /* keep the grid proportional to N (cells only get larger) */
        int kk = 0;
        for (int k = 1; k < 3; k++)
            if (nc[k] > nc[kk]) kk = k;
        total /= nc[kk];
        nc[kk] = nc[kk] > 1 ? nc[kk] / 2 : 1;
        total *= nc[kk];
        inv[kk] = (hi[kk] > lo[kk]) ? (double)nc[kk] / (hi[kk] - lo[kk]) : 0;
    }
    ensure_cells(s, total);
    memset(s->cell_start, 0, (size_t)(total + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < n; i++) {
        int64_t c[3];
        for (int k = 0; k < 3; k++) {
            int64_t v = (int64_t)((s->x[3 * i + k] - lo[k]) * inv[k]);
            if (v < 0) v = 0;
            if (v >= nc[k]) v = nc[k] - 1;
            c[k] = v;
        }
        int64_t id = c[0] + nc[0] * (c[1] + nc[1] * c[2]);
        s->cell_of[i] = id;
        s->cell_start[id + 1]++;
    }
    for (int64_t c = 0; c < total; c++) s->cell_start[c + 1] += s->cell_start[c];
    {
        /* counting sort, stable */
        int64_t* fill = (int64_t*)malloc((size_t)(total + 1) * sizeof(int64_t));
        memcpy(fill, s->cell_start, (size_t)(total + 1) * sizeof(int64_t));
        for (int64_t i = 0; i < n; i++) s->cell_items[fill[s->cell_of[i]]++] = i;
        free(fill);
    }
    double rc2 = rc * rc;
    static const int off[13][3] = {{1, 0, 0},  {-1, 1, 0}, {0, 1, 0},  {1, 1, 0},  {-1, -1, 1},
                                   {0, -1, 1}, {1, -1, 1}, {-1, 0, 1}, {0, 0, 1},  {1, 0, 1},
                                   {-1, 1, 1}, {0, 1, 1},  {1, 1, 1}};
    for (int64_t cz = 0; cz < nc[2]; cz++)
        for (int64_t cy = 0; cy < nc[1]; cy++)
            for (int64_t cx = 0; cx < nc[0]; cx++) {
                int64_t c = cx + nc[0] * (cy + nc[1] * cz);
                int64_t b0 = s->cell_start[c], e0 = s->cell_start[c + 1];
                if (b0 == e0) continue;
                /* within the cell */
                for (int64_t p = b0; p < e0; p++)
                    for (int64_t q = p + 1; q < e0; q++) {
                        int64_t i = s->cell_items[p], j = s->cell_items[q];
                        double r[3] = {s->x[3 * i] - s->x[3 * j], s->x[3 * i + 1] - s->x[3 * j + 1],
                                       s->x[3 * i + 2] - s->x[3 * j + 2]};
                        double r2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
                        if (r2 < rc2) fn(s, f, i, j, r2, r, energy, want_force);
                    }
                for (int o = 0; o < 13; o++) {
                    int64_t x2 = cx + off[o][0], y2 = cy + off[o][1], z2 = cz + off[o][2];
                    if (x2 < 0 || y2 < 0 || z2 < 0 || x2 >= nc[0] || y2 >= nc[1] || z2 >= nc[2]) continue;
                    int64_t c2 = x2 + nc[0] * (y2 + nc[1] * z2);
                    int64_t b1 = s->cell_start[c2], e1 = s->cell_start[c2 + 1];
                    for (int64_t p = b0; p < e0; p++) {
                        int64_t i = s->cell_items[p];
                        double xi = s->x[3 * i], yi = s->x[3 * i + 1], zi = s->x[3 * i + 2];
                        for (int64_t q = b1; q < e1; q++) {
                            int64_t j = s->cell_items[q];
                            double r[3] = {xi - s->x[3 * j], yi - s->x[3 * j + 1], zi - s->x[3 * j + 2]};
                            double r2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
                            if (r2 < rc2) fn(s, f, i, j, r2, r, energy, want_force);
                        }
                    }
                }
            }
}

/* ------------------------------------------------------------------------------------------------ */
/* ellipsoid wall distance (INFERRED): first-order (Sampson) distance to the surface      */
/* rho(r) = |r o (1/semiaxes)| = 1; d = |1 - rho| rho / |grad|, normal n = grad/|grad|,             */
/* grad = (rx/ax^2, ry/ay^2, rz/az^2).  Exact for a sphere.  Returns 0 if the point is degenerate.   */
static inline int ellipsoid_distance(const double* r, const double* ax, double* rho, double* d, double* nrm)
{
    double q2 = 0, g[3], g2 = 0;
    for (int k = 0; k < 3; k++) {
        double q = r[k] / ax[k];
        q2 += q * q;
        g[k] = r[k] / (ax[k] * ax[k]);
        g2 += g[k] * g[k];
    }
    if (g2 <= 0) return 0;
    double rr = sqrt(q2), gn = sqrt(g2);
    *rho = rr;
    *d = fabs(1.0 - rr) * rr / gn;
    for (int k = 0; k < 3; k++) nrm[k] = g[k] / gn;
    return 1;
}

/* ------------------------------------------------------------------------------------------------ */
/* force/energy evaluation of every registered field                                                */

static void eval_fields(gcso_system* s, int want_force, double* per_kind)
{
    int64_t n = s->n;
    double e[E_COUNT] = {0};
    double* F = s->F;
    if (want_force) {
        memset(F, 0, (size_t)(3 * n) * sizeof(double));
        for (int k = 0; k < 3; k++) s->ctx.inward_reaction[k] = s->ctx.outward_reaction[k] = 0;
    }
    double cs = s->ctx.core_scale, bs = s->ctx.bond_scale;
    for (int fi = 0; fi < s->nfields; fi++) {
        const ofield* f = &s->fields[fi];
        switch (f->kind) {
        case K_SOFTCORE: {
            double rc = f->sc.neighbor_distance * (f->sc.scaled ? cs : 1.0);
            for_each_pair(s, f, rc, pair_softcore, &e[E_PAIR], want_force);
            break;
        }
        case K_SOFTWELL: {
            /* neighbor pairs restricted to the targets (set_neighbor_targets, INFERRED: both ends),
             * apply_cutoff = plain truncation at `cutoff` (INFERRED: no energy shift) */
            const gcs_softwell_params* p = &f->sw;
            double d2 = p->decay_distance * p->decay_distance, rc2 = p->cutoff * p->cutoff;
            for (int64_t a = 0; a < f->n; a++)
                for (int64_t b = a + 1; b < f->n; b++) {
                    int64_t i = f->idx[a], j = f->idx[b];
                    double r[3], r2 = 0;
                    for (int k = 0; k < 3; k++) {
                        r[k] = s->x[3 * i + k] - s->x[3 * j + k];
                        r2 += r[k] * r[k];
                    }
                    if (r2 >= rc2) continue;
                    double u = r2 / d2;
                    double u3 = u * u * u; /* (r/decay)^6 */
                    double den = 1.0 + u3;
                    e[E_SOFTWELL] += -p->energy / den;
                    if (want_force) {
                        double c = -6.0 * p->energy * u * u / (d2 * den * den);
                        for (int k = 0; k < 3; k++) {
                            F[3 * i + k] += c * r[k];
                            F[3 * j + k] -= c * r[k];
                        }
                    }
                }
            break;
        }
        case K_BONDED: {
            /* simulation_driver_forcefield.cpp:63-89 (chain), :106-127 (loop), :146-155 (nucleolar);
             * mitotic fixed-parameter bonds stage_anatelophase/simulation_driver.cpp:145-156 */
            const gcs_bond_params* p = &f->bond;
            for (int64_t q = 0; q < f->n; q++) {
                int64_t i = f->idx[2 * q], j = f->idx[2 * q + 1];
                double K = p->a_spring, l = p->a_length;
                if (p->mix) {
                    double a = 0.5 * (s->ab[2 * i] + s->ab[2 * j]);
                    double b = 0.5 * (s->ab[2 * i + 1] + s->ab[2 * j + 1]);
                    K = a * p->a_spring + b * p->b_spring;
                    l = a * p->a_length + b * p->b_length;
                }
                if (p->scaled) {
                    K = K * (1 / (bs * bs));
                    l = l * bs;
                }
                double r[3], r2 = 0, c;
                for (int k = 0; k < 3; k++) {
                    r[k] = s->x[3 * i + k] - s->x[3 * j + k];
                    r2 += r[k] * r[k];
                }
                e[E_BONDS] += spring_like(p->potential, K, l, r2, &c);
                if (want_force)
                    for (int k = 0; k < 3; k++) {
                        F[3 * i + k] += c * r[k];
                        F[3 * j + k] -= c * r[k];
                    }
            }
            break;
        }
        case K_BENDING: {
            /* cosine_bending_potential{bending_energy}: U = eps (1 - cos theta) between successive bond
             * vectors (INFERRED form; used at stage_anatelophase/simulation_driver.cpp:165-187) */
            double eps = f->energy;
            for (int64_t q = 0; q < f->n; q++) {
                int64_t i = f->idx[q], j = i + 1, k3 = i + 2;
                double r1[3], r2[3], n1 = 0, n2 = 0, dot = 0;
                for (int k = 0; k < 3; k++) {
                    r1[k] = s->x[3 * j + k] - s->x[3 * i + k];
                    r2[k] = s->x[3 * k3 + k] - s->x[3 * j + k];
                    n1 += r1[k] * r1[k];
                    n2 += r2[k] * r2[k];
                    dot += r1[k] * r2[k];
                }
                if (n1 <= 0 || n2 <= 0) continue;
                double inv12 = 1.0 / sqrt(n1 * n2);
                double cosv = dot * inv12;
                e[E_BENDING] += eps * (1 - cosv);
                if (want_force)
                    for (int k = 0; k < 3; k++) {
                        double dc1 = r2[k] * inv12 - cosv * r1[k] / n1;
                        double dc2 = r1[k] * inv12 - cosv * r2[k] / n2;
                        double fi = -eps * dc1, fk = eps * dc2;
                        F[3 * i + k] += fi;
                        F[3 * k3 + k] += fk;
                        F[3 * j + k] -= fi + fk;
                    }
            }
            break;
        }
        case K_WALL_IN: {
            /* simulation_driver_forcefield.cpp:203-225: a = (a_i + wall_a)/2, b = (b_i + wall_b)/2,
             * a*SC<2,3>(a_energy, d_a/2 * cs) + b*SC<8,3>(b_energy, d_b/2 * cs) of the wall distance */
            const gcs_wall_params* p = &f->wall;
            double scale = p->scaled ? cs : 1.0;
            for (int64_t i = 0; i < n; i++) {
                double r[3], rho, d, nrm[3];
                for (int k = 0; k < 3; k++) r[k] = s->x[3 * i + k] - p->center[k];
                if (!ellipsoid_distance(r, s->ctx.wall_semiaxes, &rho, &d, nrm)) continue;
                if (rho >= 1.0) continue;
                double a = 1.0, b = 0.0;
                if (p->mix) {
                    a = 0.5 * (s->ab[2 * i] + p->wall_a);
                    b = 0.5 * (s->ab[2 * i + 1] + p->wall_b);
                }
                double ca = 0, cb = 0, d2 = d * d;
                e[E_WALL_IN] += a * sc23(d2, p->a_energy, p->a_diameter * scale, &ca);
                if (p->b_energy != 0 || p->mix) e[E_WALL_IN] += b * sc83(d2, p->b_energy, p->b_diameter * scale, &cb);
                if (want_force) {
                    double c = a * ca + b * cb;
                    for (int k = 0; k < 3; k++) {
                        double fk = c * (-d * nrm[k]); /* along the wall->particle vector (inward) */
                        F[3 * i + k] += fk;
                        if (!s->dom_own || s->dom_own[i]) s->ctx.inward_reaction[k] += fabs(fk);
                    }
                }
            }
            break;
        }
        case K_WALL_OUT: {
            /* simulation_driver_forcefield.cpp:230-237: harmonic{wall_packing_spring} outside the wall */
            for (int64_t i = 0; i < n; i++) {
                double r[3], rho, d, nrm[3];
                for (int k = 0; k < 3; k++) r[k] = s->x[3 * i + k] - f->center[k];
                if (!ellipsoid_distance(r, s->ctx.wall_semiaxes, &rho, &d, nrm)) continue;
                if (rho <= 1.0) continue;
                e[E_WALL_OUT] += 0.5 * f->spring * d * d;
                if (want_force)
                    for (int k = 0; k < 3; k++) {
                        double fk = -f->spring * d * nrm[k];
                        F[3 * i + k] += fk;
                        if (!s->dom_own || s->dom_own[i]) s->ctx.outward_reaction[k] += fabs(fk);
                    }
            }
            break;
        }
        case K_POINT: {
            /* stage_anatelophase/simulation_driver.cpp:221-235; stage_prometaphase/simulation_driver.cpp:210-230 */
            const gcs_point_source_params* p = &f->point;
            for (int64_t i = 0; i < n; i++) {
                double r[3], r2 = 0, c;
                for (int k = 0; k < 3; k++) {
                    r[k] = s->x[3 * i + k] - p->point[k];
                    r2 += r[k] * r[k];
                }
                if (p->potential == GCS_POT_FORCE_FLUX)
                    e[E_POINT] += force_flux(p->force, p->reactive_distance, r2, &c);
                else
                    e[E_POINT] += spring_like(p->potential, p->spring, p->length, r2, &c);
                if (want_force)
                    for (int k = 0; k < 3; k++) F[3 * i + k] += c * r[k];
            }
            break;
        }
        case K_KFIBER: {
            /* common/forcefield/kinetochore_fiber_forcefield.cpp:46-84: spring{decay/mobility, length} */
            for (int64_t q = 0; q < f->n; q++) {
                const gcs_kinetochore_spec* sp = &f->specs[q];
                int64_t i = sp->particle_index;
                double r[3], r2 = 0, c;
                for (int k = 0; k < 3; k++) {
                    r[k] = s->x[3 * i + k] - f->pole[k];
                    r2 += r[k] * r[k];
                }
                e[E_KFIBER] += spring_like(GCS_POT_SPRING, sp->decay_rate / sp->mobility, sp->stationary_length, r2, &c);
                if (want_force)
                    for (int k = 0; k < 3; k++) F[3 * i + k] += c * r[k];
            }
            break;
        }
        }
    }
    if (per_kind)
        for (int k = 0; k < E_COUNT; k++) per_kind[k] = e[k];
}

double gcso_compute_energy(gcso_system* s, double* per_kind)
{
    double pk[E_COUNT];
    eval_fields(s, 0, pk);
    double tot = 0;
    for (int k = 0; k < E_COUNT; k++) tot += pk[k];
    if (per_kind) memcpy(per_kind, pk, sizeof(pk));
    return tot;
}

void gcso_compute_forces(gcso_system* s, double* forces)
{
    eval_fields(s, 1, NULL);
    memcpy(forces, s->F, (size_t)(3 * s->n) * sizeof(double));
}

/* ------------------------------------------------------------------------------------------------ */
/* Brownian dynamics (md::simulate_brownian_dynamics, INFERRED Euler-Maruyama form; seed plumbing    */
/* PINNED at simulation_driver_interphase.cpp:57-63 / simulation_driver_relaxation.cpp:48-55)                          */

int gcso_run(gcso_system* s, const gcs_bd_config* cfg, int64_t first_step, int64_t steps)
{
    int64_t n = s->n;
    double* xi = (double*)malloc((size_t)(3 * n + 3) * sizeof(double));
    for (int64_t st = first_step + 1; st <= first_step + steps; st++) {
        if (s->dom_on) {
            if (!s->dom_own) s->dom_own = (unsigned char*)malloc((size_t)n + 1);
            for (int64_t i = 0; i < n; i++) {
                int own = 1;
                for (int k = 0; k < 3; k++) own &= s->x[3 * i + k] >= s->dom_lo[k] && s->x[3 * i + k] < s->dom_hi[k];
                s->dom_own[i] = (unsigned char)own;
            }
        }
        eval_fields(s, 1, NULL);
        double dt = cfg->timestep;
        if (cfg->spacestep > 0) {
            /* INFERRED: the step's timestep shrinks so that the largest drift displacement is spacestep */
            double m = 0;
            for (int64_t i = 0; i < n; i++) {
                double f2 = s->F[3 * i] * s->F[3 * i] + s->F[3 * i + 1] * s->F[3 * i + 1] + s->F[3 * i + 2] * s->F[3 * i + 2];
                double v = s->mu[i] * sqrt(f2);
                if (v > m) m = v;
            }
            if (m * dt > cfg->spacestep) dt = cfg->spacestep / m;
        }
        s->ctx.last_timestep = dt;
        if (cfg->noise == GCS_NOISE_PHILOX) {
            gcso_philox_normals(cfg->seed, st, n, xi);
        } else if (cfg->noise == GCS_NOISE_INJECTED) {
            if (s->noise_cursor >= s->noise_steps) {
                free(xi);
                return -1;
            }
            memcpy(xi, s->noise + s->noise_cursor * n * 3, (size_t)(3 * n) * sizeof(double));
            s->noise_cursor++;
        } else {
            memset(xi, 0, (size_t)(3 * n) * sizeof(double));
        }
        for (int64_t i = 0; i < n; i++) {
            if (s->dom_on && !s->dom_own[i]) continue; /* another domain integrates it */
            double mu = s->mu[i];
            double amp = sqrt(2 * cfg->temperature * mu * dt);
            for (int k = 0; k < 3; k++) s->x[3 * i + k] += mu * dt * s->F[3 * i + k] + amp * xi[3 * i + k];
        }
        gcso_apply_schedule(s, st);
    }
    free(xi);
    if (s->dom_on) { /* the mask is only for the steps' own evaluations */
        free(s->dom_own);
        s->dom_own = NULL;
    }
    return 0;
}

/* domain decomposition (C5, DESIGN.md "Multi-GPU"): on != 0 -> run() integrates only the particles inside the box
 * [lo, hi) (per axis) at the start of each step, and the wall reactions count those only (the caller sums them over
 * domains and applies the wall update itself) */
void gcso_set_domain(gcso_system* s, int on, const double* lo, const double* hi)
{
    s->dom_on = on;
    for (int k = 0; k < 3; k++) {
        s->dom_lo[k] = on ? lo[k] : 0.0;
        s->dom_hi[k] = on ? hi[k] : 0.0;
    }
}

