/*
 * gcs_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (fp64, single-threaded, like the reference) of the snsinfu/3d-genome-cycle hot path:
 * the micromd force fields, neighbor search and Brownian integrator as the stage drivers use them.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
 * as the checker / CPU baseline.  The product path (libgcs.so) never links or calls it.
 *
 * PARITY STATUS (see DESIGN.md "Oracle"):
 *  - micromd (github.com/snsinfu/micromd, header-only, un-vendored submodule, version UNPINNED, absent
 *    from /root/reference and not fetchable offline): the potential forms, ellipsoid distance, cutoff
 *    and spacestep semantics are RESTATED from the call sites and documented choices -> "parity
 *    unpinned" for those rows.  No golden vector of the reference covers them (the reference has no tests).
 *  - PINNED: every force-field composition and parameter expression of the drivers (file:line cited per
 *    function in gcs_oracle.c), force_flux_potential and kinetochore_fiber_forcefield arithmetic
 *    (in-repo), std::seed_seq / std::mt19937_64 / libstdc++ normal_distribution (standard-specified,
 *    checked against g++-generated fixtures in tests/golden/), Philox4x32-10 (Random123 known-answer
 *    vectors), quantize (simulation_store.cpp:22-33).
 */
#ifndef GCS_ORACLE_H
#define GCS_ORACLE_H

#include <stdint.h>

#include "../include/gcs.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gcso_system gcso_system;

gcso_system* gcso_create(const gcs_system_desc* desc);
void gcso_destroy(gcso_system* s);

int gcso_add_neighbor_softcore(gcso_system* s, const gcs_softcore_params* p);
int gcso_add_neighbor_softwell(gcso_system* s, const gcs_softwell_params* p, const int64_t* targets, int64_t n);
int gcso_add_bonded_pairwise(gcso_system* s, const gcs_bond_params* p, const int64_t* ranges, int64_t n_ranges,
                             int32_t stride, const int64_t* pairs, int64_t n_pairs);
int gcso_add_bonded_triplewise(gcso_system* s, double energy, const int64_t* ranges, int64_t n_ranges);
int gcso_add_ellipsoid_inward(gcso_system* s, const gcs_wall_params* p);
int gcso_add_ellipsoid_outward(gcso_system* s, double spring, const double center[3]);
int gcso_add_point_source(gcso_system* s, const gcs_point_source_params* p);
int gcso_add_kinetochore_fiber(gcso_system* s, const double pole[3], const gcs_kinetochore_spec* specs, int64_t n);
int gcso_remove_forcefield(gcso_system* s, int handle);

void gcso_set_positions(gcso_system* s, const double* xyz);
void gcso_get_positions(const gcso_system* s, double* xyz);
void gcso_set_context(gcso_system* s, const gcs_context* c);
void gcso_get_context(const gcso_system* s, gcs_context* c);
void gcso_set_schedule(gcso_system* s, const gcs_schedule* sc);
void gcso_apply_schedule(gcso_system* s, int64_t step);
int gcso_set_noise(gcso_system* s, const double* normals, int64_t steps);

int gcso_run(gcso_system* s, const gcs_bd_config* cfg, int64_t first_step, int64_t steps);
double gcso_compute_energy(gcso_system* s, double* per_kind /* [8] or NULL */);
void gcso_compute_forces(gcso_system* s, double* forces /* [N][3] */);

/* strict-fp32 neighbor predicate (oracle/strict_f32.c): pairs (i<j) sorted, returns the count (may
 * exceed capacity; only the first `capacity` pairs are written). */
int64_t gcso_search_neighbors(const double* xyz, int64_t n, double distance, uint32_t* pairs, int64_t capacity);
/* the same in fp64 (the fp64 engine's predicate) on the points themselves */
int64_t gcso_search_neighbors64(const double* xyz, int64_t n, double distance, uint32_t* pairs, int64_t capacity);

/* random numbers */
void gcso_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void gcso_philox_normals(uint64_t seed, int64_t step, int64_t n, double* out /* [n][3] */);
void gcso_seed_seq_generate(const uint32_t* seeds, int64_t n_seeds, uint32_t* out, int64_t n_out);
typedef struct gcso_mt19937_64 { uint64_t mt[312]; int64_t index; } gcso_mt19937_64;
void gcso_mt19937_64_seed(gcso_mt19937_64* g, uint64_t seed);
uint64_t gcso_mt19937_64_next(gcso_mt19937_64* g);
/* `count` normals of std::normal_distribution<double> driven by std::mt19937_64(seed) (libstdc++) */
void gcso_reference_normals(uint64_t seed, int64_t count, double* out);
double gcso_quantize(double value, int bits);
void gcso_set_domain(gcso_system* s, int on, const double* lo /* [3] */, const double* hi /* [3] */);

#ifdef __cplusplus
}
#endif

#endif
