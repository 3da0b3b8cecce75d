/*
 * gcs.h -- C ABI of the MI355X-native overdamped-Langevin chromosome-polymer engine.
 *
 * Drop-in boundary for the hot path of snsinfu/3d-genome-cycle: the force/integrator loop that the
 * stage drivers run through the (un-vendored, header-only) micromd library `md::`.  Every entry point
 * below replaces one micromd call site used by the reference drivers; the replaced interface is cited
 * as reference file:line (paths relative to src/simulation/ of the reference).
 *
 *   md::system{add_particle, view_mobilities, add_attribute}   -> gcs_engine_create
 *       stage_interphase/simulation_driver_particles.cpp:9-35; stage_anatelophase/simulation_driver.cpp:53-64
 *   md::make_neighbor_pairwise_forcefield(a*softcore<2,3> + b*softcore<8,3>)
 *                                                              -> gcs_add_neighbor_softcore
 *       stage_interphase/simulation_driver_forcefield.cpp:21-53; stage_anatelophase/simulation_driver.cpp:77-91;
 *       stage_prometaphase/simulation_driver.cpp:51-63
 *   md::make_neighbor_pairwise_forcefield(apply_cutoff(softwell<6>)).set_neighbor_targets
 *                                                              -> gcs_add_neighbor_softwell
 *       stage_interphase/simulation_driver_forcefield.cpp:162-186
 *   md::make_bonded_pairwise_forcefield + add_bonded_range / add_bonded_pair
 *                                                              -> gcs_add_bonded_pairwise
 *       stage_interphase/simulation_driver_forcefield.cpp:57-160; stage_anatelophase/simulation_driver.cpp:94-117;
 *       stage_prometaphase/simulation_driver.cpp:66-76; stage_prometaphase/simulation_driver.cpp:100-118
 *   md::make_bonded_triplewise_forcefield(cosine_bending_potential) -> gcs_add_bonded_triplewise
 *       stage_anatelophase/simulation_driver.cpp:119-145; stage_prometaphase/simulation_driver.cpp:78-96
 *   md::make_ellipsoid_inward_forcefield / make_ellipsoid_outward_forcefield (+ stats.axial_reaction)
 *                                                              -> gcs_add_ellipsoid_inward / _outward
 *       stage_interphase/simulation_driver_forcefield.cpp:189-244
 *   md::make_point_source_forcefield(semispring | force_flux_potential) -> gcs_add_point_source
 *       stage_anatelophase/simulation_driver.cpp:176-189; stage_prometaphase/simulation_driver.cpp:162-182;
 *       common/potentials/force_flux_potential.hpp:19-37
 *   kinetochore_fiber_forcefield (custom md::forcefield)       -> gcs_add_kinetochore_fiber
 *       common/forcefield/kinetochore_fiber_forcefield.hpp:8-30; common/forcefield/kinetochore_fiber_forcefield.cpp:9-84;
 *       used at stage_anatelophase/simulation_driver.cpp:149-172; stage_prometaphase/simulation_driver.cpp:121-159
 *   md::system::remove_forcefield                             -> gcs_remove_forcefield
 *       stage_anatelophase/simulation_driver.cpp:277-285 (anaphase -> telophase swap)
 *   md::system::view_positions (read/write)                    -> gcs_engine_set_positions / _get_positions
 *       stage_interphase/simulation_driver_relaxation.cpp:14-23; stage_interphase/simulation_driver_interphase.cpp:34
 *   md::system::compute_energy / compute_potential_energy      -> gcs_engine_compute_energy
 *       stage_interphase/simulation_driver_interphase.cpp:24-27; stage_anatelophase/simulation_driver.cpp:325;
 *       stage_prometaphase/simulation_driver.cpp:251
 *   md::simulate_brownian_dynamics(system, {T, dt, spacestep, steps, seed, callback})
 *                                                              -> gcs_engine_run (+ gcs_engine_set_schedule)
 *       stage_interphase/simulation_driver_interphase.cpp:57-63; stage_interphase/simulation_driver_relaxation.cpp:48-55;
 *       stage_anatelophase/simulation_driver.cpp:262-268; stage_anatelophase/simulation_driver.cpp:303-309;
 *       stage_prometaphase/simulation_driver.cpp:230-236
 *     The per-step callback's force-field mutations (update_core_scale, update_wall_semiaxes,
 *     stage_interphase/simulation_driver_interphase.cpp:67-90) run ON DEVICE via gcs_schedule; the host
 *     regains control only at interval boundaries (logging / sampling / contact map).
 *   md::neighbor_searcher<md::open_box>(box, dist).set_points().search() -> gcs_engine_search_neighbors
 *       stage_interphase/contact_map.cpp:60-62
 *
 * Conventions: every function returns 0 (GCS_OK) on success or a positive GCS_E* code; the message of
 * the most recent failure on the calling thread is returned by gcs_last_error().  All arrays crossing
 * the boundary are plain host pointers owned by the caller and copied; device memory is engine-owned.
 * Positions are fp64 at the boundary (md::point is double).  On the device the engine computes in fp64 like the
 * reference (GCS_PRECISION_F64, the default: positions, forces, the integrator, the pair predicate) or, when
 * asked, in fp32 (GCS_PRECISION_F32).  One engine per host thread, bound to one HIP device and one stream;
 * engines are not internally locked.
 */
#ifndef GCS_H
#define GCS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: gcs_run_stats gained fused_contact_steps (an out-struct grew: callers built against 1 must rebuild)
 * 3: gcs_system_desc.reserved became .precision (0 = fp64); gcs_run_stats lost the small-path counters and
 *    gained density_probes; gcs_list_stats gained deal; GCS_OPT_SMALL_PATH and GCS_OPT_FUSED_STEP 1 are gone;
 *    later in 3 (additive, no layout change): GCS_OPT_LIST_FORMAT; the default list skin follows the core scale;
 *    GCS_OPT_SMALL_STEP; GCS_ESTATE also reports a stalled cross-workgroup hand-off (round 6: GCS_OPT_LIST_FORMAT 3,
 *    an experiment, was removed; GCS_OPT_LIST_PHASE, GCS_OPT_LIST_SKIN_BASE added) */
#define GCS_ABI_VERSION 3

/* arithmetic precision of an engine (gcs_system_desc.precision) */
#define GCS_PRECISION_DEFAULT 0 /* = GCS_PRECISION_F64 */
#define GCS_PRECISION_F32 32    /* fp32 positions and arithmetic (fastest; all step shapes, spatial decomposition) */
#define GCS_PRECISION_F64 64    /* fp64 positions and arithmetic, as md::scalar = double; the list step */

/* status codes */
#define GCS_OK 0
#define GCS_EINVAL 1    /* bad argument */
#define GCS_EHIP 2      /* HIP runtime failure (message names the call) */
#define GCS_ESTATE 3    /* call not valid in the engine's current state */
#define GCS_ENOMEM 4    /* allocation failure */
#define GCS_ECAPACITY 5 /* output buffer too small; the required count is still returned */

/* pair potentials (micromd names) */
#define GCS_POT_SEMISPRING 0 /* U = K/2 (r-l)^2 for r > l, else 0 */
#define GCS_POT_HARMONIC 1   /* U = K/2 r^2 */
#define GCS_POT_SPRING 2     /* U = K/2 (r-l)^2 */
#define GCS_POT_FORCE_FLUX 3 /* U = b f atan2(b, r)   (common/potentials/force_flux_potential.hpp:24-37) */

/* noise sources for gcs_engine_run */
#define GCS_NOISE_PHILOX 0   /* counter-based Philox4x32-10 keyed by (seed, step, particle): production */
#define GCS_NOISE_INJECTED 1 /* normals uploaded with gcs_engine_set_noise (reference-order parity mode) */
#define GCS_NOISE_NONE 2     /* deterministic drift only */

typedef struct gcs_engine gcs_engine;

/* md::system construction: particle count, per-particle mobility and the interphase particle_data
 * attribute {a_factor, b_factor} (common/particle_data.hpp:6-13). */
typedef struct gcs_system_desc {
    int64_t particle_count;
    const double* mobilities; /* [N]; NULL -> 1 (micromd default mobility) */
    const double* ab_factors; /* [N][2]; NULL -> (0, 0) */
    int32_t device;           /* HIP device ordinal */
    int32_t precision;        /* GCS_PRECISION_* (0: fp64) */
} gcs_system_desc;

/* Neighbor-pairwise soft-core repulsion: U_ij = a_ij*SC<2,3>(r) + b_ij*SC<8,3>(r),
 * SC<p,q>(r) = eps (1 - (r/sigma)^p)^q for r < sigma.
 * mix = 1: a_ij = (a_i + a_j)/2, b_ij = (b_i + b_j)/2 (stage_interphase/simulation_driver_forcefield.cpp:34-35);
 * mix = 0: a_ij = 1, b_ij = 0 (plain softcore<2,3>, mitotic stages).
 * scaled = 1: both diameters and neighbor_distance are multiplied by the context core_scale
 * (stage_interphase/simulation_driver_forcefield.cpp:39-43, 49-51). */
typedef struct gcs_softcore_params {
    double a_energy, a_diameter;
    double b_energy, b_diameter;
    double neighbor_distance;
    int32_t mix;
    int32_t scaled;
} gcs_softcore_params;

/* Bonded pairwise potential. mix = 1: K = a*a_spring + b*b_spring, l = a*a_length + b*b_length with
 * a, b the pair means of the ab factors (stage_interphase/simulation_driver_forcefield.cpp:65-76); mix = 0: K = a_spring,
 * l = a_length.  scaled = 1: K /= s^2 and l *= s with s the context bond_scale (:81-83, :147-149). */
typedef struct gcs_bond_params {
    int32_t potential; /* GCS_POT_SEMISPRING | GCS_POT_HARMONIC | GCS_POT_SPRING */
    int32_t mix;
    int32_t scaled;
    int32_t reserved;
    double a_spring, b_spring;
    double a_length, b_length;
} gcs_bond_params;

/* Droplet attraction among a target subset: apply_cutoff(softwell<exponent>{energy, decay}, cutoff),
 * U = -energy / (1 + (r/decay)^exponent) for r < cutoff (stage_interphase/simulation_driver_forcefield.cpp:173-185). */
typedef struct gcs_softwell_params {
    double energy;
    double decay_distance;
    double cutoff;
    int32_t exponent; /* only 6 is used by the reference */
    int32_t reserved;
} gcs_softwell_params;

/* Ellipsoid wall inward field: per-particle a = (a_i + wall_a)/2, b = (b_i + wall_b)/2 and
 * a*SC<2,3>(a_energy, a_diameter) + b*SC<8,3>(b_energy, b_diameter) of the distance to the wall
 * (stage_interphase/simulation_driver_forcefield.cpp:203-225). Diameters are passed already halved (the reference
 * uses a_core_diameter / 2); scaled multiplies them by core_scale.  The ellipsoid is centred at
 * `center` with semiaxes taken from the context (:194-201). */
typedef struct gcs_wall_params {
    double a_energy, a_diameter;
    double b_energy, b_diameter;
    double wall_a, wall_b;
    double center[3];
    int32_t mix;
    int32_t scaled;
} gcs_wall_params;

/* Point source field U(x - point) (make_point_source_forcefield). */
typedef struct gcs_point_source_params {
    int32_t potential; /* GCS_POT_SEMISPRING | GCS_POT_HARMONIC | GCS_POT_SPRING | GCS_POT_FORCE_FLUX */
    int32_t reserved;
    double point[3];
    double spring, length;             /* spring-type potentials */
    double force, reactive_distance;   /* force_flux_potential {constant_force, reactive_distance} */
} gcs_point_source_params;

/* kinetochore_fiber_forcefield::kinetochore_spec (common/forcefield/kinetochore_fiber_forcefield.hpp:14-20) */
typedef struct gcs_kinetochore_spec {
    int64_t particle_index;
    double mobility;
    double decay_rate;
    double stationary_length;
} gcs_kinetochore_spec;

/* Driver context (common/simulation_context.hpp:7-18) plus the last force evaluation's statistics. */
typedef struct gcs_context {
    int64_t step;              /* last completed step */
    double time;
    double core_scale;
    double bond_scale;
    double wall_semiaxes[3];
    double inward_reaction[3]; /* ellipsoid_inward stats.axial_reaction of the last force evaluation */
    double outward_reaction[3];
    double last_timestep;      /* timestep actually used by the last step (spacestep may shrink it) */
} gcs_context;

/* Device-resident replacement of the per-step callback's state updates
 * (stage_interphase/simulation_driver_interphase.cpp:16-17, 51-52, 67-90). */
typedef struct gcs_schedule {
    int32_t update_time;   /* time = step * timestep */
    int32_t update_scales; /* core/bond scale = 1 - (1 - init) exp(-time / tau) */
    int32_t update_wall;   /* semiaxes += timestep * wall_mobility * (R_in + R_out - spring o semiaxes) */
    int32_t reserved;
    double timestep;
    double core_scale_init, core_scale_tau;
    double bond_scale_init, bond_scale_tau;
    double wall_semiaxes_spring[3];
    double wall_mobility;
} gcs_schedule;

/* md::brownian_dynamics_config {temperature, timestep, spacestep, steps, seed} */
typedef struct gcs_bd_config {
    double temperature;
    double timestep;
    double spacestep; /* > 0: the step's timestep is reduced so that max_i |mu_i F_i| dt <= spacestep */
    uint64_t seed;
    int32_t noise;    /* GCS_NOISE_* */
    int32_t reserved;
} gcs_bd_config;

/* Per-kernel timing probe (HIP events on the engine stream around every launch of each kernel). */
typedef struct gcs_profile {
    int64_t steps;
    double total_ms;          /* wall time of the probed steps (events around the whole loop) */
    double force_ms;          /* average duration of one force/integrate launch */
    double cell_ms;           /* average duration of the cell-list build (count + scan + scatter + sort) */
    double tail_ms;           /* average duration of the schedule tail launch (fused step: the last-block
                                 tail + cell-scan section inside the force launch, last step) */
    double mean_neighbors;    /* mean number of neighbours within the cutoff per particle (last step) */
} gcs_profile;

const char* gcs_last_error(void);
int gcs_abi_version(void);
int gcs_device_count(int32_t* count);

int gcs_engine_create(const gcs_system_desc* desc, gcs_engine** out);
int gcs_engine_destroy(gcs_engine* engine);
int gcs_engine_particle_count(const gcs_engine* engine, int64_t* count);
/* the engine's arithmetic precision in bits (32 or 64) */
int gcs_engine_precision(const gcs_engine* engine, int32_t* bits);

/* force fields; *handle receives an id usable with gcs_remove_forcefield */
int gcs_add_neighbor_softcore(gcs_engine* e, const gcs_softcore_params* p, int32_t* handle);
int gcs_add_neighbor_softwell(gcs_engine* e, const gcs_softwell_params* p,
                              const int64_t* targets, int64_t n_targets, int32_t* handle);
/* bonds: for each range [begin, end) the pairs (k, k + stride) with begin <= k, k + stride < end,
 * plus the explicit pairs. stride 1 = add_bonded_range; stride 2 = the i, i+2 loop bonds. */
int gcs_add_bonded_pairwise(gcs_engine* e, const gcs_bond_params* p,
                            const int64_t* ranges, int64_t n_ranges, int32_t stride,
                            const int64_t* pairs, int64_t n_pairs, int32_t* handle);
/* cosine bending U = energy (1 - cos theta) over the triples (k, k+1, k+2) inside each range */
int gcs_add_bonded_triplewise(gcs_engine* e, double bending_energy,
                              const int64_t* ranges, int64_t n_ranges, int32_t* handle);
int gcs_add_ellipsoid_inward(gcs_engine* e, const gcs_wall_params* p, int32_t* handle);
int gcs_add_ellipsoid_outward(gcs_engine* e, double spring, const double center[3], int32_t* handle);
int gcs_add_point_source(gcs_engine* e, const gcs_point_source_params* p, int32_t* handle);
int gcs_add_kinetochore_fiber(gcs_engine* e, const double pole[3],
                              const gcs_kinetochore_spec* specs, int64_t n_specs, int32_t* handle);
int gcs_remove_forcefield(gcs_engine* e, int32_t handle);

int gcs_engine_set_positions(gcs_engine* e, const double* xyz, int64_t n);
int gcs_engine_get_positions(gcs_engine* e, double* xyz, int64_t n);
int gcs_engine_set_context(gcs_engine* e, const gcs_context* ctx);
int gcs_engine_get_context(gcs_engine* e, gcs_context* ctx);
int gcs_engine_set_schedule(gcs_engine* e, const gcs_schedule* s);
/* Apply the schedule once for `step` with the current reaction statistics (the driver's callback(0)). */
int gcs_engine_apply_schedule(gcs_engine* e, int64_t step);

/* Injected normals, [steps][N][3] in the order the reference integrator draws them; consumed by
 * subsequent GCS_NOISE_INJECTED runs. */
int gcs_engine_set_noise(gcs_engine* e, const double* normals, int64_t steps);

/* Advance steps first_step+1 .. first_step+steps.  After each step the schedule is applied with that
 * step's index (the reference callback order).  Asynchronous w.r.t. the host until a get_* call. */
int gcs_engine_run(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps);
int gcs_engine_synchronize(gcs_engine* e);

/* Total potential energy (md::system::compute_energy) and, if per_kind != NULL, a breakdown
 * [pair, softwell, bonds, bending, wall_in, wall_out, point_source, kinetochore_fiber]. */
int gcs_engine_compute_energy(gcs_engine* e, double* total, double* per_kind);
/* Forces on every particle at the current positions/context ([N][3]); refreshes reaction stats. */
int gcs_engine_compute_forces(gcs_engine* e, double* forces, int64_t n);

/* Pairs (i < j) of `points` closer than `distance` (the strict predicate (dx^2 + dy^2) + dz^2 < distance^2 with
 * every operation rounded, in the engine's precision), sorted by (i, j).  points == NULL searches the
 * engine's current positions. pairs receives [count][2]. */
int gcs_engine_search_neighbors(gcs_engine* e, const double* points, int64_t n, double distance,
                                uint32_t* pairs, int64_t capacity, int64_t* count);

int gcs_engine_profile(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps,
                       gcs_profile* out);

/* Contact map (replaces contact_map::update / accumulate / clear, stage_interphase/contact_map.cpp:28-85, driven
 * from stage_interphase/simulation_driver_interphase.cpp:38-45).  update: count every pair i < j of the CURRENT positions closer
 * than `distance` (the strict predicate of gcs_engine_search_neighbors) into the engine's device hash map;
 * enqueued on the engine stream, no host synchronisation (call it between gcs_engine_run chunks).
 * read: the accumulated (i, j, count) triples sorted by (i, j) into ijc[count][3] (count = distinct pairs;
 * GCS_ECAPACITY with *count set when capacity is too small, GCS_ECAPACITY without a count when the map
 * overflowed — raise GCS_OPT_CONTACT_BITS).  clear: empty the map. */
int gcs_engine_contacts_update(gcs_engine* e, double distance);
int gcs_engine_contacts_read(gcs_engine* e, uint32_t* ijc, int64_t capacity, int64_t* count);
int gcs_engine_contacts_clear(gcs_engine* e);

/* Sampled positions as simulation_store::save_positions writes them (common/simulation_store.cpp:22-33,
 * 192-216): every coordinate quantised to `fraction_bits` mantissa bits (16 in the reference), as f32 [N][3]. */
int gcs_engine_sample_positions(gcs_engine* e, float* xyz, int64_t n, int32_t fraction_bits);

/* Spatial domain decomposition (C5: one trajectory over several GPUs; SURVEY.md 8e, DESIGN.md "Multi-GPU").
 * Every engine holds all N particles by global index and integrates those that lie in its box
 * box = {lo[3], hi[3]} ([lo, hi) per axis; the domains' boxes tile space, outer faces at +-inf) at the start of a
 * step; the particles within `halo` of the box (its region) are kept fresh by the owners' bands, and the list step
 * bins those within list radius + one skin of the box (the tile step the whole region).  `peer_boxes` [npeer][6] are the boxes of
 * the domains whose regions overlap this one's: after each step the band of owned particles whose old or new
 * position lies in a peer's region (its box extended by `halo`) is packed for that peer.  Every engine derives the
 * regions with one fp32 formula, so membership is bit-identical on both sides.  `index` / `ndomains`: this domain's number and the domain
 * count (one slot each in the allreduce buffer).  halo <= 0 turns decomposition off.
 * The step shape follows the engine's: the list step (GCS_OPT_FUSED_STEP 3, the default) when the halo holds the
 * list radius (cutoff + skin at core scale 1), the tile step (fp32 engines only) otherwise.  Band records are in the
 * engine's precision: {x, y, z, index bits} as 4 floats (fp32 engine) or 4 doubles (fp64; the index in the low word
 * of the fourth), the count of a band in the first int of its header row.
 * One step = gcs_engine_domain_step (force + update of the owned particles, local reduction into
 * dev_reaction[nred] on the device) -> the caller's allreduce(sum) of dev_reaction over all domains ->
 * gcs_engine_domain_finish(allreduced buffer: wall ODE + schedule) -> gcs_engine_domain_pack (band records
 * {x, y, z, index bits} into dev_out[npeer][cap][4] floats or doubles, counts per peer; dev_flags[0] |= 1 a bond longer than the
 * halo, |= 2 a band over cap, |= 4 a particle owned by no domain's lists, |= 8 cutoff + largest displacement since
 * the last list build beyond the halo) -> exchange -> gcs_engine_domain_unpack(received buffers).  All calls only
 * enqueue on the engine stream (gcs_engine_stream), so the caller's collectives can be ordered on it too.
 * Replaces nothing in the reference (single-threaded); the per-step callback order is kept (wall update after
 * the force evaluation of the step, stage_interphase/simulation_driver_interphase.cpp:51-52, 80-90). */
int gcs_engine_set_domain(gcs_engine* e, const double* box /* [6] */, double halo,
                          const double* peer_boxes /* [npeer][6] */, int32_t npeer, int32_t index, int32_t ndomains);
/* Shared particles: fresh on every domain every step (carried in the reaction allreduce, which then holds
 * 10 + 3 * count + ndomains doubles).  For particles whose bonds are too soft for any practical halo (nucleolar
 * beads and their NOR partners; nucleolus_bond_spring 10 vs chain 50-100). */
int gcs_engine_set_domain_shared(gcs_engine* e, const int64_t* idx, int32_t count);
int gcs_engine_stream(gcs_engine* e, void** stream);
int gcs_engine_domain_step(gcs_engine* e, const gcs_bd_config* cfg, int64_t step, double* dev_reaction);
int gcs_engine_domain_finish(gcs_engine* e, const double* dev_reaction);
int gcs_engine_domain_pack(gcs_engine* e, void* dev_out, int32_t* dev_counts, int32_t cap, int32_t* dev_flags);
int gcs_engine_domain_unpack(gcs_engine* e, const void* dev_in, const int32_t* dev_counts, int32_t nbuf,
                             int32_t cap);

/* Engine-owned exchange of a decomposed run (C5): band buffers of `cap` records per peer (the band's first row
 * holds its count, so one message per peer carries both), the reaction/shared-position allreduce buffer of
 * *nred doubles, the overflow flags.  After gcs_engine_set_domain / _set_domain_shared. */
int gcs_engine_domain_buffers(gcs_engine* e, int32_t cap, int32_t* nred);
/* RCCL transport (one domain per GPU): rank 0 draws the communicator id, the host hands it to every rank over any
 * channel; peer_ranks[p] is the rank of the p-th peer region given to gcs_engine_set_domain.  librccl.so.1 is
 * opened at first use. */
int gcs_rccl_unique_id(uint8_t* id /* [128] */);
int gcs_engine_domain_rccl(gcs_engine* e, const uint8_t* id, int32_t nranks, int32_t rank, const int32_t* peer_ranks);
/* `steps` decomposed steps on the engine stream: per step the domain kernels, ncclAllReduce of the reaction buffer
 * (simulation_driver_interphase.cpp:80-90 sees the sum over domains), the tail, then one grouped ncclSend/ncclRecv
 * of the band with each peer and the unpack; chunks of GCS_OPT_GRAPH_STEPS steps are captured in a hipGraph. */
int gcs_engine_domain_run(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps);
/* Host-staged transport (tests; any process layout, e.g. several processes on one device): a step's halves with
 * host buffers -- the local reduction out, the summed one in; the bands out ([npeer][cap + 1][4] floats, doubles for
 * an fp64 engine) and in.  With these engine-owned buffers the list step packs its bands itself (k_lstep). */
int gcs_engine_domain_step_host(gcs_engine* e, const gcs_bd_config* cfg, int64_t step, double* red, int32_t nred);
int gcs_engine_domain_finish_host(gcs_engine* e, const double* glob, int32_t nred);
int gcs_engine_domain_pack_host(gcs_engine* e, void* bands /* NULL: pack on the device only */);
int gcs_engine_domain_unpack_host(gcs_engine* e, const void* bands);
/* In-process transport (several domains on one device): copy src's band src_slot into dst's received band
 * dst_slot (ordered after src's stream), then unpack everything received. */
int gcs_engine_domain_receive(gcs_engine* dst, int32_t dst_slot, gcs_engine* src, int32_t src_slot);
int gcs_engine_domain_unpack_received(gcs_engine* e);
int gcs_engine_domain_flags(gcs_engine* e, int32_t* flags);

/* tuning knobs */
#define GCS_OPT_GRAPH_STEPS 1   /* steps captured per hipGraph replay (0 = eager launches) */
#define GCS_OPT_WAVES_PER_TILE 2 /* waves sharing one 64-particle tile of the pair loop: 1, 2, 4 or 8 */
#define GCS_OPT_CHUNK_ORDER 3    /* pair-loop candidate chunks: 0 contiguous, 1 strided across stencil rows (default) */
#define GCS_OPT_FUSED_STEP 4     /* 3 (default): neighbour-list step (1 launch per step + a list rebuild every few
                                    steps; systems with > 256 pair classes or >= 2^24 particles: fp32 step 2, fp64
                                    step 0); 0 unfused (a fresh cell list every step; fp64: k_eval64 + k_red64 +
                                    k_update + k_tail); fp32 only: 2 launches per step (force + cell-list rebuild) */
#define GCS_OPT_SPLIT_TILES 5    /* step launches: 0 (default) off, 1 split every tile over two workgroups, 2 only the
                                    densest tiles, picked by the cell scan within the resident-workgroup budget */
#define GCS_OPT_SUBTILES 7       /* pair-loop stencils per 64-particle tile: 1, 2 or 4 (default 2) */
#define GCS_OPT_SCAN_BLOCKS 8    /* cell scan: 1 = multi-block look-back scan (default), 0 = one workgroup */
#define GCS_OPT_TILE_PRIORITY 6  /* n > 0: pair-loop wave priority min(3, tile candidates / n); 0 = off (default 700) */
#define GCS_OPT_CONTACT_BITS 9   /* contact map: 2^bits hash slots (0 = default: >= 256 N slots, <= 2^28, sized at the first update) */
#define GCS_OPT_LIST_SKIN 10      /* list step: skin in 1/1000 of the pair cutoff (0 = default: 500 fp32, 350 fp64 at core
                                     scale 1; x core scale (fp32) / sqrt(core scale) (fp64) while a schedule grows it: 250 / 250 at 0.5) */
#define GCS_OPT_LIST_EVERY 11     /* list step: rebuild period in steps (0 = default: from the noise amplitude) */
#define GCS_OPT_LIST_CAP 12       /* list step: list entries per particle (default 1024; a longer list: exact search) */
#define GCS_OPT_LIST_WAVES 13     /* list step: waves per 64-particle tile, 4 (default: lowest step latency) or 2 (more
                                     tiles resident: the better throughput when several trajectories share a GPU) */
#define GCS_OPT_DENSE_NEIGHBORS 15 /* fp32 list step (GCS_OPT_FUSED_STEP 3): a fresh run whose mean neighbour count within the
                                     cutoff, x 2 when list entries are 32-bit (GCS_OPT_LIST_FORMAT 2), exceeds this takes the
                                     unfused tile step instead (default 96; 0: never) */
#define GCS_OPT_LIST_DEAL 16      /* list build: which wave segment takes each candidate chunk; -1 (default) the tuned
                                     pattern for the waves per tile, 0 round robin, else period T (1..15) << 60 | the
                                     wave (< waves per tile) of chunk p of each period in nibble p.  Only the split of
                                     a slot's list over the segments changes (the list step's last wave also carries
                                     the particle-local terms); the pair set and the results do not */
#define GCS_OPT_LIST_FORMAT 17    /* list entries: 0 (default) 16-bit absolute slots up to 65,536 particles, the relative
                                     form beyond; 1 16-bit slots relative to the particle's cell planes (an entry out of
                                     their range sends the particle to the exact search); 2 32-bit absolute slots.  Every
                                     form holds the same pairs in the same order: the results do not change */
#define GCS_OPT_SMALL_STEP 18     /* systems of <= 1,536 particles (the mitotic stages): 1 (default) one cooperative launch
                                     per chunk of steps, every workgroup holding the whole system in LDS (all pairs; the
                                     new positions handed between workgroups as tagged granules every step), unless
                                     GCS_OPT_FUSED_STEP was set; 0 the step shapes above */
#define GCS_OPT_LIST_PHASE 19     /* list step: rebuild at the steps s with (s + phase) % period == 0 (default 0).  Several
                                     trajectories sharing a GPU (bench.py's replicas) stagger their rebuilds with it, so
                                     one's short cell kernels overlap the others' step kernels; a trajectory is bitwise
                                     reproducible for a given phase (its lists' entry order, hence its sums' order,
                                     follows the rebuild steps) */
#define GCS_OPT_LIST_SKIN_BASE 20 /* list step: the skin at core scale 1 that the default skin follows (s1 sqrt(cs) at fp64,
                                     s1 cs at fp32; 0 = the precision's default, 350 / 500 per mille).  The default
                                     suits several trajectories per GPU; one trajectory alone (the stage drivers) is
                                     latency-bound and prefers longer lists and fewer rebuilds.  Set before a
                                     decomposed engine's domain (it sizes the binning halo) */
int gcs_engine_set_option(gcs_engine* e, int32_t option, int64_t value);

/* List-step diagnostics (the neighbour lists md::neighbor_searcher keeps between rebuilds; micromd, called at
 * stage_interphase/simulation_driver_interphase.cpp:57-63). */
typedef struct gcs_list_stats {
    int32_t active;                   /* 1: the engine runs the list step (GCS_OPT_FUSED_STEP 3, system admits it) */
    int32_t rebuild_every;            /* steps between list rebuilds of the last run */
    int64_t builds;                   /* list builds so far */
    int64_t fallback_particle_steps;  /* particle-steps evaluated by the exact cell search instead of the list */
    double skin;                      /* list radius - pair cutoff */
    double max_displacement;          /* largest displacement of a particle since the last build */
    int32_t pair_classes;             /* distinct (a, b) pair-factor classes */
    int32_t capacity;                 /* list entries per particle */
    int64_t sync_stalls;              /* multi-block cell-scan look-backs that gave up waiting; must stay 0 */
    int64_t deal;                     /* the chunk deal the list build applies (GCS_OPT_LIST_DEAL resolved) */
} gcs_list_stats;
int gcs_engine_get_list_stats(gcs_engine* e, gcs_list_stats* out);

/* How gcs_engine_run / gcs_engine_domain_run issued their steps (cumulative over the engine's life): steps
 * replayed from captured hipGraphs (any stretch of up to GCS_OPT_GRAPH_STEPS steps, captured once per rebuild
 * phase, starting buffer parity, length and whether its first step counts a deferred contact update) and steps
 * launched eagerly (a run start's forced list rebuild, GCS_OPT_GRAPH_STEPS 0).  Replaces nothing in the reference (the
 * integrator loop of micromd, stage_interphase/simulation_driver_interphase.cpp:57-63, has no launches). */
typedef struct gcs_run_stats {
    int64_t graph_launches;   /* hipGraphLaunch calls */
    int64_t graph_steps;      /* steps inside those replays */
    int64_t eager_steps;      /* steps launched one by one */
    int64_t graphs_captured;  /* captures (a cache miss: new phase / parity / length, or changed settings) */
    int64_t graphs_cached;    /* captured sequences held now */
    int64_t fused_contact_steps; /* list steps that counted a deferred contact update (gcs_engine_contacts_update) */
    int64_t density_probes;   /* fresh fp32 chains whose mean neighbour count was probed (GCS_OPT_DENSE_NEIGHBORS) */
} gcs_run_stats;
int gcs_engine_get_run_stats(gcs_engine* e, gcs_run_stats* out);

/* Restrict the engine's stream to a set of compute units (bit i of mask[i / 32] = CU i; words = 0: all CUs), e.g.
 * one group of XCDs per trajectory when several share a GPU.  Recreates the stream: call between runs. */
int gcs_engine_set_cu_mask(gcs_engine* e, const uint32_t* mask, int32_t words);

#ifdef __cplusplus
}
#endif

#endif /* GCS_H */
