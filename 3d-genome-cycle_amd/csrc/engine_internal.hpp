// engine_internal.hpp -- device-side data layout and kernel interfaces of the gcs engine (gfx950).
//
// HBM layout (fp32, 16-B aligned rows so every particle access is one dwordx4):
//   pos[2][N]   float4 {x, y, z, 0}      double-buffered particle positions, particle order
//   kmu[N]      float4 {mu, a, b, t}     per-particle constants (mobility, A/B factors, t = 1: droplet target)
//   spos[N]     float4 {x, y, z, a}      positions re-ordered by cell (rebuilt every step)
//   sb[N], sidx[N], scell[N]             b factor, particle index and cell of each sorted slot
//   cstart[ncell+1]                      first sorted slot of each cell (cell = x + nx (y + ny z))
//   bonded CSR (boff/bent/bval), bend_eps[N], tether CSR (toff/tent)   topology, particle order
//   DevCtx                               device-resident driver context + the current cell grid
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gcs {

constexpr int kTile = 64;          // particles per tile of the pair loop = one wave's lanes
constexpr int kMaxRows = 64;       // stencil rows per batch of the pair loop's row table
constexpr int kPairFx = 2;         // x subdivision of the pair cell grid
constexpr int kMaxUnits = 8192;  // heavy-tile unit table / split budget capacity
constexpr int kBucketCap = 16;   // particles filed per cell by the rebuild step's binning (more: overflow list)
constexpr int kScanSeg = 16;        // cells per thread per iteration of the cell scan
constexpr int kScanPad = kScanSeg * 1024 + 8;  // count/cstart padding: the scan touches whole iterations (<= 1024 threads)
constexpr int kMaxPointSources = 4;
constexpr int kForcePartials = 8;  // per force block: reaction in[3], out[3], max mu|F|, neighbours
constexpr int kBBoxPartials = 6;   // per block: bbox lo[3], hi[3]
constexpr int kBBoxStride = 8;     // row stride of the bbox partials (rows of 8: one component per lane & 7)
constexpr int kEnergyKinds = 8;
constexpr unsigned long long kContactEmpty = ~0ull;  // contact-map hash table: free slot
constexpr int kContactMaxProbe = 4096;               // linear-probe bound of one insert (then: overflow flag)

// Count one contact pair (key = i << 32 | j) into the open-addressing table (Fibonacci hash onto 2^bits slots, linear
// probing).  Each probed key is LOADED first and claimed by CAS only when the slot is empty: a key never moves or
// leaves its slot between clears (a memset between launches), so a load can be stale only as "empty", which the
// CAS then settles; a pair already in the table (the common case: the same contacts recur every update of a window)
// costs one atomic instead of two.  false: kContactMaxProbe slots probed without a place (the caller flags overflow).
__device__ __forceinline__ bool contact_count(unsigned long long* keys, unsigned* counts, int bits,
                                              unsigned long long key)
{
    const unsigned long long mask = (1ull << bits) - 1ull;
    unsigned long long h = (key * 0x9E3779B97F4A7C15ull) >> (64 - bits);
    for (int probe = 0; probe < kContactMaxProbe; ++probe) {
        unsigned long long cur = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == kContactEmpty) cur = atomicCAS(&keys[h], kContactEmpty, key);
        if (cur == kContactEmpty || cur == key) {
            atomicAdd(&counts[h], 1u);
            return true;
        }
        h = (h + 1) & mask;
    }
    return false;
}

struct Grid {
    float lo[3];
    float inv[3];
    int n[3];
    int ncell;
    int fx;     // x cell edge = rc / fx (the pair stencil spans +-fx cells in x, +-1 in y and z)
    float rc;   // pair cutoff of this step
    float rc2;
};

struct DevCtx {
    double time, cs, bs;
    double wall[3];
    double react_in[3], react_out[3];
    double dt_used;
    double max_drift;      // max_i mu_i |F_i| of the last force evaluation (spacestep)
    double neighbors;      // mean neighbours within the cutoff per particle (last force evaluation)
    long long step;        // last completed step
    long long noise_cursor;
    int parity;            // index of the current position buffer
    int ntiles;            // k_force tiles of the current cell list (k_cell_scan)
    float bbox_lo[3], bbox_hi[3];
    Grid grid;             // bins the current positions (the next force evaluation's stencil)
    Grid grid_next;        // bins the positions the next step produces (fused path)
    unsigned ticket;       // arrival counter of the fused force kernel's blocks (0 between launches)
    int scan_stall;        // multi-block cell scans whose look-back gave up waiting (must stay 0)
    int units_ok;          // the last cell scan wrote the heavy-tile unit table (ForceArgs::units)
    int nunits;            // its length
    int nactive;           // workgroups of the last force launch that had work (its partial rows)
    int pad3;
    unsigned long long t_tail[2];  // wall clock at the start / end of k_tail
    unsigned long long t_rows[8];  // wall clock probes inside the cell scan's row pass (GCS_DEBUG)
    unsigned long long t_cells[8];  // wall clock probes inside the cell scan's cell pass (GCS_DEBUG)
    unsigned long long t_last[4];  // wall clock: fused last-block section start, after tail, after scan, end
    // rebuild step (GCS_OPT_FUSED_STEP 2): what the step's force kernel binned with, stashed by its block 0 so the
    // rebuild kernel reads them while that kernel's tail block advances grid / parity / step
    Grid rb_grid;
    long long rb_step;
    int rb_parity;
    int pad4;
    // list step (GCS_OPT_FUSED_STEP 3): the grid the neighbour lists were built on (its rc = build cutoff + skin),
    // the build cutoff, the largest displacement of any particle from its build position (the last tail's
    // reduction), cumulative list builds and fallback particle-steps (diagnostics)
    Grid lgrid;
    float lrc_b;
    float ldisp;
    long long lbuilds;
    long long lfallback;
    int lnslots;  // slots of the current lists (binned particles: N, or a decomposed domain's owned + ghosts)
    float contact_d2;  // the squared distance of the contact update a list step counts (k_set_contact, fp32 product)
    double contact_d2_64;  // the same in fp64 (the fp64 list step's predicate; k_set_contact, fp64 product)
};

// an axis-aligned box [lo, hi) (a decomposed domain's own box, or a peer's region: its box extended by the halo)
struct DomBox {
    float lo[3], hi[3];
};
__host__ __device__ inline bool box_has(const DomBox& b, float x, float y, float z)
{
    return x >= b.lo[0] && x < b.hi[0] && y >= b.lo[1] && y < b.hi[1] && z >= b.lo[2] && z < b.hi[2];
}

enum BondType : int { kSemispring = 0, kHarmonic = 1, kSpring = 2, kSoftwell = 3 };

struct BondParam {
    int type, mix, scaled, pad;
    double ka, kb, la, lb;  // softwell: ka = energy, kb = 1/decay^2, la = cutoff^2
};

// Arithmetic precision (gcs_system_desc::precision).  The reference computes in double (md::scalar; e.g.
// stage_transition/transition_interphase.cpp:38 brace-inits md::point from doubles): GCS_PRECISION_F64 runs the list
// step, the particle-local terms, the integrator, the force / energy evaluations, the neighbour predicate and the
// contact map in fp64 on fp64 positions; GCS_PRECISION_F32 is the fp32 engine (and the only one with the tile-step
// shapes).  Kernels shared by both are templated on the scalar R; real4<R> is the 16- or 32-byte position record.
template <typename R> struct RealVec;
template <> struct RealVec<float> { using v4 = float4; using v2 = float2; };
template <> struct RealVec<double> { using v4 = double4; using v2 = double2; };
template <typename R> using real4 = typename RealVec<R>::v4;
template <typename R> using real2 = typename RealVec<R>::v2;
// the .w word of a slot-ordered position or a band record: an integer's bits (fp64: in the low word of the double)
__device__ __forceinline__ int wbits(float w) { return __float_as_int(w); }
__device__ __forceinline__ int wbits(double w) { return (int)__double_as_longlong(w); }
template <typename R> __device__ __forceinline__ R wpack(int v)
{
    if constexpr (sizeof(R) == 4) return __int_as_float(v); else return __longlong_as_double((long long)(unsigned)v);
}
template <typename R> __device__ __forceinline__ real4<R> mk4(R x, R y, R z, R w)
{
    if constexpr (sizeof(R) == 4) return make_float4(x, y, z, w); else return make_double4(x, y, z, w);
}

template <typename R>
struct TetherT {  // kinetochore fiber spring to a fixed pole
    R px, py, pz, k, l, pad0, pad1, pad2;
};
using Tether = TetherT<float>;

template <typename R>
struct PointSrcT {
    int type;      // GCS_POT_*
    R px, py, pz, k, l, f, b;
};

template <typename R>
struct WallInT {
    R a_eps, a_sig, b_eps, b_sig, wall_a, wall_b, cx, cy, cz;
    int mix, scaled;
};

// every scalar parameter of the compiled force fields and the BD config, once per precision (ForceArgs::pf / pd)
template <typename R>
struct FieldPrm {
    R pa_eps, pa_sig, pb_eps, pb_sig, pair_dist;  // neighbour soft-core
    R sw_ka, sw_kb, sw_la;                        // droplet softwell: energy, 1 / decay^2, cutoff^2
    PointSrcT<R> point[kMaxPointSources];
    WallInT<R> win;
    R wout_k, wout_cx, wout_cy, wout_cz;
    R temperature, timestep;
};

enum Mode : int { kModeStep = 0, kModeForce = 1, kModeEnergy = 2, kModeList = 3 };  // kModeList: build the neighbour lists

struct ForceArgs {
    int n;
    // state
    float4* pos0;
    float4* pos1;
    const float4* kmu;
    const float4* spos;
    const float* sb;
    const int* sidx;
    const int* scell;
    const int* cstart;
    const int2* tile_range; // [tiles] sorted-slot range [begin, end) of each k_force tile (k_cell_scan)
    // neighbor soft-core pair field
    int has_pair, pair_mix, pair_scaled, chunk_mode;
    // the fields' scalar parameters at each precision (the fp32 kernels read pf, the fp64 ones pd)
    FieldPrm<float> pf;
    FieldPrm<double> pd;
    int prec;  // 32 or 64: which of the state pointers below hold the system (GCS_PRECISION_*)
    // bonded CSR (particle order)
    int has_bonds;
    const int* boff;
    const int2* bent;
    const float4* bval;  // per CSR entry: {K, l, 0, 0} (A/B mixed at compile), softwell {energy, 1/decay^2, cutoff^2, 0};
                         // bent[q] = {partner, type | scaled << 4}
    // the nucleolar droplet (a softwell among <= 64 targets): evaluated wave-cooperatively (local_terms), not
    // through the bond CSR; targets carry kmu[i].w = 1
    int sw_n;
    const int* sw_idx;
    // the list step's slot-indexed partners (engine.hip slot_bonds; nullptr: by particle index): per bond CSR entry q
    // the slot of its partner bent[q].x, per droplet target t the slot of sw_idx[t] -- filed by k_cell_sort at every
    // rebuild -- so the particle-local terms read the slot-order positions (psort) and the particle-order copy need be
    // written only before a rebuild and at the end of a stretch of steps (kLFlagPos)
    const int* bslot;
    const int* swslot;
    // bending
    int has_bend;
    const float* bend_eps;
    // kinetochore fibers
    int has_tether;
    const int* toff;
    const Tether* tent;
    // point sources
    int n_point;
    // ellipsoid walls
    int has_wall_in, has_wall_out;
    // Brownian dynamics
    unsigned seed_lo, seed_hi;
    int noise_mode;
    const float* noise;
    long long noise_steps;
    // outputs
    float* part_force;    // [blocks][kForcePartials]
    float* part_bbox;     // [blocks][kBBoxStride] (kBBoxPartials used)
    double* part_energy;  // [blocks][kEnergyKinds]
    float4* force_out;    // [N] (kModeForce)
    // fused step (kModeStep, FUSED): binning of the new positions + last-block tail and cell scan
    int* cell_of;
    int* slot;
    int* count;
    int* cstart_w;
    int* tile_start_w;
    int2* tile_range_w;
    const double* sched;
    int ncell_max;
    int apply_sched;
    int subtiles;   // pair-loop stencil groups per tile: 1, 2 or 4 (GCS_OPT_SUBTILES)
    int prio_step;  // > 0: wave priority = min(3, candidates / prio_step) (GCS_OPT_TILE_PRIORITY)
    int split;      // step launches: 1 split every tile in two units, 2 the heavy ones the scan picks (GCS_OPT_SPLIT_TILES)
    const int4* units;  // [units] {s_begin, s_end, tile, part | nparts << 8} (split == 2)
    int split_cap;  // tiles that may be split (pbuf / tcnt capacity)
    float4* pbuf;   // [2 * split_cap][kTile] partial forces of split units
    int* tcnt;      // [split_cap] arrival counters of split tiles (0 between launches)
    unsigned long long* dbg_build;  // optional (GCS_DEBUG_BUILD): k_lbuild per workgroup {start, tile end, wave 0..3
                                    // sweep end, candidates, tile} of the first tile
    unsigned long long* dbg_times;  // optional (GCS_DEBUG_TIMES): per block {start, end, smid/candidates, tile} then 4 phase stamps
    // rebuild step: the force kernel files each new position's sorted record under its cell: bucket_p / bucket_q
    // [c][slot] = {x, y, z, a factor} / {particle, b factor bits} for slot < kBucketCap, the rest on the overflow
    // list ovf_p / ovf_q ({particle, b bits, cell, 0}) counted in ovf_n[step & 1]; bucket_p == nullptr: slot binning
    float4* bucket_p;
    int2* bucket_q;
    float4* ovf_p;
    int4* ovf_q;
    int* ovf_n;
    // spatial domain decomposition (C5; DESIGN.md "Multi-GPU"): every engine holds all N particles by global index;
    // it integrates only the particles it OWNS (inside its box `dom` at step start) and bins only those within
    // dom_halo of the box (owned + ghosts, refreshed every step by the owners' band exchange).  dom_on == 0: off.
    int dom_on;
    DomBox dom;
    float dom_halo;      // the exchange halo: a peer receives the owned particles within it of its box (bond reach)
    float dom_bin_halo;  // the binning halo (<= dom_halo): the decomposed list step bins only the ghosts within the
                         // list radius + a skin of the box; the motion check holds cutoff + displacement below it
    const double* ext_react;  // != nullptr: the step's wall reaction summed over all domains (allreduced), [6]
    // decomposed list step: the local reduction goes to dom_red (layout kDomainRed), the per-domain slot of the
    // largest displacement at dom_red[dom_dbase + dom_index] (dom_ndom slots: a sum-allreduce carries the max);
    // islot[i]: particle i's slot in the current lists (-1: not binned), written by the rebuild
    double* dom_red;
    int dom_dbase, dom_index, dom_ndom;
    int* dom_flags;
    int* islot;
    // the band pack and the shared particles' positions fused into k_lstep<..., DOM> (the engine's RCCL run;
    // dom_bands == nullptr: the separate k_domain_pack / k_domain_shared_out launches): each owned particle's record
    // {new x, y, z, index} goes to every peer p whose region holds its old or new position (band p's records at
    // dom_bands[p * dom_bstride + 1 + k], k < cap, its count in the header row p * dom_bstride, zeroed by the previous
    // step's unpack), an owned shared particle's new position into its row of dom_red's shared block (k_ldom_tail
    // zeroes the block for the next step), and a bond of an owned particle reaching beyond the halo raises
    // dom_flags bit 0 (the local-terms wave)
    void* dom_bands;  // real4<R> records
    int dom_bstride, dom_cap, dom_npeer;
    const DomBox* dom_regions;
    const int* dom_shared;  // [N] k + 1 for the k-th shared particle, 0 otherwise
    // list step (GCS_OPT_FUSED_STEP 3; DESIGN.md "The list step"): per sorted slot s and wave w (w < 4) the
    // sorted slots of the pair partners found within build cutoff + list_skin are
    // list[(w * list_cap + k) * list_stride + s], k < count, count = lcount[w * list_stride + s] & kListCountMask
    // (bit 30: some wave of the slot overflowed list_cap).  psort[2]: the current positions in sorted-slot order
    // (ping-pong with ctx->parity), .w = particle | class << 24 (class: the (a, b) pair factors, type_ab[class]).
    int* list;
    int* lcount;
    int4* lbase;            // list_fmt kListFmtRel16: per slot the partner planes' first slots (kernels.hip ListRel16)
    const int* ptype;       // [N] pair-factor class of each particle
    float4* psort0;
    float4* psort1;
    float4* skmu;           // [N] per slot: kmu of its particle (list path, k_cell_sort)
    int2* sbrow;            // [N] per slot: its particle's bond CSR row [boff[i], boff[i + 1])
    const float2* type_ab;  // [kMaxTypes] (a, b) pair factors of each class
    int ntypes;
    int list_cap;           // entries per (slot, wave)
    int list_stride;        // >= N
    float list_skin;        // > 0 only in the list path's own argument block
    int list_waves;         // waves per tile (list segments): 4, or 2 (GCS_OPT_LIST_WAVES)
    int list_fmt;           // list entries: kListFmtAbs16 / kListFmtInt / kListFmtRel16 (list_format)
    int list_nt;            // read the list words with the non-temporal hint (lists far beyond the L2s)
    // the persistent small-system step (kernels.hip k_pstep): the hand-off halves (zeroed before every launch)
    unsigned* psync;
    // k_pstep's stall word (device, zeroed by the engine): a workgroup whose hand-off poll gives up adds 1 and stops
    // integrating, every other workgroup stops at its next poll; the host fails the run (engine.hip run_small)
    int* pstall;
    int pstep_skip;  // GCS_DEBUG_PSTEP_SKIP (tests): workgroup << 16 | step that does not publish its hand-off; -1: none
    unsigned long long list_deal;  // list build: candidate chunk -> wave segment pattern (GCS_OPT_LIST_DEAL; 0: round robin)
    int par_hint;           // >= 0: ctx->parity of this launch, known to the host at enqueue (the slot loads need not
                            // wait for the context); -1: read it
    // the relaxation list step (k_lstep<..., RLX> + k_lupdate): the run's spacestep and the largest timestep
    double relax_spacestep;
    double relax_timestep;
    // the contact-map update fused into a list step (stage_interphase/contact_map.cpp:33-63): every pair i < j of
    // the step's START positions closer than sqrt(DevCtx::contact_d2) (strict fp32 predicate) is counted into the table
    int contact_on;
    unsigned long long* c_keys;
    unsigned* c_counts;
    int c_bits;
    int* c_overflow;
    unsigned* lticket;      // list step arrival counters: [32 g] per group of workgroups (g < 8), [32 * 8] groups;
                            // then the launch accumulators (kListAccBase)
    // fp64 state (prec == 64; the fp32 buffers above then hold only the cell lists and the fp32 sorted copies the
    // list build bins): positions {x, y, z, 0} in particle order (ping-pong), per-particle {mu, a, b, target}, the
    // slot-ordered positions (.w: the bits of particle | class << 24 as a 64-bit integer) and constants, the pair
    // classes' (a, b), the bond CSR values, bending, tethers, injected normals, forces, and the partial rows of
    // the fp64 force / energy evaluation ([blocks][8])
    double4* dpos0;
    double4* dpos1;
    const double4* dkmu;
    double4* dpsort0;
    double4* dpsort1;
    double4* dskmu;
    const double2* dtype_ab;
    const double4* dbval;
    const double* dbend_eps;
    const TetherT<double>* dtent;
    const double* dnoise;
    double4* dforce_out;
    double* dpart;
};

// Precision-generic access to the state of ForceArgs (St<float>: the fp32 buffers, St<double>: the fp64 ones)
template <typename R> struct St;
template <> struct St<float> {
    __host__ __device__ static float4* pos(const ForceArgs& a, int par) { return par ? a.pos1 : a.pos0; }
    __host__ __device__ static float4* psort(const ForceArgs& a, int par) { return par ? a.psort1 : a.psort0; }
    __host__ __device__ static const float4* kmu(const ForceArgs& a) { return a.kmu; }
    __host__ __device__ static const float4* skmu(const ForceArgs& a) { return a.skmu; }
    __host__ __device__ static const float2* type_ab(const ForceArgs& a) { return a.type_ab; }
    __host__ __device__ static const float4* bval(const ForceArgs& a) { return a.bval; }
    __host__ __device__ static const float* bend(const ForceArgs& a) { return a.bend_eps; }
    __host__ __device__ static const TetherT<float>* tent(const ForceArgs& a) { return a.tent; }
    __host__ __device__ static const float* noise(const ForceArgs& a) { return a.noise; }
    __host__ __device__ static float4* force(const ForceArgs& a) { return a.force_out; }
    __host__ __device__ static const FieldPrm<float>& prm(const ForceArgs& a) { return a.pf; }
    __host__ __device__ static float4* fsort(const ForceArgs&, int) { return nullptr; }
};
template <> struct St<double> {
    __host__ __device__ static double4* pos(const ForceArgs& a, int par) { return par ? a.dpos1 : a.dpos0; }
    __host__ __device__ static double4* psort(const ForceArgs& a, int par) { return par ? a.dpsort1 : a.dpsort0; }
    __host__ __device__ static const double4* kmu(const ForceArgs& a) { return a.dkmu; }
    __host__ __device__ static const double4* skmu(const ForceArgs& a) { return a.dskmu; }
    __host__ __device__ static const double2* type_ab(const ForceArgs& a) { return a.dtype_ab; }
    __host__ __device__ static const double4* bval(const ForceArgs& a) { return a.dbval; }
    __host__ __device__ static const double* bend(const ForceArgs& a) { return a.dbend_eps; }
    __host__ __device__ static const TetherT<double>* tent(const ForceArgs& a) { return a.dtent; }
    __host__ __device__ static const double* noise(const ForceArgs& a) { return a.dnoise; }
    __host__ __device__ static double4* force(const ForceArgs& a) { return a.dforce_out; }
    __host__ __device__ static const FieldPrm<double>& prm(const ForceArgs& a) { return a.pd; }
    // the fp64 list step's prefilter copy: the fp32 roundings of psort's positions (slot order, .w unused), in the
    // fp32 slot-order buffers an fp64 engine does not otherwise use; nullptr outside the list path
    __host__ __device__ static float4* fsort(const ForceArgs& a, int par) { return par ? a.psort1 : a.psort0; }
};
// a slot's new position into the slot-order buffer of parity par and, fp64, into its prefilter copy (every writer of
// psort goes through here, so the copy is the rounding of psort at every step)
template <typename R>
__device__ __forceinline__ void put_slot(const ForceArgs& a, int par, int s, const real4<R>& q)
{
    St<R>::psort(a, par)[s] = q;
    if constexpr (sizeof(R) == 8) {
        float4* const f = St<R>::fsort(a, par);
        if (f) f[s] = make_float4((float)q.x, (float)q.y, (float)q.z, 0.f);
    }
}

// list step launch accumulators behind the arrival counters in ForceArgs::lticket (unsigned words, 128 B per slot):
// per group of workgroups (b % 8) kListAccSlots slots + one overflow flag (kernels.hip list_accumulate)
constexpr int kListAccBase = 32 * 9;
constexpr int kListAccSlots = 23;
constexpr int kListTicketWords = kListAccBase + 8 * 32 * (kListAccSlots + 1);
// identity of accumulator slot k (what list_accumulate starts from)
__host__ __device__ inline unsigned long long list_acc_identity(int k)
{
    return (k >= 9 && k < 12) ? 0xffffffffull : 0ull;  // bbox lo: the largest ordered value; everything else 0
}
// the list build's default chunk deal per waves per tile (kernels.hip deal_nth; 0: round robin): the last wave, which
// also carries the step's particle-local terms, takes 1 chunk in 3 ("001") / 1 in 7 ("0120123").  Same-box A/B
// (tools/deal_sweep.sh, profiles/r03c_deal_sweep.txt): 4 replicas 5.85-6.21 -> 6.24-6.26e9, single 2.52-2.53 -> 2.60-2.61e9
constexpr unsigned long long kListDeal2 = (3ull << 60) | 0x100ull;
constexpr unsigned long long kListDeal4 = (7ull << 60) | 0x3210210ull;
constexpr int kListSkinPm32 = 500;  // default list skin, 1/1000 of the pair cutoff (GCS_OPT_LIST_SKIN 0)
constexpr int kListSkinPm64 = 350;
constexpr int kMaxListWaves = 4;  // waves per tile of the list kernels (each owns one list segment): 2 or 4
constexpr int kMaxTypes = 256;          // pair-factor classes (8 bits of a list entry)
constexpr int kListIndexBits = 24;      // particle index bits of a list entry
// list entry formats (GCS_OPT_LIST_FORMAT): 16-bit absolute slots (N <= 65,536), 32-bit absolute slots, 16-bit
// slots relative to the slot's plane bases (kernels.hip ListRel16: the default beyond 65,536 particles)
constexpr int kListFmtAbs16 = 0;
constexpr int kListFmtInt = 1;
constexpr int kListFmtRel16 = 2;
constexpr int kPMax = 1536;         // particles of the persistent small-system step (kernels.hip k_pstep: LDS images)
constexpr int kPHalfBytes = kPMax * 48 + 256 * 144;  // its hand-off buffer (psync): two halves (kernels.hip k_pstep)
constexpr int kPSyncWords = 2 * kPHalfBytes / 4;
#ifndef GCS_LIST_PREFILTER
// the fp64 list step's fp32 prefilter (kernels.hip k_lstep, PF; engine.hip keeps its fp32 slot-order copy): 0 (default:
// measured slower, DESIGN.md §4 "fp32 prefilter") gathers every list entry's fp64 record, 1 the prefilter pipeline
#define GCS_LIST_PREFILTER 0
#endif
constexpr int kListCountMask = (1 << 30) - 1;
constexpr int kListOverflow = 1 << 30;

// the decomposed runs' band unpack (domain.hip k_domain_unpack, kernels.hip k_ldom_finish): received records
// {x, y, z, index bits} of nbuf bands (band b's records at in[b * istride + k], k < counts[b * cstride] <= cap) into
// both position buffers by index and, with slots, into both slot-order buffers at the particle's list slot (islot);
// thread t of nt, grid-stride
template <typename R>
__device__ __forceinline__ void dom_unpack_records(const ForceArgs& a, const real4<R>* __restrict__ in,
                                                   const int* __restrict__ counts, int nbuf, int cap, int istride,
                                                   int cstride, int slots, int t, int nt)
{
    using R4 = real4<R>;
    for (int b = 0; b < nbuf; ++b) {
        const int c = min(counts[(size_t)b * cstride], cap);
        for (int k = t; k < c; k += nt) {
            const R4 r = in[(size_t)b * istride + k];
            const int i = wbits(r.w);
            if (i < 0 || i >= a.n) continue;
            const R4 p = mk4<R>(r.x, r.y, r.z, R(0));
            St<R>::pos(a, 0)[i] = p;
            St<R>::pos(a, 1)[i] = p;
            const int sl = slots ? a.islot[i] : -1;
            if (sl >= 0) {
                const R4 q = mk4<R>(r.x, r.y, r.z, wpack<R>(i | (a.ptype[i] << kListIndexBits)));
                put_slot<R>(a, 0, sl, q);
                put_slot<R>(a, 1, sl, q);
            }
        }
    }
}

// ---- Philox4x32-10 + Box-Muller: the production noise stream (identical on host for the oracle) ----
__host__ __device__ inline void philox4x32_10(unsigned c[4], unsigned k0, unsigned k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        unsigned long long p0 = (unsigned long long)0xD2511F53u * c[0];
        unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c[2];
        unsigned n0 = (unsigned)(p1 >> 32) ^ c[1] ^ k0;
        unsigned n1 = (unsigned)p1;
        unsigned n2 = (unsigned)(p0 >> 32) ^ c[3] ^ k1;
        unsigned n3 = (unsigned)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
    }
}

// launch wrappers (kernels.hip); those taking a ForceArgs run the precision it names (a.prec)
void launch_prime(hipStream_t s, DevCtx* ctx, const ForceArgs& a, float rc_fixed, int ncell_max, const double* sched);
// reg != nullptr: bin only the particles inside *reg (a decomposed domain's region); islot != nullptr: reset to -1
void launch_cell_count(hipStream_t s, const DevCtx* ctx, const float4* pos0, const float4* pos1, int n,
                       int* cell_of, int* slot, int* count, const DomBox* reg = nullptr, int* islot = nullptr);
void launch_cell_count(hipStream_t s, const DevCtx* ctx, const double4* pos0, const double4* pos1, int n,
                       int* cell_of, int* slot, int* count, const DomBox* reg = nullptr, int* islot = nullptr);
void launch_cell_scan(hipStream_t s, DevCtx* ctx, int n, int* count, int* cstart, int* tile_start, int2* tile_range,
                      bool use_next = false, int4* units = nullptr, int resident = 0,
                      unsigned long long* scan_sync = nullptr, int ncell_max = 0);
int scan_sync_words(int ncell_max);  // u64 words of the multi-block scan's look-back buffer
// rebuild step: cell scan + tile table + cell-sorted copies from the force kernel's buckets, and the step's tail
void launch_rebuild(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int* tmp, unsigned long long* scan_sync,
                    int fblocks, int apply_sched);
int rebuild_sync_words(int ncell_max);
int rebuild_blocks(int ncell_max);
int force_step_resident(int waves);
void launch_cell_scatter(hipStream_t s, int n, const int* cell_of, const int* slot, const int* cstart, int* tmp,
                         int* count);
void launch_cell_sort(hipStream_t s, const DevCtx* ctx, const float4* pos0, const float4* pos1, const float4* kmu,
                      int n, const int* tmp, const int* cell_of, const int* cstart, int* sidx, int* scell,
                      float4* spos, float* sb, int pair_mix, const int* ptype = nullptr, float4* psort0 = nullptr,
                      float4* psort1 = nullptr, float4* skmu = nullptr, int2* sbrow = nullptr,
                      const int* boff = nullptr, int* islot = nullptr, const int* brev = nullptr,
                      int* bslot = nullptr, const int* swt = nullptr, int* swslot = nullptr);
// fp64 positions: the fp32 sorted copies (spos / sb, what the list build bins) are their roundings; psort / skmu
// are the fp64 slot-ordered copies the fp64 list step reads
void launch_cell_sort(hipStream_t s, const DevCtx* ctx, const double4* pos0, const double4* pos1, const double4* kmu,
                      int n, const int* tmp, const int* cell_of, const int* cstart, int* sidx, int* scell,
                      float4* spos, float* sb, int pair_mix, const int* ptype = nullptr, double4* psort0 = nullptr,
                      double4* psort1 = nullptr, double4* skmu = nullptr, int2* sbrow = nullptr,
                      const int* boff = nullptr, int* islot = nullptr, float4* fsort0 = nullptr,
                      float4* fsort1 = nullptr, const int* brev = nullptr, int* bslot = nullptr,
                      const int* swt = nullptr, int* swslot = nullptr);
// list step: build the neighbour lists on the current cell list (grid rc = cutoff + skin); one step from them
void launch_list_build(hipStream_t s, DevCtx* ctx, const ForceArgs& a);
// flags: 1 apply the schedule, 2 the next step rebuilds (bounding box -> grid), 4 neighbour-count statistics,
// 8 decomposed (a.dom_on): the owned slots only, the local reduction into a.dom_red instead of the tail
void launch_list_step(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int flags);
// the relaxation (spacestep) step on the lists: forces + the adapted timestep (k_lstep<..., RLX>: forces into
// a.force_out / a.dforce_out in slot order, its final workgroup sets ctx->dt_used), then the update (k_lupdate)
void launch_list_relax(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int force_flags, int update_flags);
void launch_set_contact(hipStream_t s, DevCtx* ctx, float d2, double d2_64);
// the decomposed list step's tail from the allreduced buffer glob (one workgroup), then the shared particles'
// positions into both buffers (by index and by slot) and the send bands' header rows zeroed
// a decomposed list run's cell grid at the current list radius over the domain's local box padded by the binning
// halo (the skin changed: engine.hip enqueue_dom_list_step)
void launch_dom_grid(hipStream_t s, DevCtx* ctx, const ForceArgs& a);
void launch_list_domain_tail(hipStream_t s, DevCtx* ctx, const ForceArgs& a, const double* glob, int flags,
                             const int* shared, int nshared, void* bands, int npeer, int band_stride);
// the engine-issued RCCL list step's finish, ONE launch after both collectives: the tail of launch_list_domain_tail
// (block 0) beside the band unpack of launch_domain_unpack with slots (every block; the send bands' headers zeroed)
void launch_list_domain_finish(hipStream_t s, DevCtx* ctx, const ForceArgs& a, const double* glob, int flags,
                               const int* shared, int nshared, const void* in, const int* counts, int nbuf, int cap,
                               int istride, int cstride, void* send, int nsend, int sstride);
int list_step_grid(const ForceArgs& a);
// the persistent small-system step: `steps` steps of n <= kPMax particles in ONE cooperative launch (a.psync zeroed
// by the caller first); flags: kernels.hip kLFlagSched when the schedule applies
int launch_pstep(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int steps, int flags);
// GCS_DEBUG_POISON: fill `bytes` (a multiple of 4) with hashed garbage words
void launch_poison(hipStream_t s, void* p, size_t bytes);
// k_pstep_guard: restore 0 keeps *ctx in *keep unless *stall; restore 1 puts *keep back into *ctx if *stall
void launch_pstep_guard(hipStream_t s, DevCtx* ctx, DevCtx* keep, const int* stall, int restore);
void launch_force(hipStream_t s, int mode, int waves, DevCtx* ctx, const ForceArgs& a, bool fused);
// fp64 force / energy evaluation on the current cell list (one thread per sorted slot; kernels.hip k_eval64):
// kModeForce -> a.dforce_out + partial rows a.dpart [blocks][8] (reactions in[3], out[3], max mu|F|, neighbours),
// kModeEnergy -> a.part_energy [blocks][kEnergyKinds]
int eval64_blocks(int n);
void launch_eval64(hipStream_t s, int mode, const DevCtx* ctx, const ForceArgs& a);
// reduce the fp64 evaluation's rows (fixed order) into the context's reactions, max drift and neighbour count, and
// into react_out[6] when given (the tail's ext_react); spacestep >= 0: also dt_used = min(timestep, spacestep /
// max drift) (spacestep 0: timestep)
void launch_red64(hipStream_t s, DevCtx* ctx, const ForceArgs& a, double spacestep, double timestep,
                  double* react_out);
void launch_update(hipStream_t s, const DevCtx* ctx, const ForceArgs& a);
void launch_adapt(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int force_blocks, float spacestep, float timestep);
void launch_tail(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int force_blocks, int bbox_blocks, int advance,
                 int apply_sched, int ncell_max, const double* sched /* device: gcs_schedule mirror */);
// pos64 != nullptr: the pair predicate runs in fp64 on pos64[sidx[slot]] (strict: no contraction) instead of fp32 on
// the sorted copies
void launch_search_count(hipStream_t s, const DevCtx* ctx, int n, const float4* spos, const int* sidx,
                         const int* scell, const int* cstart, int* counts, const double4* pos64 = nullptr,
                         double d64 = 0.0);
void launch_search_emit(hipStream_t s, const DevCtx* ctx, int n, const float4* spos, const int* sidx,
                        const int* scell, const int* cstart, const int* offsets, unsigned long long* keys,
                        const double4* pos64 = nullptr, double d64 = 0.0);
void launch_exclusive_scan_small(hipStream_t s, const int* in, int* out, int n, int* total);
void sort_u64_keys(hipStream_t s, unsigned long long* keys, unsigned long long* tmp, int n, void* temp, size_t temp_bytes);
size_t sort_u64_temp_bytes(int n);

// contacts.hip: contact map + sampled-position quantisation
void launch_contact_insert(hipStream_t s, const DevCtx* ctx, int n, double dist, const float4* spos, const int* sidx,
                           const int* scell, const int* cstart, unsigned long long* keys, unsigned* counts, int bits,
                           int* overflow, const double4* pos64 = nullptr);
void launch_contact_occupied(hipStream_t s, const unsigned long long* keys, long long slots, int* total);
void launch_contact_compact(hipStream_t s, const unsigned long long* keys, const unsigned* counts, long long slots,
                            unsigned long long* out_k, unsigned* out_c, int* total);
size_t sort_pairs_u64_u32_temp_bytes(int n);
// keys below 2^end_bit (end_bit <= 64: fewer radix passes)
void sort_pairs_u64_u32(hipStream_t s, const unsigned long long* k_in, unsigned long long* k_out, const unsigned* v_in,
                        unsigned* v_out, int n, void* temp, size_t temp_bytes, int end_bit = 64);
void launch_contact_emit(hipStream_t s, const unsigned long long* k, const unsigned* c, int n, unsigned* out);
void launch_quantize(hipStream_t s, const float4* pos, float* out, int n, int bits);
void launch_quantize(hipStream_t s, const double4* pos, float* out, int n, int bits);
// domain.hip: spatial decomposition (band pack / unpack) + the local partial reduction of a decomposed step
constexpr int kMaxPeers = 32;
constexpr int kMaxDomains = 256;
// band records: {x, y, z, index bits} in the engine's precision (16 B fp32, 32 B fp64)
inline size_t band_record_bytes(int prec) { return prec == 64 ? 32 : 16; }
// allreduce buffer: [0, kDomainRed) the local reduction (reactions in[3] out[3]; tile step: max drift, neighbours;
// list step: neighbours, owned particles, fallback particles), then 3 doubles per shared particle, then (list step)
// one slot per domain for the largest displacement from the build
constexpr int kDomainRed = 10;
// domain flags (gcs_engine_domain_flags)
constexpr int kDomFlagBond = 1;      // a bond of an owned particle is longer than the halo
constexpr int kDomFlagCapacity = 2;  // a band exceeded its capacity
constexpr int kDomFlagLost = 4;      // a particle owned by no domain's lists (moved further than the halo allows)
constexpr int kDomFlagMotion = 8;    // cutoff + largest displacement since the build exceeds the halo
// pack: slots != 0 packs from the list slots (the decomposed list step), else by particle index
void launch_domain_pack(hipStream_t s, const DevCtx* ctx, const ForceArgs& a, const DomBox* regions, int npeer,
                        void* out, int* counts, int cap, int* flags, const int* shared = nullptr, int ostride = 0,
                        int cstride = 1, int slots = 0);
void launch_band_headers_zero(hipStream_t s, void* bands, int npeer, int stride, int prec);
void launch_domain_shared_out(hipStream_t s, const DevCtx* ctx, const ForceArgs& a, const int* idx, int nshared,
                              double* buf);
void launch_domain_shared_in(hipStream_t s, const ForceArgs& a, const int* idx, int nshared, const double* buf);
// slots != 0 also refreshes the records' list slots (both psort buffers)
void launch_domain_unpack(hipStream_t s, const ForceArgs& a, const void* in, const int* counts, int nbuf, int cap,
                          int istride = 0, int cstride = 1, int slots = 0, void* send = nullptr, int nsend = 0,
                          int sstride = 0);
void launch_tail_reduce(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int fblocks, double* out);

inline int force_blocks(int n) { return (n + kTile - 1) / kTile; }
// k_force launch size: tiles never cross a cell row, so there are up to (rows) more tiles than force_blocks;
// blocks walk the tiles grid-stride, any launch size is correct
#ifndef GCS_FORCE_GRID_PCT
#define GCS_FORCE_GRID_PCT 125  // force launch size in % of N / 64 (+ 64 blocks)
#endif
inline int force_grid(int n)
{
    return ((int)((long long)force_blocks(n) * GCS_FORCE_GRID_PCT / 100) + 64 + 7) & ~7;  // multiple of 8 (XCDs)
}
// step launches with split tiles: up to two units per tile
inline int force_grid_split(int n) { return 2 * force_grid(n); }
constexpr int kUpdateBlock = 256;
inline int update_blocks(int n) { return (n + kUpdateBlock - 1) / kUpdateBlock; }

// device schedule mirror (double[16]): layout used by launch_tail
enum SchedIdx {
    kSchedFlags = 0,  // bit0 time, bit1 scales, bit2 wall
    kSchedDt = 1,
    kSchedCs0 = 2,
    kSchedCsTau = 3,
    kSchedBs0 = 4,
    kSchedBsTau = 5,
    kSchedK0 = 6,
    kSchedMuW = 9,
    kSchedCount = 16,
};

}  // namespace gcs
