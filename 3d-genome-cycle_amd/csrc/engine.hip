// engine.hip -- host side of the gcs engine and its C ABI (include/gcs.h).
//
// The engine owns all device memory of one simulated system on one HIP device/stream.  Force fields are
// registered like md::system::add_forcefield (returning a handle that gcs_remove_forcefield accepts) and
// compiled lazily into flat device tables (bonded CSR, bending table, tethers, point sources, walls)
// before the next launch.  gcs_engine_run replaces md::simulate_brownian_dynamics: the per-step callback's
// state updates run on the device (k_tail), and chunks of steps are replayed from a captured hipGraph.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: librccl.so.1 is opened at first use (dlopen)

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/gcs.h"
#include "engine_internal.hpp"

using namespace gcs;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg)
{
    g_last_error = msg;
    return code;
}

#define HIPCHK(call)                                                                                        \
    do {                                                                                                    \
        hipError_t e_ = (call);                                                                             \
        if (e_ != hipSuccess) return fail(GCS_EHIP, std::string(#call) + ": " + hipGetErrorString(e_));     \
    } while (0)

enum FieldKind { F_SOFTCORE = 1, F_SOFTWELL, F_BONDED, F_BENDING, F_WALL_IN, F_WALL_OUT, F_POINT, F_KFIBER };

struct FieldRec {
    int kind = 0;
    int handle = 0;
    gcs_softcore_params sc{};
    gcs_softwell_params sw{};
    gcs_bond_params bond{};
    gcs_wall_params wall{};
    gcs_point_source_params point{};
    double spring = 0, energy = 0;
    double center[3] = {0, 0, 0};
    double pole[3] = {0, 0, 0};
    std::vector<int64_t> idx;
    std::vector<gcs_kinetochore_spec> specs;
};

// What a captured step sequence depends on beyond its (phase, parity, length) key: anything else that changes
// drops every cached graph before the next capture.
struct GraphKey {
    int topo_version, fused, list_every, sched_flags, waves, chunk, spacestep, list_waves, skin_pm;
    gcs_bd_config cfg;
};
bool same_key(const GraphKey& x, const GraphKey& y)
{
    return x.topo_version == y.topo_version && x.fused == y.fused && x.list_every == y.list_every &&
           x.sched_flags == y.sched_flags && x.waves == y.waves && x.chunk == y.chunk && x.spacestep == y.spacestep &&
           x.list_waves == y.list_waves && x.skin_pm == y.skin_pm && x.cfg.temperature == y.cfg.temperature &&
           x.cfg.timestep == y.cfg.timestep && x.cfg.spacestep == y.cfg.spacestep && x.cfg.seed == y.cfg.seed &&
           x.cfg.noise == y.cfg.noise;
}
struct GraphEntry {
    int phase, parity, len;
    hipGraph_t graph;
    hipGraphExec_t exec;
    unsigned long long used;
};
constexpr size_t kMaxGraphs = 32;  // cached step sequences per engine (least recently used evicted)
constexpr int kInflight = 8;       // graph launches an engine lets run ahead of the device

template <class T>
int dalloc(T** p, size_t count)
{
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) return fail(GCS_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    // GCS_DEBUG_POISON=2 (diagnostics): every allocation starts as hashed garbage (what a recycled allocation may
    // hold), so a read of memory nothing wrote shows up in a fresh process too
    const char* pv = std::getenv("GCS_DEBUG_POISON");
    if (pv && std::atoi(pv) >= 2) {
        launch_poison(nullptr, *p, count * sizeof(T) / 4 * 4);
        (void)hipDeviceSynchronize();
    }
    return GCS_OK;
}

// GCS_DEBUG_SYNC (diagnostics): synchronise after each launch of the decomposed path and report, on stderr, the
// launch after which the stream first holds an error (the kernel that faulted)
void dbg_sync(gcs_engine* e, const char* what);

template <class T>
void dfree(T*& p)
{
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

}  // namespace

struct gcs_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    int n = 0;
    int prec = 64;  // GCS_PRECISION_F64 (the reference's double; default) or GCS_PRECISION_F32
    std::vector<double> mu, ab;
    std::vector<FieldRec> fields;
    int next_handle = 1;
    bool dirty = true;
    int topo_version = 0;
    int ncell_max = 0;

    // device state
    float4* pos[2] = {nullptr, nullptr};
    float4* kmu = nullptr;
    float4* spos = nullptr;
    float* sb = nullptr;
    int *sidx = nullptr, *scell = nullptr, *cell_of = nullptr, *slot = nullptr, *tmp = nullptr;
    int *count = nullptr, *cstart = nullptr, *tile_start = nullptr;
    int2* tile_range = nullptr;
    DevCtx* ctx = nullptr;
    double* dsched = nullptr;
    float* part_force = nullptr;
    float* part_bbox = nullptr;
    double* part_energy = nullptr;
    float4* force_out = nullptr;
    float4* pbuf = nullptr;  // split-tile partial forces
    int4* units = nullptr;    // heavy-tile unit table (cell scan -> force kernel)
    unsigned long long* scan_sync = nullptr;  // multi-block cell scan: epoch word + look-back granules
    int resident = 0;         // force-step workgroups resident at once (split budget)
    int* tcnt = nullptr;     // split-tile arrival counters
    float4* bucket_p = nullptr;  // rebuild step: [ncell_max][kBucketCap] sorted records filed by the force kernel
    int2* bucket_q = nullptr;
    float4* ovf_p = nullptr;     // rebuild step: bucket overflow list [n]
    int4* ovf_q = nullptr;
    int* ovf_n = nullptr;    // rebuild step: its two counters (step parity)
    unsigned long long* rb_sync = nullptr;  // rebuild step: epoch word + look-back granules
    // topology tables
    int* boff = nullptr;
    int2* bent = nullptr;
    float4* bval = nullptr;
    int* sw_idx = nullptr;  // droplet targets (<= 64)
    int nbent = 0;          // bond CSR entries
    int* bslot = nullptr;   // list step: the slot of each bond CSR entry's partner (ForceArgs::bslot)
    int* swslot = nullptr;  // list step: the slot of each droplet target
    int bslot_cap = 0;
    int* brev = nullptr;    // per bond CSR entry: its reverse entry (the partner's entry pointing back)
    bool brev_ok = false;
    int* swt = nullptr;     // per particle: its droplet target index, -1 none
    float* bend_eps = nullptr;
    int* toff = nullptr;
    Tether* tent = nullptr;
    // fp64 state (prec 64; include/gcs.h GCS_PRECISION_F64): positions, constants, forces, the evaluation's partial
    // rows and reaction buffer, the topology values, the list step's slot-ordered copies, injected normals
    double4* dpos[2] = {nullptr, nullptr};
    double4* dkmu = nullptr;
    double4* dforce_out = nullptr;
    double* dpart = nullptr;
    double* dred = nullptr;  // [6] the reactions of a spacestep step's force pass (k_red64 -> the tail's ext_react)
    double4* dbval = nullptr;
    double* dbend_eps = nullptr;
    TetherT<double>* dtent = nullptr;
    double2* dtype_ab = nullptr;
    double4* dpsort[2] = {nullptr, nullptr};
    double4* dskmu = nullptr;
    double* dnoise = nullptr;
    double4* s_pts64 = nullptr;  // fp64 query points of gcs_engine_search_neighbors
    // injected noise
    float* noise = nullptr;
    int64_t noise_steps = 0;
    int64_t noise_cursor = 0;  // host mirror
    // search scratch
    int search_cap = 0;
    float4 *s_pts = nullptr, *s_spos = nullptr;
    float* s_sb = nullptr;
    int *s_sidx = nullptr, *s_scell = nullptr, *s_cell_of = nullptr, *s_slot = nullptr, *s_tmp = nullptr;
    int *s_count = nullptr, *s_cstart = nullptr, *s_counts = nullptr, *s_offsets = nullptr, *s_total = nullptr;
    int* s_tile = nullptr;
    int2* s_tile_range = nullptr;
    int s_ncell_max = 0;
    DevCtx* s_ctx = nullptr;
    DevCtx s_ctx_host{};
    unsigned long long* s_scan_sync = nullptr;
    unsigned long long *s_keys = nullptr, *s_keys2 = nullptr;
    void* s_sort_temp = nullptr;
    size_t s_sort_bytes = 0;
    int64_t s_key_cap = 0;
    // contact map (stage_interphase/contact_map.cpp): hash table of 2^c_bits slots + compaction/sort scratch
    int c_bits = 0;
    unsigned long long* c_keys = nullptr;
    unsigned* c_counts = nullptr;
    int* c_flags = nullptr;  // [0] overflow, [1] compacted entries
    int64_t c_updates = 0;   // host mirror: updates since the last clear
    // contacts_read scratch, kept between reads (compaction into the table's size, the sorted copies, sort temp)
    unsigned long long *c_ck = nullptr, *c_ck2 = nullptr;
    unsigned *c_cv = nullptr, *c_cv2 = nullptr;
    unsigned* c_rows = nullptr;  // the read's (i, j, count) rows, 3 x c_sorted_cap
    void* c_temp = nullptr;
    size_t c_temp_bytes = 0;
    int64_t c_sorted_cap = 0;
    int c_bits_opt = 0;      // GCS_OPT_CONTACT_BITS (0: sized from N at the first update)
    // sampled positions (store quantisation)
    float* q_out = nullptr;
    float* q_host = nullptr;  // pinned staging of the quantised sample (a pageable D2H copy stages through the runtime)
    // spatial domain decomposition (gcs_engine_set_domain): own box, halo, peer regions, domain index / count
    bool dom = false;
    DomBox dom_box{};
    float dom_halo = 0.f;
    DomBox* dom_regions = nullptr;  // device copy of the peers' regions [npeer] (box - halo, box + halo)
    int dom_npeer = 0;
    int dom_index = 0, dom_ndom = 1;
    bool dom_list = false;  // the decomposed run takes the list step (decided when it is primed)
    int dom_flags_step = 0;  // k_lstep flags of the last decomposed list step (its tail uses the same)
    int* islot = nullptr;   // [n] particle -> slot of the current lists (-1: not binned), decomposed list step
    bool dom_cont = false;  // the next domain step continues the previous one (no re-priming)
    int* dom_shared_idx = nullptr;   // shared particles (gcs_engine_set_domain_shared) [nshared]
    int* dom_shared_flag = nullptr;  // [n] k + 1 for the k-th shared particle, 0 = not shared
    bool dom_fused = false;          // the last decomposed step packed its bands itself (k_lstep<..., DOM>)
    int dom_nshared = 0;
    int64_t dom_next = 0;
    // engine-owned decomposed-run exchange (gcs_engine_domain_buffers) and its RCCL transport
    // [npeer][cap + 1] records of band_record_bytes(prec): row 0 of a band = {count bits, 0, 0, 0}, then records
    unsigned char* dom_send = nullptr;
    unsigned char* dom_recv = nullptr;
    int dom_cap = 0;
    double* dom_red = nullptr;   // [nred]: local reduction + shared positions; dom_glob: the sum over domains
    double* dom_glob = nullptr;
    int dom_nred = 0;
    int* dom_flags = nullptr;
    int dom_peer_rank[kMaxPeers] = {};
    ncclComm_t nccl = nullptr;
    int nccl_ranks = 0;
    hipGraphExec_t dgexec = nullptr;
    hipGraph_t dgraph = nullptr;
    int dg_steps = 0;
    gcs_bd_config dg_cfg{};
    int dg_version = -1, dg_sched_flags = -1, dg_phase = -1, dg_skin = -1;

    ForceArgs fa{};
    gcs_schedule sched{};
    int sched_flags = 0;
    int parity = 0;  // host mirror of ctx->parity

    // options / graph cache
    int graph_steps = 32;
    int waves = 4;
    int fused = 3;  // GCS_OPT_FUSED_STEP: 3 = the list step, 2 = the 2-launch rebuild step, 1 = the 4-launch step, 0 = unfused
    bool scan_mb = true;  // GCS_OPT_SCAN_BLOCKS: multi-block cell scan (the heavy-tile split keeps one block)
    // captured step sequences, keyed by what a replay bakes in besides the launch arguments below: the list
    // step's rebuild phase (first step mod M) and starting position-buffer parity, and the sequence length
    std::vector<GraphEntry> graphs;
    unsigned long long graph_clock = 0;  // LRU stamp
    GraphKey g_key{};                     // what every cached graph was captured under (else the cache is dropped)
    bool g_key_set = false;
    // bounded run-ahead: an event after every graph launch; the host waits for the one kInflight launches back
    // before enqueueing another (a host that enqueues thousands of replays ahead of the device gains nothing and
    // exhausted a tracing profiler's per-dispatch records)
    hipEvent_t inflight[kInflight] = {};
    unsigned long long inflight_n = 0;
    gcs_run_stats rstats{};

    // list step (GCS_OPT_FUSED_STEP 3): neighbour lists, pair-factor classes, rebuild period
    int* list = nullptr;
    int* lcount = nullptr;
    int4* lbase = nullptr;
    unsigned* psync = nullptr;  // the persistent small-system step's hand-off halves
    int* pstall = nullptr;      // its stall word (ForceArgs::pstall)
    DevCtx* pkeep = nullptr;    // the context at the start of the current k_pstep launch (k_pstep_guard)
    int small_opt = 1;          // GCS_OPT_SMALL_STEP
    bool fused_explicit = false;  // GCS_OPT_FUSED_STEP was set: the step shape it names, never the small step
    float4* psort[2] = {nullptr, nullptr};
    float4* skmu = nullptr;  // list step: slot-ordered kmu and bond CSR rows
    int2* sbrow = nullptr;
    int* ptype = nullptr;
    unsigned* lticket = nullptr;  // list step: two-level arrival counters (8 groups + the top), 128 B apart
    float2* type_ab = nullptr;
    int ntypes = 0;
    bool list_ok = false;       // the system admits the list step (a pair field, <= 256 classes, N < 2^24)
    int list_cap = 1024;        // GCS_OPT_LIST_CAP: list entries per particle (split over the tile's waves)
    size_t list_alloc = 0;      // allocated entries
    int list_skin_pm = 0;       // GCS_OPT_LIST_SKIN: skin in 1/1000 of the pair cutoff (0: the precision's default)
    int skin_level_pm = 0;      // the skin (1/1000 of the pair cutoff) of the current undecomposed list run (skin_level)
    int list_every_opt = 0;     // GCS_OPT_LIST_EVERY: rebuild period in steps (0: from the noise amplitude)
    int list_every = 1;         // the period of the current run
    int list_skin_base_pm = 0;  // GCS_OPT_LIST_SKIN_BASE: the core-scale-following default skin's s1 (0: the precision's)
    int list_phase = 0;         // GCS_OPT_LIST_PHASE: rebuilds at the steps s with (s + list_phase) % list_every == 0
    int list_waves = 4;         // GCS_OPT_LIST_WAVES: waves per tile (2: more tiles resident, for replica runs)
    int list_fmt_opt = 0;       // GCS_OPT_LIST_FORMAT: 0 (default) 16-bit slots (absolute up to 65,536 particles,
                                // plane-relative beyond), 1 plane-relative 16-bit, 2 absolute 32-bit
    long long list_deal_opt = -1;  // GCS_OPT_LIST_DEAL: chunk -> wave pattern of the list build (-1: the default for
                                   // list_waves, 0: round robin)
    bool l_need_build = true;   // the next list step must rebuild (run start without continuity)
    // dense systems: mean neighbours within the cutoff above which a fresh run takes the 2-launch tile step instead
    // of the list step (GCS_OPT_DENSE_NEIGHBORS; 0: never), and the current chain's verdict
    int dense_opt = 96;
    bool dense = false;
    double dense_mean = -1.0;  // the last probe's mean neighbour count
    double c_pending = 0;      // a contact update fused into the next list step (its distance; 0: none)

    // fused-step continuity: after a fused run the cells of the next positions are already binned with the
    // grid the next step expects, so a run that continues at chain_step skips re-priming (bitwise identical
    // to one longer run).  Anything that touches positions, context, schedule or cells clears it.
    bool chain_valid = false;
    // a dense chain (the fp32 tile step picked by the density probe) keeps its verdict while it continues: the
    // tile step leaves no fused state (chain_valid stays false), so the verdict has its own continuity record
    bool dense_chain = false;
    int64_t chain_step = 0;
    double chain_dt = 0;  // the timestep begin_run last wrote to ctx->dt_used
    int chain_version = -1;

};

namespace {

// the decomposed run's captured chunk (kernels + RCCL collectives): it bakes in the domain geometry, the
// exchange buffers and the communicator, so every change of those drops it
void drop_domain_graph(gcs_engine* e)
{
    if (e->dgexec) (void)hipStreamSynchronize(e->stream);  // it may still be executing
    if (e->dgexec) (void)hipGraphExecDestroy(e->dgexec);
    if (e->dgraph) (void)hipGraphDestroy(e->dgraph);
    e->dgexec = nullptr;
    e->dgraph = nullptr;
}

void drop_graph(gcs_engine* e)
{
    if (!e->graphs.empty() || e->dgexec) (void)hipStreamSynchronize(e->stream);  // none may still be executing
    for (GraphEntry& g : e->graphs) {
        (void)hipGraphExecDestroy(g.exec);
        (void)hipGraphDestroy(g.graph);
    }
    e->graphs.clear();
    e->g_key_set = false;
    drop_domain_graph(e);
}

FieldRec* new_field(gcs_engine* e, int kind)
{
    e->fields.emplace_back();
    FieldRec& f = e->fields.back();
    f.kind = kind;
    f.handle = e->next_handle++;
    e->dirty = true;
    return &f;
}

bool valid_index(const gcs_engine* e, int64_t i) { return i >= 0 && i < e->n; }

// Flatten the registered fields into device tables (DESIGN.md "device layout"): the fp32 parameter block always, the
// fp64 block and tables (dkmu, dbval, dbend_eps, dtent, dtype_ab) for an fp64 engine.  Every derived value (mixed
// bond constants, 1 / decay^2, cutoff^2, K / mobility) is formed in double first; the fp32 engine rounds it once.
int compile(gcs_engine* e)
{
    if (!e->dirty) return GCS_OK;
    const int n = e->n;
    const bool f64 = e->prec == 64;
    ForceArgs& a = e->fa;
    a.has_pair = 0;
    a.has_bonds = 0;
    a.has_bend = 0;
    a.has_tether = 0;
    a.n_point = 0;
    a.has_wall_in = 0;
    a.has_wall_out = 0;
    FieldPrm<double> pd = e->fa.pd;  // keeps temperature / timestep (begin_run sets them)

    std::vector<std::vector<int2>> blist(n);
    std::vector<BondParam> params;
    std::vector<double> bend(n, 0.0);
    std::vector<std::vector<TetherT<double>>> tlist(n);
    int pair_mix = 1;
    bool sw_done = false;
    std::vector<int> sw_idx;
    a.sw_n = 0;

    for (const FieldRec& f : e->fields) {
        switch (f.kind) {
        case F_SOFTCORE:
            if (a.has_pair) return fail(GCS_EINVAL, "only one neighbor soft-core field may be active");
            a.has_pair = 1;
            a.pair_mix = f.sc.mix ? 1 : 0;
            pair_mix = a.pair_mix;
            a.pair_scaled = f.sc.scaled ? 1 : 0;
            pd.pa_eps = f.sc.a_energy;
            pd.pa_sig = f.sc.a_diameter;
            pd.pb_eps = f.sc.mix ? f.sc.b_energy : 0.0;
            pd.pb_sig = f.sc.b_diameter > 0 ? f.sc.b_diameter : 1.0;
            pd.pair_dist = f.sc.neighbor_distance;
            break;
        case F_SOFTWELL: {
            if (!sw_done && f.idx.size() <= 64) {  // the wave-cooperative droplet (local_terms)
                sw_done = true;
                a.sw_n = (int)f.idx.size();
                pd.sw_ka = f.sw.energy;
                pd.sw_kb = 1.0 / (f.sw.decay_distance * f.sw.decay_distance);
                pd.sw_la = f.sw.cutoff * f.sw.cutoff;
                sw_idx.assign(f.idx.begin(), f.idx.end());
                break;
            }
            BondParam bp{};
            bp.type = kSoftwell;
            bp.ka = f.sw.energy;
            bp.kb = 1.0 / (f.sw.decay_distance * f.sw.decay_distance);
            bp.la = f.sw.cutoff * f.sw.cutoff;
            const int pid = (int)params.size();
            params.push_back(bp);
            for (size_t p = 0; p < f.idx.size(); ++p)
                for (size_t q = 0; q < f.idx.size(); ++q)
                    if (p != q && f.idx[p] != f.idx[q]) blist[f.idx[p]].push_back(make_int2((int)f.idx[q], pid));
            break;
        }
        case F_BONDED: {
            // a field whose spring constants are all zero contributes exactly nothing (the reference's
            // i,i+2 loop field with a/b_core_2nd_bond_spring = 0, simulation_driver_forcefield.cpp:99-136)
            if (f.bond.a_spring == 0 && f.bond.b_spring == 0) break;
            BondParam bp{};
            bp.type = f.bond.potential == GCS_POT_HARMONIC ? kHarmonic
                      : (f.bond.potential == GCS_POT_SPRING ? kSpring : kSemispring);
            bp.mix = f.bond.mix ? 1 : 0;
            bp.scaled = f.bond.scaled ? 1 : 0;
            bp.ka = f.bond.a_spring;
            bp.kb = f.bond.b_spring;
            bp.la = f.bond.a_length;
            bp.lb = f.bond.b_length;
            if (e->prec != 64) {  // the fp32 engine took the field's constants as fp32 (its own parameter rounding)
                bp.ka = (float)bp.ka;
                bp.kb = (float)bp.kb;
                bp.la = (float)bp.la;
                bp.lb = (float)bp.lb;
            }
            const int pid = (int)params.size();
            params.push_back(bp);
            for (size_t q = 0; q + 1 < f.idx.size(); q += 2) {
                const int i = (int)f.idx[q], j = (int)f.idx[q + 1];
                blist[i].push_back(make_int2(j, pid));
                blist[j].push_back(make_int2(i, pid));
            }
            break;
        }
        case F_BENDING:
            for (int64_t k : f.idx) bend[k] += f64 ? f.energy : (double)(float)f.energy;
            break;
        case F_WALL_IN:
            if (a.has_wall_in) return fail(GCS_EINVAL, "only one ellipsoid inward field may be active");
            a.has_wall_in = 1;
            pd.win.a_eps = f.wall.a_energy;
            pd.win.a_sig = f.wall.a_diameter;
            pd.win.b_eps = f.wall.mix ? f.wall.b_energy : 0.0;
            pd.win.b_sig = f.wall.b_diameter > 0 ? f.wall.b_diameter : 1.0;
            pd.win.wall_a = f.wall.wall_a;
            pd.win.wall_b = f.wall.wall_b;
            pd.win.cx = f.wall.center[0];
            pd.win.cy = f.wall.center[1];
            pd.win.cz = f.wall.center[2];
            pd.win.mix = f.wall.mix ? 1 : 0;
            pd.win.scaled = f.wall.scaled ? 1 : 0;
            break;
        case F_WALL_OUT:
            if (a.has_wall_out) return fail(GCS_EINVAL, "only one ellipsoid outward field may be active");
            a.has_wall_out = 1;
            pd.wout_k = f.spring;
            pd.wout_cx = f.center[0];
            pd.wout_cy = f.center[1];
            pd.wout_cz = f.center[2];
            break;
        case F_POINT: {
            if (a.n_point >= kMaxPointSources) return fail(GCS_EINVAL, "too many point-source fields (max 4)");
            PointSrcT<double>& p = pd.point[a.n_point++];
            p.type = f.point.potential;
            p.px = f.point.point[0];
            p.py = f.point.point[1];
            p.pz = f.point.point[2];
            p.k = f.point.spring;
            p.l = f.point.length;
            p.f = f.point.force;
            p.b = f.point.reactive_distance;
            break;
        }
        case F_KFIBER:
            for (const gcs_kinetochore_spec& sp : f.specs) {
                TetherT<double> t{};
                t.px = f.pole[0];
                t.py = f.pole[1];
                t.pz = f.pole[2];
                t.k = sp.decay_rate / sp.mobility;  // kinetochore_fiber_forcefield.cpp:46-53
                t.l = sp.stationary_length;
                tlist[sp.particle_index].push_back(t);
            }
            break;
        }
    }
    if (a.has_wall_in && a.has_wall_out) {
        if (pd.win.cx != pd.wout_cx || pd.win.cy != pd.wout_cy || pd.win.cz != pd.wout_cz)
            return fail(GCS_EINVAL, "inward and outward ellipsoid fields must share the centre");
    }
    // the fp32 block: every parameter rounded once
    FieldPrm<float>& pf = a.pf;
    pf.pa_eps = (float)pd.pa_eps;
    pf.pa_sig = (float)pd.pa_sig;
    pf.pb_eps = (float)pd.pb_eps;
    pf.pb_sig = (float)pd.pb_sig;
    pf.pair_dist = (float)pd.pair_dist;
    pf.sw_ka = (float)pd.sw_ka;
    pf.sw_kb = (float)pd.sw_kb;
    pf.sw_la = (float)pd.sw_la;
    for (int q = 0; q < kMaxPointSources; ++q) {
        const PointSrcT<double>& d = pd.point[q];
        pf.point[q] = PointSrcT<float>{d.type, (float)d.px, (float)d.py, (float)d.pz, (float)d.k, (float)d.l,
                                       (float)d.f, (float)d.b};
    }
    const WallInT<double>& w = pd.win;
    pf.win = WallInT<float>{(float)w.a_eps, (float)w.a_sig, (float)w.b_eps, (float)w.b_sig, (float)w.wall_a,
                            (float)w.wall_b, (float)w.cx, (float)w.cy, (float)w.cz, w.mix, w.scaled};
    pf.wout_k = (float)pd.wout_k;
    pf.wout_cx = (float)pd.wout_cx;
    pf.wout_cy = (float)pd.wout_cy;
    pf.wout_cz = (float)pd.wout_cz;
    a.pd = pd;

    // per-particle constants {mu, a, b, t}
    std::vector<float4> hk(n);
    std::vector<double4> hkd(f64 ? n : 0);
    for (int i = 0; i < n; ++i) {
        hk[i] = make_float4((float)e->mu[i], (float)e->ab[2 * i], (float)e->ab[2 * i + 1], 0.f);
        if (f64) hkd[i] = make_double4(e->mu[i], e->ab[2 * i], e->ab[2 * i + 1], 0.0);
    }
    for (int t : sw_idx) {  // droplet target
        hk[t].w = 1.f;
        if (f64) hkd[t].w = 1.0;
    }
    dfree(e->sw_idx);
    dfree(e->swt);
    if (a.sw_n > 0) {
        int rc;
        if ((rc = dalloc(&e->sw_idx, 64))) return rc;
        HIPCHK(hipMemcpyAsync(e->sw_idx, sw_idx.data(), sw_idx.size() * sizeof(int), hipMemcpyHostToDevice, e->stream));
        // particle -> its droplet target index (-1: none): k_cell_sort files a target's slot (slot_bonds)
        std::vector<int> swt(n, -1);
        for (size_t t = 0; t < sw_idx.size(); ++t) swt[sw_idx[t]] = (int)t;
        if ((rc = dalloc(&e->swt, n))) return rc;
        HIPCHK(hipMemcpyAsync(e->swt, swt.data(), n * sizeof(int), hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    a.sw_idx = e->sw_idx;
    HIPCHK(hipMemcpyAsync(e->kmu, hk.data(), n * sizeof(float4), hipMemcpyHostToDevice, e->stream));
    if (f64) HIPCHK(hipMemcpyAsync(e->dkmu, hkd.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->stream));

    // list step: pair-factor classes (the (a, b) the pair field mixes; k_cell_sort's spos.w / sb), keyed by the
    // double factors (the fp32 engine's table holds their roundings)
    std::vector<int> pt(n, 0);
    std::vector<float2> tab;
    std::vector<double2> tabd;
    {
        std::map<std::pair<double, double>, int> cls;
        bool ok = a.has_pair && n > 0 && n < (1 << kListIndexBits);
        for (int i = 0; ok && i < n; ++i) {
            const std::pair<double, double> key =
                pair_mix ? std::make_pair(e->ab[2 * i], e->ab[2 * i + 1]) : std::make_pair(1.0, 0.0);
            auto it = cls.find(key);
            if (it == cls.end()) {
                if ((int)cls.size() >= kMaxTypes) {
                    ok = false;
                    break;
                }
                it = cls.emplace(key, (int)cls.size()).first;
                tab.push_back(make_float2((float)key.first, (float)key.second));
                tabd.push_back(make_double2(key.first, key.second));
            }
            pt[i] = it->second;
        }
        e->list_ok = ok;
        e->ntypes = ok ? (int)tab.size() : 0;
        if (ok) {
            int rc;
            if (!e->ptype && (rc = dalloc(&e->ptype, n))) return rc;
            if (!e->type_ab && (rc = dalloc(&e->type_ab, kMaxTypes))) return rc;
            if (f64 && !e->dtype_ab && (rc = dalloc(&e->dtype_ab, kMaxTypes))) return rc;
            HIPCHK(hipMemcpyAsync(e->ptype, pt.data(), n * sizeof(int), hipMemcpyHostToDevice, e->stream));
            HIPCHK(hipMemcpyAsync(e->type_ab, tab.data(), tab.size() * sizeof(float2), hipMemcpyHostToDevice, e->stream));
            if (f64)
                HIPCHK(hipMemcpyAsync(e->dtype_ab, tabd.data(), tabd.size() * sizeof(double2), hipMemcpyHostToDevice,
                                      e->stream));
        }
    }

    dfree(e->boff);
    dfree(e->bent);
    dfree(e->bval);
    dfree(e->bend_eps);
    dfree(e->toff);
    dfree(e->tent);
    dfree(e->dbval);
    dfree(e->dbend_eps);
    dfree(e->dtent);

    size_t nb = 0;
    for (auto& l : blist) nb += l.size();
    if (nb > 0) {
        std::vector<int> off(n + 1, 0);
        std::vector<int2> ent;
        std::vector<float4> val;
        std::vector<double4> vald;
        ent.reserve(nb);
        val.reserve(nb);
        for (int i = 0; i < n; ++i) {
            off[i] = (int)ent.size();
            for (const int2& b : blist[i]) {
                const BondParam& bp = params[b.y];
                const int j = b.x;
                double4 v = make_double4(bp.ka, bp.kb, bp.la, 0.0);
                if (bp.type != kSoftwell) {
                    // simulation_driver_forcefield.cpp:71-76: K = a k_a + b k_b, l = a l_a + b l_b with the pair's
                    // mean factors a = (a_i + a_j) / 2, b = (b_i + b_j) / 2 (mix), else k_a, l_a
                    double K = bp.ka, l = bp.la;
                    if (bp.mix) {
                        const double A = 0.5 * (e->ab[2 * i] + e->ab[2 * j]), B = 0.5 * (e->ab[2 * i + 1] + e->ab[2 * j + 1]);
                        K = A * bp.ka + B * bp.kb;
                        l = A * bp.la + B * bp.lb;
                    }
                    v = make_double4(K, l, 0.0, 0.0);
                }
                ent.push_back(make_int2(j, bp.type | (bp.scaled ? 16 : 0)));
                val.push_back(make_float4((float)v.x, (float)v.y, (float)v.z, 0.f));
                if (f64) vald.push_back(v);
            }
        }
        off[n] = (int)ent.size();
        int rc;
        if ((rc = dalloc(&e->boff, n + 1))) return rc;
        if ((rc = dalloc(&e->bent, ent.size()))) return rc;
        if ((rc = dalloc(&e->bval, val.size()))) return rc;
        if (f64 && (rc = dalloc(&e->dbval, vald.size()))) return rc;
        HIPCHK(hipMemcpyAsync(e->boff, off.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipMemcpyAsync(e->bent, ent.data(), ent.size() * sizeof(int2), hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipMemcpyAsync(e->bval, val.data(), val.size() * sizeof(float4), hipMemcpyHostToDevice, e->stream));
        if (f64)
            HIPCHK(hipMemcpyAsync(e->dbval, vald.data(), vald.size() * sizeof(double4), hipMemcpyHostToDevice, e->stream));
        // the reverse of every entry (j's entry pointing back at i; the k-th such entry for the k-th duplicate):
        // k_cell_sort then tells each partner's entry its particle's slot (slot_bonds).  Every pairwise field is
        // entered in both directions; an entry without its reverse turns the slot-indexed partners off
        std::vector<int> rev(ent.size(), -1);
        bool rev_ok = true;
        for (int i = 0; i < n && rev_ok; ++i)
            for (int q = off[i]; q < off[i + 1]; ++q) {
                const int j = ent[q].x;
                int k = 0;  // this is the k-th entry of row i pointing at j
                for (int r = off[i]; r < q; ++r) k += ent[r].x == j ? 1 : 0;
                int found = -1;
                for (int r = off[j]; r < off[j + 1]; ++r)
                    if (ent[r].x == i && k-- == 0) {
                        found = r;
                        break;
                    }
                if (found < 0) {
                    rev_ok = false;
                    break;
                }
                rev[q] = found;
            }
        e->brev_ok = rev_ok;
        dfree(e->brev);
        if (rev_ok) {
            if ((rc = dalloc(&e->brev, rev.size()))) return rc;
            HIPCHK(hipMemcpyAsync(e->brev, rev.data(), rev.size() * sizeof(int), hipMemcpyHostToDevice, e->stream));
        }
        HIPCHK(hipStreamSynchronize(e->stream));  // val / ent / rev die at the end of this block
        e->nbent = (int)ent.size();
        a.has_bonds = 1;
    }
    bool any_bend = false;
    for (double v : bend) any_bend |= (v != 0.0);
    if (any_bend) {
        std::vector<float> bf(n);
        for (int i = 0; i < n; ++i) bf[i] = (float)bend[i];
        int rc;
        if ((rc = dalloc(&e->bend_eps, n))) return rc;
        HIPCHK(hipMemcpyAsync(e->bend_eps, bf.data(), n * sizeof(float), hipMemcpyHostToDevice, e->stream));
        if (f64) {
            if ((rc = dalloc(&e->dbend_eps, n))) return rc;
            HIPCHK(hipMemcpyAsync(e->dbend_eps, bend.data(), n * sizeof(double), hipMemcpyHostToDevice, e->stream));
        }
        HIPCHK(hipStreamSynchronize(e->stream));  // bf dies here
        a.has_bend = 1;
    }
    size_t nt = 0;
    for (auto& l : tlist) nt += l.size();
    if (nt > 0) {
        std::vector<int> off(n + 1, 0);
        std::vector<Tether> ent;
        std::vector<TetherT<double>> entd;
        for (int i = 0; i < n; ++i) {
            off[i] = (int)ent.size();
            for (const TetherT<double>& t : tlist[i]) {
                ent.push_back(Tether{(float)t.px, (float)t.py, (float)t.pz, (float)t.k, (float)t.l, 0.f, 0.f, 0.f});
                entd.push_back(t);
            }
        }
        off[n] = (int)ent.size();
        int rc;
        if ((rc = dalloc(&e->toff, n + 1))) return rc;
        if ((rc = dalloc(&e->tent, ent.size()))) return rc;
        HIPCHK(hipMemcpyAsync(e->toff, off.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipMemcpyAsync(e->tent, ent.data(), ent.size() * sizeof(Tether), hipMemcpyHostToDevice, e->stream));
        if (f64) {
            if ((rc = dalloc(&e->dtent, entd.size()))) return rc;
            HIPCHK(hipMemcpyAsync(e->dtent, entd.data(), entd.size() * sizeof(TetherT<double>), hipMemcpyHostToDevice,
                                  e->stream));
        }
        a.has_tether = 1;
    }
    a.boff = e->boff;
    a.bent = e->bent;
    a.bval = e->bval;
    a.bend_eps = e->bend_eps;
    a.toff = e->toff;
    a.tent = e->tent;
    a.dbval = e->dbval;
    a.dbend_eps = e->dbend_eps;
    a.dtent = e->dtent;
    HIPCHK(hipStreamSynchronize(e->stream));  // host vectors die here
    e->dirty = false;
    e->topo_version++;
    drop_graph(e);
    return GCS_OK;
}

void fill_state_args(gcs_engine* e)
{
    ForceArgs& a = e->fa;
    a.n = e->n;
    a.prec = e->prec;
    a.pos0 = e->pos[0];
    a.pos1 = e->pos[1];
    a.kmu = e->kmu;
    a.dpos0 = e->dpos[0];
    a.dpos1 = e->dpos[1];
    a.dkmu = e->dkmu;
    a.dforce_out = e->dforce_out;
    a.dpart = e->dpart;
    a.dnoise = e->dnoise;
    a.spos = e->spos;
    a.sb = e->sb;
    a.sidx = e->sidx;
    a.scell = e->scell;
    a.cstart = e->cstart;
    a.tile_range = e->tile_range;
    a.part_force = e->part_force;
    a.part_bbox = e->part_bbox;
    a.part_energy = e->part_energy;
    a.force_out = e->force_out;
    a.noise = e->noise;
    a.noise_steps = e->noise_steps;
    a.cell_of = e->cell_of;
    a.slot = e->slot;
    a.count = e->count;
    a.cstart_w = e->cstart;
    a.tile_start_w = e->tile_start;
    a.tile_range_w = e->tile_range;
    a.sched = e->dsched;
    a.ncell_max = e->ncell_max;
    a.apply_sched = e->sched_flags != 0;
    a.pbuf = e->pbuf;
    a.units = e->units;
    a.tcnt = e->tcnt;
    a.bucket_p = e->fused == 2 ? e->bucket_p : nullptr;
    a.bucket_q = e->bucket_q;
    a.ovf_p = e->ovf_p;
    a.ovf_q = e->ovf_q;
    a.ovf_n = e->ovf_n;
    a.split_cap = std::max(force_grid(e->n), kMaxUnits);
}

// scan the binned counts of ctx->grid (or ctx->grid_next): cstart, tile_start, tile table
void enqueue_scan(gcs_engine* e, bool use_next)
{
    const bool heavy = e->fa.split == 2;
    launch_cell_scan(e->stream, e->ctx, e->n, e->count, e->cstart, e->tile_start, e->tile_range, use_next, e->units,
                     heavy ? e->resident : 0, e->scan_mb ? e->scan_sync : nullptr, e->ncell_max);
}

// bin the current positions into ctx->grid: per-cell counts + slots, scan, tile table
// count the current positions (either precision) into ctx->grid's cells; reg / islot: a decomposed domain's region
void enqueue_count(gcs_engine* e, const DomBox* reg = nullptr, int* islot = nullptr)
{
    if (e->prec == 64)
        launch_cell_count(e->stream, e->ctx, e->dpos[0], e->dpos[1], e->n, e->cell_of, e->slot, e->count, reg, islot);
    else
        launch_cell_count(e->stream, e->ctx, e->pos[0], e->pos[1], e->n, e->cell_of, e->slot, e->count, reg, islot);
}

void enqueue_bin(gcs_engine* e)
{
    enqueue_count(e);
    enqueue_scan(e, false);
}

// order each (scattered) cell by particle index: the cell-sorted copies the pair loop reads; lists: also the
// slot-ordered positions, constants and bond rows of the list step (islot: a decomposed build's particle -> slot)
bool slot_bonds(const gcs_engine* e);
void enqueue_cell_order(gcs_engine* e, bool lists = false, int* islot = nullptr)
{
    // slot-indexed partners (undecomposed lists): particle -> slot, each partner's entry and droplet target slot
    const bool sbm = lists && !islot && slot_bonds(e);
    const int* sb_rev = sbm && e->fa.has_bonds ? e->brev : nullptr;
    int* sb_slot = sbm && e->fa.has_bonds ? e->bslot : nullptr;
    const int* sb_swt = sbm && e->fa.sw_n > 0 ? e->swt : nullptr;
    int* sb_swslot = sbm && e->fa.sw_n > 0 ? e->swslot : nullptr;
    if (sbm) islot = e->islot;
    const int mix = e->fa.has_pair ? e->fa.pair_mix : 1;
    const int* boff = e->fa.has_bonds ? e->boff : nullptr;
    if (e->prec == 64) {
        if (lists)
            launch_cell_sort(e->stream, e->ctx, e->dpos[0], e->dpos[1], e->dkmu, e->n, e->tmp, e->cell_of, e->cstart,
                             e->sidx, e->scell, e->spos, e->sb, mix, e->ptype, e->dpsort[0], e->dpsort[1], e->dskmu,
                             e->sbrow, boff, islot, e->psort[0], e->psort[1], sb_rev, sb_slot, sb_swt, sb_swslot);
        else
            launch_cell_sort(e->stream, e->ctx, e->dpos[0], e->dpos[1], e->dkmu, e->n, e->tmp, e->cell_of, e->cstart,
                             e->sidx, e->scell, e->spos, e->sb, mix);
    } else {
        if (lists)
            launch_cell_sort(e->stream, e->ctx, e->pos[0], e->pos[1], e->kmu, e->n, e->tmp, e->cell_of, e->cstart,
                             e->sidx, e->scell, e->spos, e->sb, mix, e->ptype, e->psort[0], e->psort[1], e->skmu,
                             e->sbrow, boff, islot, sb_rev, sb_slot, sb_swt, sb_swslot);
        else
            launch_cell_sort(e->stream, e->ctx, e->pos[0], e->pos[1], e->kmu, e->n, e->tmp, e->cell_of, e->cstart,
                             e->sidx, e->scell, e->spos, e->sb, mix);
    }
}

// scatter into the cells and order each cell by particle index
void enqueue_sort(gcs_engine* e)
{
    launch_cell_scatter(e->stream, e->n, e->cell_of, e->slot, e->cstart, e->tmp, e->count);
    enqueue_cell_order(e);
}

void enqueue_cells(gcs_engine* e)
{
    enqueue_bin(e);
    enqueue_sort(e);
}

// the dense-system switch applies to undecomposed runs (a decomposed run picks its shape when it is primed)
bool dense_switch(const gcs_engine* e) { return e->dense && !e->dom && e->prec != 64; }
// the step shape a fixed-timestep run takes (GCS_OPT_FUSED_STEP semantics): the list step (3) falls back to the
// rebuild step (2) when the system does not admit lists, and hands a dense chain to the unfused tile step (0)
int eff_fused(const gcs_engine* e)
{
    // the fp64 engine: the list step, or its cell-list step (list_ok false, or GCS_OPT_FUSED_STEP 0)
    if (e->prec == 64) return e->fused == 0 ? 0 : 3;
    if (e->fused != 3) return e->fused;
    if (!e->list_ok) return 2;
    return dense_switch(e) ? 0 : 3;
}
// the list step, and the relaxation (spacestep) step on the same lists (k_lstep<..., RLX> + k_lupdate) when the
// system admits lists; other spacestep runs take the cell-list evaluation (fp32: k_force + k_adapt + k_update, fp64:
// k_eval64 + k_red64 + k_update)
bool list_path(const gcs_engine* e, bool spacestep)
{
    return eff_fused(e) == 3 && e->list_ok && (!spacestep || !e->dom);
}
bool fused_path(const gcs_engine* e, bool spacestep) { return spacestep ? list_path(e, true) : eff_fused(e) != 0; }
bool rebuild_path(const gcs_engine* e, bool spacestep) { return eff_fused(e) == 2 && !spacestep; }

// the precision's default skin at core scale 1.  The fp64 step gathers 32-B partners, so shorter lists pay for more
// frequent rebuilds sooner than at fp32 (4-replica bench sweeps: fp32 profiles/r03_skin_sweep.txt, 500 per mille / 16
// steps best; fp64 profiles/r04_skin_sweep_f64*.txt)
// (GCS_OPT_LIST_SKIN_BASE replaces s1: one trajectory alone on a GPU, e.g. a stage CLI, is latency-bound and
// takes fewer rebuilds for longer lists -- profiles/r06g4_skin.txt)
int default_skin_pm(const gcs_engine* e)
{
    if (e->list_skin_base_pm > 0) return e->list_skin_base_pm;
    return e->prec == 64 ? kListSkinPm64 : kListSkinPm32;
}

// the list skin: the option, the current run's level (skin_level), or the default
float list_skin(const gcs_engine* e)
{
    const int pm = e->list_skin_pm > 0 ? e->list_skin_pm : e->skin_level_pm > 0 ? e->skin_level_pm : default_skin_pm(e);
    return 1e-3f * (float)pm * e->fa.pf.pair_dist;
}
// the largest skin any level takes (the option, or the default at core scale 1): what a decomposed run's binning halo
// is sized from, so a level change never needs a wider region
float list_skin_max(const gcs_engine* e)
{
    return 1e-3f * (float)(e->list_skin_pm > 0 ? e->list_skin_pm : default_skin_pm(e)) * e->fa.pf.pair_dist;
}

// The core scale the schedule gives step st (the closed form the tails evaluate, stage_interphase/
// simulation_driver_interphase.cpp:67-76), or -1 when the host cannot know it: no scale schedule on step time, or a
// cutoff that does not scale
double sched_cs(const gcs_engine* e, int64_t st)
{
    if ((e->sched_flags & 3) != 3 || !e->fa.pair_scaled || !(e->sched.core_scale_tau > 0)) return -1.0;
    const double t = (double)st * e->sched.timestep;
    return 1.0 - (1.0 - e->sched.core_scale_init) * std::exp(-(t / e->sched.core_scale_tau));
}

// The list skin of step st (1/1000 of the pair cutoff at core scale 1) when GCS_OPT_LIST_SKIN is 0: the precision's
// default s1 (the optimum at cs = 1) x sqrt(cs) at fp64, x cs at fp32, rounded to 10 per mille.  The list radius is
// rc(cs) + skin: per step a list costs ~ (rc + skin)^3, a rebuild (every M ~ kappa skin^2 steps, auto_list_every) some
// beta steps' worth, and at the production start (cs 0.5) a skin sized for cs = 1 makes the lists
// (0.5 + 0.35)^3 / 0.5^3 = 4.9 x the pairs they hold.  Minimising (cs + s)^3 (1 + beta / (kappa s^2)) with beta
// fixed by s1 being the optimum at cs = 1 gives u = s / s1 = 0.76 at cs 0.5; the sweeps put it lower
// (profiles/r04_skin_cs.txt; the build's cost grows with the list too): fp64 250 of 150..350 at C5's start (u 0.71),
// fp32 250 of 250..370 there (u 0.5; its C2 start window 370 > 500).
// The scheduled core scale is a closed form of the step, so the skin changes at steps the schedule fixes (a few
// times while cs grows; each change re-primes and rebuilds, gcs_engine_run), and a run split into chunks changes it
// where the whole run does.
int skin_level(const gcs_engine* e, int64_t st)
{
    if (e->list_skin_pm > 0) return e->list_skin_pm;
    const int s1 = default_skin_pm(e);
    const double cs = sched_cs(e, st);
    if (!(cs > 0.0) || cs >= 1.0) return s1;
    const double u = e->prec == 64 ? std::sqrt(cs) : cs;
    return std::max(50, (int)std::lround(s1 * u / 10.0) * 10);
}

void dbg_sync(gcs_engine* e, const char* what)
{
    static const bool on = std::getenv("GCS_DEBUG_SYNC") != nullptr;
    if (!on) return;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(e->stream, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone)
        return;  // (a graph being captured: nothing runs until it is launched)
    hipError_t he = hipStreamSynchronize(e->stream);
    if (he == hipSuccess) he = hipGetLastError();
    if (he != hipSuccess) std::fprintf(stderr, "GCS_DEBUG_SYNC: the stream failed after %s: %s\n", what, hipGetErrorString(he));
}

// the list entry format (GCS_OPT_LIST_FORMAT): 0 (default) absolute 16-bit slots up to 65,536 particles and
// plane-relative 16-bit slots beyond (kernels.hip ListRel16), 1 plane-relative at any size, 2 absolute 32-bit slots.
// Every format holds the same pairs in the same order: the trajectories are bitwise the same
int list_format(const gcs_engine* e)
{
    if (e->list_fmt_opt == 2) return kListFmtInt;
    if (e->list_fmt_opt == 1) return kListFmtRel16;
    return e->n <= 65536 ? kListFmtAbs16 : kListFmtRel16;
}

// the list build's chunk deal (kernels.hip deal_nth): the option, or the default for the waves per tile
unsigned long long list_deal(const gcs_engine* e)
{
    if (e->list_deal_opt != -1) return (unsigned long long)e->list_deal_opt;
    return e->list_waves == 2 ? kListDeal2 : kListDeal4;
}
// a deal pattern is valid for W waves when its period is 1..15 and every nibble of the period names a wave < W
bool deal_valid(long long d, int W)
{
    if (d == 0) return true;
    const int T = (int)((unsigned long long)d >> 60);
    if (T < 1 || T > 15) return false;
    for (int p = 0; p < 15; ++p) {
        const int w = (int)(((unsigned long long)d >> (4 * p)) & 15ull);
        if (p < T ? w >= W : w != 0) return false;
    }
    return true;
}

// the list step's argument block: the shared one plus the lists and the skin (> 0 also makes the prime and the
// tail build cell grids at cutoff + skin, so only list-path launches get it)
ForceArgs list_args(const gcs_engine* e)
{
    ForceArgs a = e->fa;
    a.list = e->list;
    a.lcount = e->lcount;
    a.ptype = e->ptype;
    a.psort0 = e->psort[0];
    a.psort1 = e->psort[1];
    a.skmu = e->skmu;
    a.dpsort0 = e->dpsort[0];
    a.dpsort1 = e->dpsort[1];
    a.dskmu = e->dskmu;
    a.dtype_ab = e->dtype_ab;
    a.sbrow = e->sbrow;
    a.lticket = e->lticket;
    a.type_ab = e->type_ab;
    a.ntypes = e->ntypes;
    a.list_cap = e->list_cap / e->list_waves;  // per (particle, wave) segment
    a.list_stride = (e->n + 63) & ~63;
    a.list_skin = list_skin(e);
    a.list_waves = e->list_waves;
    a.list_fmt = list_format(e);
    a.lbase = e->lbase;
    // the non-temporal hint beyond 16-bit absolute lists that the L2s keep (kernels.hip k_lstep)
    a.list_nt = (a.list_fmt == kListFmtRel16 || a.list_fmt == kListFmtInt) ? 1 : 0;
    a.list_deal = list_deal(e);
    a.par_hint = -1;
    if (slot_bonds(e)) {
        a.bslot = e->bslot;
        a.swslot = e->swslot;
    }
    return a;
}

#ifndef GCS_LIST_SLOT_BONDS
#define GCS_LIST_SLOT_BONDS 1  // 1: the list step reads bonded / droplet partners by slot (kernels.hip kLFlagPos)
#endif
// the undecomposed list step with slot-indexed partners: every partner of the particle-local terms is a bond CSR
// entry or a droplet target (no bending triples or kinetochore fibers: those read i +- 1, i +- 2 and poles by
// particle index -- the mitotic fields, whose stages run the small-system step anyway)
bool slot_bonds(const gcs_engine* e)
{
    return GCS_LIST_SLOT_BONDS && !e->dom && !e->fa.has_bend && !e->fa.has_tether && e->bslot != nullptr &&
           (!e->fa.has_bonds || e->brev_ok) && (e->fa.sw_n == 0 || e->swt != nullptr);
}

int ensure_list(gcs_engine* e)
{
    const size_t stride = (size_t)((e->n + 63) & ~63);
    const size_t need = stride * (size_t)e->list_cap;  // every segment layout fits: waves x (cap / waves)
    int rc;
    // slot-indexed partners (slot_bonds): particle -> slot, and the partners' slots (k_lbuild writes them); sized
    // by the current bond table (a topology change may grow it: graphs holding the old pointer are dropped)
    if (GCS_LIST_SLOT_BONDS && !e->dom && (!e->bslot || e->nbent > e->bslot_cap)) {
        dfree(e->bslot);
        dfree(e->swslot);
        e->bslot_cap = std::max(1, e->nbent);
        if ((!e->islot && (rc = dalloc(&e->islot, e->n))) || (rc = dalloc(&e->bslot, e->bslot_cap)) ||
            (rc = dalloc(&e->swslot, 64)))
            return rc;
        drop_graph(e);
    }
    if (need <= e->list_alloc && e->lcount) return GCS_OK;
    dfree(e->list);
    dfree(e->lcount);
    dfree(e->lbase);
    dfree(e->psort[0]);
    dfree(e->psort[1]);
    dfree(e->skmu);
    dfree(e->sbrow);
    dfree(e->dpsort[0]);
    dfree(e->dpsort[1]);
    dfree(e->dskmu);
    e->list_alloc = 0;
    if ((rc = dalloc(&e->list, need)) || (rc = dalloc(&e->lcount, stride * kMaxListWaves)) ||
        (rc = dalloc(&e->lbase, stride)) || (rc = dalloc(&e->sbrow, stride)))
        return rc;
    if (e->prec == 64) {  // the slot-ordered copies in the engine's precision (+ the prefilter's fp32 copies, psort)
        if ((rc = dalloc(&e->dpsort[0], stride)) || (rc = dalloc(&e->dpsort[1], stride)) ||
            (rc = dalloc(&e->dskmu, stride)) ||
            (GCS_LIST_PREFILTER && ((rc = dalloc(&e->psort[0], stride)) || (rc = dalloc(&e->psort[1], stride)))))
            return rc;
    } else {
        if ((rc = dalloc(&e->psort[0], stride)) || (rc = dalloc(&e->psort[1], stride)) || (rc = dalloc(&e->skmu, stride)))
            return rc;
    }
    if (!e->lticket) {
        // arrival counters 0, the launch accumulators at their identities (k_lstep resets them after every launch)
        if ((rc = dalloc(&e->lticket, kListTicketWords))) return rc;
        std::vector<unsigned> h(kListTicketWords, 0u);
        for (int k = 0; k < 8 * (kListAccSlots + 1); ++k) {
            const unsigned long long v = list_acc_identity(k % (kListAccSlots + 1));
            std::memcpy(&h[kListAccBase + 32 * k], &v, sizeof(v));
        }
        HIPCHK(hipMemcpyAsync(e->lticket, h.data(), h.size() * sizeof(unsigned), hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    // GCS_DEBUG_POISON (tests): the per-slot buffers start as hashed garbage instead of whatever the allocator hands
    // out (fresh pages are zero, a recycled allocation is not): every read of a slot the current build did not write
    // then shows up -- the round-5 decomposed fault (k_cell_sort's sentinel records)
    if (std::getenv("GCS_DEBUG_POISON")) {
        launch_poison(e->stream, e->lcount, stride * kMaxListWaves * sizeof(int));
        launch_poison(e->stream, e->lbase, stride * sizeof(int4));
        launch_poison(e->stream, e->sbrow, stride * sizeof(int2));
        if (e->prec == 64) {
            launch_poison(e->stream, e->dpsort[0], stride * sizeof(double4));
            launch_poison(e->stream, e->dpsort[1], stride * sizeof(double4));
            launch_poison(e->stream, e->dskmu, stride * sizeof(double4));
        } else {
            launch_poison(e->stream, e->psort[0], stride * sizeof(float4));
            launch_poison(e->stream, e->psort[1], stride * sizeof(float4));
            launch_poison(e->stream, e->skmu, stride * sizeof(float4));
        }
        HIPCHK(hipGetLastError());
    }
    // entries past a slot's count are read (never gathered): keep them defined
    HIPCHK(hipMemsetAsync(e->list, 0, need * sizeof(int), e->stream));
    e->list_alloc = need;
    return GCS_OK;
}

// rebuild period: the skin must hold the largest displacement of ~4.15 sigma on each side of a pair for that many
// steps (sigma = sqrt(2 T mu_max dt) per step; C2: 16 steps at skin 0.5 rc); the rare particle that outruns it is
// searched exactly (k_lstep), so the period trades rebuild cost against fallbacks, never correctness.  Skin and
// factor from a sweep on the bench (profiles/r03_skin_sweep.txt: 4 replicas, bead-updates/s): skin 0.4 / M 8 (4.5 sigma)
// 6.17e9, 0.45 / 14 6.33e9, 0.5 / 13 6.27e9, 0.5 / 16 6.32e9, 0.5 / 18 6.1e9, 0.55 / 18 6.13e9, 0.6 / 20 5.97e9
// (C2's largest mobility 1, dt 1e-5: (0.075 / (4.15 sigma))^2 = 16.3 -> 16; 3.95 sigma gave 18, whose fallbacks
// reach 1.7e-3 of the particle-steps over 20,000 C2 steps)
int auto_list_every(const gcs_engine* e, double temperature, double timestep)
{
    if (e->list_every_opt > 0) return e->list_every_opt;
    double mu = 0;
    for (double m : e->mu) mu = std::max(mu, m);
    const double sigma = std::sqrt(2.0 * std::max(temperature, 0.0) * mu * timestep);
    const double half = 0.5 * (double)list_skin(e);
    if (!(sigma > 0)) return 64;
    const double m = std::floor((half / (4.15 * sigma)) * (half / (4.15 * sigma)));
    return (int)std::min(64.0, std::max(1.0, m));
}

// k_lstep launch flags of the step that starts at step index st: the schedule; the bounding box when the next step
// rebuilds (its grid); neighbour-count statistics on those steps too (ctx->neighbors)
int list_flags(const gcs_engine* e, int64_t st)
{
    const bool next_build = ((st + e->list_phase + 1) % e->list_every) == 0;
    return (e->sched_flags != 0 ? 1 : 0) | (next_build ? 2 | 4 | 16 : 0);  // 16: kLFlagPos
}

// one list step: on a rebuild step the cell list at cutoff + skin (ctx->grid, set by the prime or the last
// bounding-box step's tail), the lists, then the step itself (forces + local terms + update + tail in the final
// workgroup)
void enqueue_list_step(gcs_engine* e, bool build, int lflags, double contact = 0, int parity = -1,
                       const gcs_bd_config* relax = nullptr)
{
    ForceArgs la = list_args(e);
    la.par_hint = parity;
    if (relax) {
        la.relax_spacestep = relax->spacestep;
        la.relax_timestep = relax->timestep;
    }
    if (contact > 0) {  // the pending contact update, counted from this step's start positions (its distance: ctx)
        la.contact_on = 1;
        la.c_keys = e->c_keys;
        la.c_counts = e->c_counts;
        la.c_bits = e->c_bits;
        la.c_overflow = e->c_flags;
    }
    if (build) {
        enqueue_count(e);
        enqueue_scan(e, false);
        launch_cell_scatter(e->stream, e->n, e->cell_of, e->slot, e->cstart, e->tmp, e->count);
        enqueue_cell_order(e, true);
        launch_list_build(e->stream, e->ctx, la);
    }
    if (relax)  // neighbour statistics from the force launch; the schedule and the next build's grid from the update
        launch_list_relax(e->stream, e->ctx, la, lflags & 4, lflags & (1 | 2));
    else
        launch_list_step(e->stream, e->ctx, la, lflags);
}
int step_grid(const gcs_engine* e) { return e->fa.split ? force_grid_split(e->n) : force_grid(e->n); }

// One BD step.  Rebuild (fixed timestep, 2 launches, default): force + update, which also files the new positions
// under the predicted next grid's cells; k_rebuild scans, builds the tile table and the cell-sorted copies from
// those buckets, and runs the step's tail in its block 0.  begin_run built the first cell list.
// Fused (fixed timestep, 4 launches): sort the cells the previous step scattered; force + update,
// which also bins the new positions into the predicted next grid; scan those counts; scatter them, with the
// step's tail (reduction, schedule, wall, grid rotation) in one extra block.  begin_run binned, scanned and
// scattered the first positions.  Otherwise (spacestep, or fusion off): count, scan, scatter, sort, force,
// [adapt, update], tail.
void enqueue_step(gcs_engine* e, bool spacestep, double spacestep_v, double timestep)
{
    if (e->prec == 64) {
        // fp64 without the list step (spacestep relaxation off the lists; any run of a system the list step does not
        // admit: no pair field, > 256 pair classes): cells, the fp64 force pass, its reduction (reactions, max drift
        // -> the adapted dt; spacestep 0: the fixed timestep), the update, the tail with those reactions
        enqueue_cells(e);
        launch_eval64(e->stream, kModeForce, e->ctx, e->fa);
        launch_red64(e->stream, e->ctx, e->fa, spacestep ? spacestep_v : 0.0, timestep, e->dred);
        launch_update(e->stream, e->ctx, e->fa);
        ForceArgs t = e->fa;
        t.ext_react = e->dred;
        launch_tail(e->stream, e->ctx, t, 0, update_blocks(e->n), 1, e->sched_flags != 0, e->ncell_max, e->dsched);
        return;
    }
    const int fb = force_grid(e->n);
    const int sb = step_grid(e);  // kModeStep launch size (split tiles: two units per tile)
    if (rebuild_path(e, spacestep)) {
        launch_force(e->stream, kModeStep, e->waves, e->ctx, e->fa, true);
        launch_rebuild(e->stream, e->ctx, e->fa, e->tmp, e->rb_sync, sb, e->sched_flags != 0);
        return;
    }
    enqueue_cells(e);
    if (!spacestep) {
        launch_force(e->stream, kModeStep, e->waves, e->ctx, e->fa, false);
        launch_tail(e->stream, e->ctx, e->fa, sb, sb, 1, e->sched_flags != 0, e->ncell_max, e->dsched);
    } else {
        launch_force(e->stream, kModeForce, e->waves, e->ctx, e->fa, false);
        launch_adapt(e->stream, e->ctx, e->fa, fb, (float)spacestep_v, (float)timestep);
        launch_update(e->stream, e->ctx, e->fa);
        launch_tail(e->stream, e->ctx, e->fa, fb, update_blocks(e->n), 1, e->sched_flags != 0, e->ncell_max, e->dsched);
    }
}

int upload_sched(gcs_engine* e)
{
    double h[kSchedCount] = {0};
    const gcs_schedule& s = e->sched;
    e->sched_flags = (s.update_time ? 1 : 0) | (s.update_scales ? 2 : 0) | (s.update_wall ? 4 : 0);
    h[kSchedFlags] = e->sched_flags;
    h[kSchedDt] = s.timestep;
    h[kSchedCs0] = s.core_scale_init;
    h[kSchedCsTau] = s.core_scale_tau;
    h[kSchedBs0] = s.bond_scale_init;
    h[kSchedBsTau] = s.bond_scale_tau;
    for (int k = 0; k < 3; ++k) h[kSchedK0 + k] = s.wall_semiaxes_spring[k];
    h[kSchedMuW] = s.wall_mobility;
    HIPCHK(hipMemcpyAsync(e->dsched, h, sizeof(h), hipMemcpyHostToDevice, e->stream));
    return GCS_OK;
}

int set_ctx_field(gcs_engine* e, size_t offset, const void* src, size_t bytes)
{
    HIPCHK(hipMemcpyAsync((char*)e->ctx + offset, src, bytes, hipMemcpyHostToDevice, e->stream));
    return GCS_OK;
}

int prepare(gcs_engine* e)
{
    HIPCHK(hipSetDevice(e->device));
    int rc = compile(e);
    if (rc) return rc;
    fill_state_args(e);
    return GCS_OK;
}

int ensure_search(gcs_engine* e, int64_t n);
int enqueue_search_cells(gcs_engine* e, const float4* src, const double4* src64, int ni, double distance);

// The step shape of a fresh chain: the list step walks ~2.5 x (neighbours within the cutoff) entries per particle
// with one gather each, the tile step shares each staged candidate among a tile's 64 lanes, so above a density the
// unfused tile step is faster.  Measured single-trajectory bead-updates/s (tools/shape_probe.py):
// C2 window, 25 neighbours, 16-bit entries: list 2.32e9 / tile 1.09e9; C2 start, 32: 1.44e9 / 1.05e9; C5 start, 43,
// 32-bit entries: 1.34e9 / 2.37e9 (the rebuild step: 0.6e9, its 16-slot cell buckets overflow there).  So the
// verdict weighs the neighbour count by the entry size (list bytes per particle): dense when mean neighbours x
// (entry bytes / 2) exceeds GCS_OPT_DENSE_NEIGHBORS.  The mean over the current positions within the current cutoff
// (the neighbour search's count kernel) decides once per chain, so a chain's trajectory is reproducible.
int probe_density(gcs_engine* e)
{
    // (rocprofv3 --kernel-trace segfaults in the first graph launch after this probe, measured with every variant of
    // its copies and kernels; profiling runs turn the probe off: GCS_OPT_DENSE_NEIGHBORS 0, tools/profile.sh)
    double cs = 1.0;
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpyAsync(&cs, (const char*)e->ctx + offsetof(DevCtx, cs), sizeof(cs), hipMemcpyDeviceToHost,
                          e->stream));  // (the engine's stream: no legacy null-stream work anywhere in the library)
    HIPCHK(hipStreamSynchronize(e->stream));
    const double rc = (double)e->fa.pf.pair_dist * (e->fa.pair_scaled ? cs : 1.0);
    int rc_;
    if (!(rc > 0) || e->n < 2) return GCS_OK;
    if ((rc_ = ensure_search(e, e->n))) return rc_;
    if ((rc_ = enqueue_search_cells(e, e->pos[e->parity], nullptr, e->n, rc))) return rc_;
    launch_search_count(e->stream, e->s_ctx, e->n, e->s_spos, e->s_sidx, e->s_scell, e->s_cstart, e->s_counts);
    launch_exclusive_scan_small(e->stream, e->s_counts, e->s_offsets, e->n, e->s_total);
    HIPCHK(hipGetLastError());
    int pairs = 0;
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpyAsync(&pairs, e->s_total, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->dense_mean = 2.0 * pairs / (double)e->n;
    e->dense = e->dense_mean * (list_format(e) == kListFmtInt ? 2.0 : 1.0) > (double)e->dense_opt;
    return GCS_OK;
}

// before a run of the default shape: a fresh undecomposed chain probes the density (the verdict holds while the
// chain continues)
int choose_shape(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step)
{
    int rc = prepare(e);
    if (rc) return rc;
    if (e->fused != 3 || e->dense_opt <= 0 || !e->list_ok || e->prec == 64) {
        e->dense = false;
        return GCS_OK;
    }
    const bool same = e->chain_step == first_step && e->chain_version == e->topo_version;
    const bool cont = same && (e->chain_valid || (e->dense && e->dense_chain));
    if (e->dom || cfg->spacestep > 0 || cont) return GCS_OK;
    const bool was = e->dense;
    if ((rc = probe_density(e))) return rc;
    e->rstats.density_probes++;
    if (e->dense != was) e->chain_valid = false;
    return GCS_OK;
}

// compile, load the BD parameters into the kernel arguments, set the step counter, build the first grid
int begin_run(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step)
{
    int rc = prepare(e);
    if (rc) return rc;
    ForceArgs& a = e->fa;
    a.pf.temperature = (float)cfg->temperature;
    a.pf.timestep = (float)cfg->timestep;
    a.pd.temperature = cfg->temperature;
    a.pd.timestep = cfg->timestep;
    a.seed_lo = (unsigned)cfg->seed;
    a.seed_hi = (unsigned)(cfg->seed >> 32);
    a.noise_mode = cfg->noise;
    const bool fused = fused_path(e, cfg->spacestep > 0);
    const bool cont = fused && e->chain_valid && e->chain_step == first_step && e->chain_version == e->topo_version;
    // a continuing list-step chain at the same timestep already has ctx->step == first_step (its tails counted the
    // steps) and this dt_used (only spacestep changes it): no host copy, which from pageable memory would stall the
    // host until the stream drained (the interphase driver runs a chunk per contact update, every 20 steps)
    if (!(cont && list_path(e, cfg->spacestep > 0) && e->chain_dt == cfg->timestep)) {
        long long st = first_step;
        if ((rc = set_ctx_field(e, offsetof(DevCtx, step), &st, sizeof(st)))) return rc;
        double dt = cfg->timestep;
        if ((rc = set_ctx_field(e, offsetof(DevCtx, dt_used), &dt, sizeof(dt)))) return rc;
    }
    e->chain_dt = cfg->timestep;
    e->chain_valid = false;
    if (list_path(e, cfg->spacestep > 0)) {
        if ((rc = ensure_list(e))) return rc;
        e->list_every = auto_list_every(e, cfg->temperature, cfg->timestep);
        if (!cont) {
            launch_prime(e->stream, e->ctx, list_args(e), 0.f, e->ncell_max, e->dsched);
            e->l_need_build = true;
        }
    } else if (!cont) {
        launch_prime(e->stream, e->ctx, a, 0.f, e->ncell_max, e->dsched);
        if (rebuild_path(e, cfg->spacestep > 0)) {
            enqueue_cells(e);  // the first cell list; the steps rebuild it from the force kernel's buckets
            HIPCHK(hipMemsetAsync(e->ovf_n, 0, 2 * sizeof(int), e->stream));
        }
    }
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

// The cached graph of `len` steps from rebuild phase `phase` and parity `parity`, captured by `body` on a miss
// (the least recently used entry makes room).  `key` is what the run would capture under: a different key than
// the cache's drops the whole cache first.
template <class Body>
int cached_graph(gcs_engine* e, const GraphKey& key, int phase, int parity, int len, Body body, hipGraphExec_t* out)
{
    if (!e->g_key_set || !same_key(e->g_key, key)) {
        drop_graph(e);
        e->g_key = key;
        e->g_key_set = true;
    }
    for (GraphEntry& g : e->graphs)
        if (g.phase == phase && g.parity == parity && g.len == len) {
            g.used = ++e->graph_clock;
            *out = g.exec;
            return GCS_OK;
        }
    if (e->graphs.size() >= kMaxGraphs) {
        auto lru = std::min_element(e->graphs.begin(), e->graphs.end(),
                                    [](const GraphEntry& x, const GraphEntry& y) { return x.used < y.used; });
        HIPCHK(hipStreamSynchronize(e->stream));  // it may still be executing
        (void)hipGraphExecDestroy(lru->exec);
        (void)hipGraphDestroy(lru->graph);
        e->graphs.erase(lru);
    }
    GraphEntry g{phase, parity, len, nullptr, nullptr, ++e->graph_clock};
    HIPCHK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
    body();
    HIPCHK(hipStreamEndCapture(e->stream, &g.graph));
    const hipError_t he = hipGraphInstantiate(&g.exec, g.graph, nullptr, nullptr, 0);
    if (he != hipSuccess) {
        (void)hipGraphDestroy(g.graph);
        return fail(GCS_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(he));
    }
    e->graphs.push_back(g);
    e->rstats.graphs_captured++;
    *out = g.exec;
    return GCS_OK;
}

// hipGraphLaunch with the engine's run-ahead bound (see gcs_engine::inflight)
int launch_graph(gcs_engine* e, hipGraphExec_t x)
{
    hipEvent_t& ev = e->inflight[e->inflight_n % kInflight];
    if (!ev) {
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    } else if (e->inflight_n >= (unsigned long long)kInflight) {
        HIPCHK(hipEventSynchronize(ev));
    }
    HIPCHK(hipGraphLaunch(x, e->stream));
    HIPCHK(hipEventRecord(ev, e->stream));
    e->inflight_n++;
    e->rstats.graph_launches++;
    return GCS_OK;
}

GraphKey run_key(const gcs_engine* e, const gcs_bd_config* cfg, bool spacestep)
{
    GraphKey k;
    std::memset(&k, 0, sizeof(k));
    k.topo_version = e->topo_version;
    k.fused = eff_fused(e);  // the shape the run takes
    k.list_every = e->list_every;
    k.sched_flags = e->sched_flags;
    k.waves = e->waves;
    k.chunk = e->fa.chunk_mode;
    k.spacestep = spacestep ? 1 : 0;
    k.list_waves = e->list_waves;
    k.skin_pm = e->skin_level_pm;
    k.cfg = *cfg;
    return k;
}

int flush_contacts(gcs_engine* e);  // (below)

// after a run's steps were enqueued
void end_run(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps)
{
    e->chain_valid = fused_path(e, cfg->spacestep > 0);
    e->dense_chain = dense_switch(e) && cfg->spacestep <= 0;
    e->chain_step = first_step + steps;
    e->chain_version = e->topo_version;
}

}  // namespace

// ------------------------------------------------------------------------------------------------------
// RCCL, opened at first use (no link-time dependency: only decomposed multi-GPU runs need it; a process that has
// already loaded a librccl.so.1, e.g. torch's, shares that one through the soname)

namespace {

struct RcclApi {
    bool tried = false;
    void* h = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
};
RcclApi g_rccl;

const RcclApi* rccl()
{
    if (!g_rccl.tried) {
        g_rccl.tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            g_rccl.getUniqueId = (decltype(g_rccl.getUniqueId))dlsym(h, "ncclGetUniqueId");
            g_rccl.commInitRank = (decltype(g_rccl.commInitRank))dlsym(h, "ncclCommInitRank");
            g_rccl.commDestroy = (decltype(g_rccl.commDestroy))dlsym(h, "ncclCommDestroy");
            g_rccl.allReduce = (decltype(g_rccl.allReduce))dlsym(h, "ncclAllReduce");
            g_rccl.send = (decltype(g_rccl.send))dlsym(h, "ncclSend");
            g_rccl.recv = (decltype(g_rccl.recv))dlsym(h, "ncclRecv");
            g_rccl.groupStart = (decltype(g_rccl.groupStart))dlsym(h, "ncclGroupStart");
            g_rccl.groupEnd = (decltype(g_rccl.groupEnd))dlsym(h, "ncclGroupEnd");
            g_rccl.errorString = (decltype(g_rccl.errorString))dlsym(h, "ncclGetErrorString");
            if (g_rccl.getUniqueId && g_rccl.commInitRank && g_rccl.commDestroy && g_rccl.allReduce && g_rccl.send &&
                g_rccl.recv && g_rccl.groupStart && g_rccl.groupEnd && g_rccl.errorString)
                g_rccl.h = h;
        }
    }
    return g_rccl.h ? &g_rccl : nullptr;
}

void rccl_comm_destroy(ncclComm_t c)
{
    if (const RcclApi* r = rccl()) (void)r->commDestroy(c);
}

#define NCCLCHK(expr)                                                                                         \
    do {                                                                                                      \
        ncclResult_t _r = (expr);                                                                             \
        if (_r != ncclSuccess) return fail(GCS_EHIP, std::string(#expr) + ": " + rccl()->errorString(_r));   \
    } while (0)

}  // namespace

// ------------------------------------------------------------------------------------------------------
// C ABI

namespace {

// search scratch (neighbour search, contact map) for up to n points
int ensure_search(gcs_engine* e, int64_t n)
{
    if (n <= e->search_cap) return GCS_OK;
    int rc;
    dfree(e->s_pts);
    dfree(e->s_spos);
    dfree(e->s_sb);
    dfree(e->s_sidx);
    dfree(e->s_scell);
    dfree(e->s_cell_of);
    dfree(e->s_slot);
    dfree(e->s_tmp);
    dfree(e->s_count);
    dfree(e->s_cstart);
    dfree(e->s_tile);
    dfree(e->s_tile_range);
    dfree(e->s_counts);
    dfree(e->s_offsets);
    dfree(e->s_total);
    dfree(e->s_ctx);
    dfree(e->s_scan_sync);
    e->search_cap = 0;
    const int cap = (int)n;
    const int ncm = std::min(1 << 21, std::max(4096, 4 * cap));
    if ((rc = dalloc(&e->s_pts, cap)) || (rc = dalloc(&e->s_spos, cap)) || (rc = dalloc(&e->s_sb, cap)) ||
        (rc = dalloc(&e->s_sidx, cap)) || (rc = dalloc(&e->s_scell, cap)) || (rc = dalloc(&e->s_cell_of, cap)) ||
        (rc = dalloc(&e->s_slot, cap)) || (rc = dalloc(&e->s_tmp, cap)) || (rc = dalloc(&e->s_count, ncm + kScanPad)) ||
        (rc = dalloc(&e->s_cstart, ncm + kScanPad)) || (rc = dalloc(&e->s_counts, cap)) ||
        (rc = dalloc(&e->s_tile, ncm + 2)) || (rc = dalloc(&e->s_tile_range, (size_t)force_blocks(cap) + ncm + 2)) ||
        (rc = dalloc(&e->s_offsets, cap)) || (rc = dalloc(&e->s_total, 1)) || (rc = dalloc(&e->s_ctx, 1)) ||
        (rc = dalloc(&e->s_scan_sync, scan_sync_words(ncm))))
        return rc;
    HIPCHK(hipMemsetAsync(e->s_count, 0, (ncm + kScanPad) * sizeof(int), e->stream));
    HIPCHK(hipMemsetAsync(e->s_scan_sync, 0, scan_sync_words(ncm) * sizeof(unsigned long long), e->stream));
    e->search_cap = cap;
    e->s_ncell_max = ncm;
    return GCS_OK;
}

// the search cell list (grid edge >= distance) of n points at src (fp32) or src64 (fp64: binned by their roundings),
// on the engine stream, no host sync: s_spos / s_sidx / s_scell / s_cstart and s_ctx->grid
int enqueue_search_cells(gcs_engine* e, const float4* src, const double4* src64, int ni, double distance)
{
    // the source outlives the (possibly deferred) async copy: it is a member of the engine
    e->s_ctx_host = DevCtx{};
    e->s_ctx_host.cs = 1.0;
    e->s_ctx_host.bs = 1.0;
    HIPCHK(hipMemcpyAsync(e->s_ctx, &e->s_ctx_host, sizeof(DevCtx), hipMemcpyHostToDevice, e->stream));
    ForceArgs sa{};
    sa.n = ni;
    sa.prec = src64 ? 64 : 32;
    sa.pos0 = const_cast<float4*>(src);
    sa.pos1 = const_cast<float4*>(src);
    sa.dpos0 = const_cast<double4*>(src64);
    sa.dpos1 = const_cast<double4*>(src64);
    launch_prime(e->stream, e->s_ctx, sa, (float)distance, e->s_ncell_max, nullptr);
    if (src64)
        launch_cell_count(e->stream, e->s_ctx, src64, src64, ni, e->s_cell_of, e->s_slot, e->s_count);
    else
        launch_cell_count(e->stream, e->s_ctx, src, src, ni, e->s_cell_of, e->s_slot, e->s_count);
    launch_cell_scan(e->stream, e->s_ctx, ni, e->s_count, e->s_cstart, e->s_tile, e->s_tile_range, false, nullptr, 0,
                     e->scan_mb ? e->s_scan_sync : nullptr, e->s_ncell_max);
    launch_cell_scatter(e->stream, ni, e->s_cell_of, e->s_slot, e->s_cstart, e->s_tmp, e->s_count);
    if (src64)
        launch_cell_sort(e->stream, e->s_ctx, src64, src64, (const double4*)nullptr, ni, e->s_tmp, e->s_cell_of,
                         e->s_cstart, e->s_sidx, e->s_scell, e->s_spos, e->s_sb, 1);
    else
        launch_cell_sort(e->stream, e->s_ctx, src, src, nullptr, ni, e->s_tmp, e->s_cell_of, e->s_cstart, e->s_sidx,
                         e->s_scell, e->s_spos, e->s_sb, 1);
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

// count every pair of the current positions closer than `distance` into the contact table (allocated)
int contacts_insert_now(gcs_engine* e, double distance)
{
    int rc;
    if (e->prec != 64 && e->fused == 2 && e->chain_valid) {
        // right after a rebuild-step run the engine's own cell list holds the current positions (k_rebuild built
        // it from the records the last force kernel filed): no cell build of our own
        launch_contact_insert(e->stream, e->ctx, e->n, distance, e->spos, e->sidx, e->scell, e->cstart,
                              e->c_keys, e->c_counts, e->c_bits, e->c_flags);
    } else {
        if ((rc = ensure_search(e, e->n))) return rc;
        const double4* p64 = e->prec == 64 ? e->dpos[e->parity] : nullptr;
        if ((rc = enqueue_search_cells(e, e->pos[e->parity], p64, e->n, distance))) return rc;
        launch_contact_insert(e->stream, e->s_ctx, e->n, distance, e->s_spos, e->s_sidx, e->s_scell,
                              e->s_cstart, e->c_keys, e->c_counts, e->c_bits, e->c_flags, p64);
    }
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

// a contact update deferred into the next list step is done now instead (positions or the table are about to be
// changed or read by something other than that step)
int flush_contacts(gcs_engine* e)
{
    if (!(e->c_pending > 0)) return GCS_OK;
    const double d = e->c_pending;
    e->c_pending = 0;
    HIPCHK(hipSetDevice(e->device));
    return contacts_insert_now(e, d);
}

}  // namespace

extern "C" {

const char* gcs_last_error(void) { return g_last_error.c_str(); }

int gcs_abi_version(void) { return GCS_ABI_VERSION; }

int gcs_device_count(int32_t* count)
{
    int c = 0;
    HIPCHK(hipGetDeviceCount(&c));
    *count = c;
    return GCS_OK;
}

int gcs_engine_create(const gcs_system_desc* d, gcs_engine** out)
{
    if (!d || !out) return fail(GCS_EINVAL, "null argument");
    *out = nullptr;
    if (d->particle_count <= 0 || d->particle_count > (int64_t)1 << 30)
        return fail(GCS_EINVAL, "particle_count must be in [1, 2^30]");
    if (d->precision != GCS_PRECISION_DEFAULT && d->precision != GCS_PRECISION_F32 && d->precision != GCS_PRECISION_F64)
        return fail(GCS_EINVAL, "precision must be 0 (default: fp64), 32 or 64");
    gcs_engine* e = new gcs_engine();
    e->device = d->device;
    e->prec = d->precision == GCS_PRECISION_F32 ? 32 : 64;
    e->n = (int)d->particle_count;
    e->fa.chunk_mode = 1;  // strided candidate chunks (GCS_OPT_CHUNK_ORDER)
    e->fa.split = 0;       // split tiles (GCS_OPT_SPLIT_TILES): 1 and 2 measured slower on C2
    e->fa.prio_step = 700; // tile-cost wave priority (GCS_OPT_TILE_PRIORITY): +2 % on C2
    e->fa.subtiles = 2;    // per-group stencils (GCS_OPT_SUBTILES)
    const int n = e->n;
    e->mu.assign(n, 1.0);
    e->ab.assign(2 * (size_t)n, 0.0);
    for (int i = 0; i < n; ++i) {
        if (d->mobilities) e->mu[i] = d->mobilities[i];
        if (d->ab_factors) {
            e->ab[2 * i] = d->ab_factors[2 * i];
            e->ab[2 * i + 1] = d->ab_factors[2 * i + 1];
        }
    }
    auto bail = [&](int rc) {
        gcs_engine_destroy(e);
        return rc;
    };
    hipError_t he = hipSetDevice(e->device);
    if (he != hipSuccess) return bail(fail(GCS_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(he)));
    he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) return bail(fail(GCS_EHIP, std::string("hipStreamCreate: ") + hipGetErrorString(he)));
    e->ncell_max = std::min(1 << 21, std::max(4096, 4 * n));
    int rc = 0;
    const int fb = force_grid_split(n), ub = update_blocks(n);  // partial rows for the largest launch
    if ((rc = dalloc(&e->pos[0], n)) || (rc = dalloc(&e->pos[1], n)) || (rc = dalloc(&e->kmu, n)) ||
        (rc = dalloc(&e->spos, n)) || (rc = dalloc(&e->sb, n)) || (rc = dalloc(&e->sidx, n)) ||
        (rc = dalloc(&e->scell, n)) || (rc = dalloc(&e->cell_of, n)) || (rc = dalloc(&e->slot, n)) ||
        (rc = dalloc(&e->tmp, n)) || (rc = dalloc(&e->count, e->ncell_max + kScanPad)) ||
        (rc = dalloc(&e->cstart, e->ncell_max + kScanPad)) || (rc = dalloc(&e->tile_start, e->ncell_max + 2)) ||
        (rc = dalloc(&e->tile_range, (size_t)force_blocks(n) + e->ncell_max + 2)) ||
        (rc = dalloc(&e->ctx, 1)) || (rc = dalloc(&e->dsched, kSchedCount)) ||
        (rc = dalloc(&e->part_force, (size_t)(std::max(fb, ub) + 8) * kForcePartials)) ||  // + the list step's
        (rc = dalloc(&e->part_bbox, (size_t)(std::max(fb, ub) + 8) * kBBoxStride)) ||       // 8 group rows
        (rc = dalloc(&e->part_energy, (size_t)std::max(fb, eval64_blocks(n)) * kEnergyKinds)) ||
        (rc = dalloc(&e->force_out, n)) ||
        (rc = dalloc(&e->pbuf, (size_t)2 * std::max(force_grid(n), kMaxUnits) * kTile)) ||
        (rc = dalloc(&e->tcnt, std::max(force_grid(n), kMaxUnits))) || (rc = dalloc(&e->units, 2 * kMaxUnits)) ||
        (rc = dalloc(&e->scan_sync, scan_sync_words(e->ncell_max))) ||
        (rc = dalloc(&e->bucket_p, (size_t)e->ncell_max * kBucketCap)) ||
        (rc = dalloc(&e->bucket_q, (size_t)e->ncell_max * kBucketCap)) || (rc = dalloc(&e->ovf_p, n)) ||
        (rc = dalloc(&e->ovf_q, n)) ||
        (rc = dalloc(&e->ovf_n, 2)) || (rc = dalloc(&e->rb_sync, rebuild_sync_words(e->ncell_max))))
        return bail(rc);
    he = hipMemsetAsync(e->count, 0, (e->ncell_max + kScanPad) * sizeof(int), e->stream);
    if (he == hipSuccess)
        he = hipMemsetAsync(e->scan_sync, 0, scan_sync_words(e->ncell_max) * sizeof(unsigned long long), e->stream);
    if (he == hipSuccess)
        he = hipMemsetAsync(e->rb_sync, 0, rebuild_sync_words(e->ncell_max) * sizeof(unsigned long long), e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->ovf_n, 0, 2 * sizeof(int), e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->tcnt, 0, std::max(force_grid(n), kMaxUnits) * sizeof(int), e->stream);
    e->resident = std::min(force_step_resident(e->waves), kMaxUnits);
    if (he == hipSuccess) he = hipMemsetAsync(e->pos[0], 0, n * sizeof(float4), e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->pos[1], 0, n * sizeof(float4), e->stream);
    if (e->prec == 64) {  // the fp64 state (the fp32 pos buffers above stay allocated but unused: a few MB)
        if ((rc = dalloc(&e->dpos[0], n)) || (rc = dalloc(&e->dpos[1], n)) || (rc = dalloc(&e->dkmu, n)) ||
            (rc = dalloc(&e->dforce_out, n)) || (rc = dalloc(&e->dpart, (size_t)eval64_blocks(n) * 8)) ||
            (rc = dalloc(&e->dred, 8)))
            return bail(rc);
        if (he == hipSuccess) he = hipMemsetAsync(e->dpos[0], 0, n * sizeof(double4), e->stream);
        if (he == hipSuccess) he = hipMemsetAsync(e->dpos[1], 0, n * sizeof(double4), e->stream);
    }
    DevCtx c{};
    c.cs = 1.0;
    c.bs = 1.0;
    if (he == hipSuccess) he = hipMemcpyAsync(e->ctx, &c, sizeof(c), hipMemcpyHostToDevice, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he != hipSuccess) return bail(fail(GCS_EHIP, std::string("engine init: ") + hipGetErrorString(he)));
    if ((rc = upload_sched(e))) return bail(rc);
    *out = e;
    return GCS_OK;
}

int gcs_engine_destroy(gcs_engine* e)
{
    if (!e) return GCS_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    drop_graph(e);
    for (hipEvent_t& ev : e->inflight)
        if (ev) (void)hipEventDestroy(ev);
    dfree(e->pos[0]);
    dfree(e->pos[1]);
    dfree(e->kmu);
    dfree(e->sw_idx);
    dfree(e->list);
    dfree(e->lcount);
    dfree(e->lbase);
    dfree(e->psync);
    dfree(e->pstall);
    dfree(e->pkeep);
    dfree(e->psort[0]);
    dfree(e->psort[1]);
    dfree(e->skmu);
    dfree(e->sbrow);
    dfree(e->lticket);
    dfree(e->ptype);
    dfree(e->type_ab);
    dfree(e->spos);
    dfree(e->sb);
    dfree(e->sidx);
    dfree(e->scell);
    dfree(e->cell_of);
    dfree(e->slot);
    dfree(e->tmp);
    dfree(e->count);
    dfree(e->cstart);
    dfree(e->tile_start);
    dfree(e->tile_range);
    dfree(e->ctx);
    dfree(e->dsched);
    dfree(e->part_force);
    dfree(e->pbuf);
    dfree(e->units);
    dfree(e->scan_sync);
    dfree(e->bucket_p);
    dfree(e->bucket_q);
    dfree(e->ovf_p);
    dfree(e->ovf_q);
    dfree(e->ovf_n);
    dfree(e->rb_sync);
    dfree(e->tcnt);
    dfree(e->part_bbox);
    dfree(e->part_energy);
    dfree(e->force_out);
    dfree(e->boff);
    dfree(e->bent);
    dfree(e->bval);
    dfree(e->bend_eps);
    dfree(e->toff);
    dfree(e->tent);
    dfree(e->noise);
    dfree(e->dom_regions);
    dfree(e->islot);
    dfree(e->bslot);
    dfree(e->swslot);
    dfree(e->brev);
    dfree(e->swt);
    dfree(e->dom_send);
    dfree(e->dom_recv);
    dfree(e->dom_red);
    dfree(e->dom_glob);
    dfree(e->dom_flags);
    if (e->nccl) rccl_comm_destroy(e->nccl);
    dfree(e->dom_shared_idx);
    dfree(e->dom_shared_flag);
    dfree(e->dpos[0]);
    dfree(e->dpos[1]);
    dfree(e->dkmu);
    dfree(e->dforce_out);
    dfree(e->dpart);
    dfree(e->dred);
    dfree(e->dbval);
    dfree(e->dbend_eps);
    dfree(e->dtent);
    dfree(e->dtype_ab);
    dfree(e->dpsort[0]);
    dfree(e->dpsort[1]);
    dfree(e->dskmu);
    dfree(e->dnoise);
    dfree(e->s_pts64);
    dfree(e->c_keys);
    dfree(e->c_counts);
    dfree(e->c_flags);
    dfree(e->c_ck);
    dfree(e->c_cv);
    dfree(e->c_ck2);
    dfree(e->c_cv2);
    dfree(e->c_rows);
    if (e->c_temp) (void)hipFree(e->c_temp);
    dfree(e->q_out);
    if (e->q_host) (void)hipHostFree(e->q_host);
    e->q_host = nullptr;
    dfree(e->s_pts);
    dfree(e->s_spos);
    dfree(e->s_sb);
    dfree(e->s_sidx);
    dfree(e->s_scell);
    dfree(e->s_cell_of);
    dfree(e->s_slot);
    dfree(e->s_tmp);
    dfree(e->s_count);
    dfree(e->s_cstart);
    dfree(e->s_tile);
    dfree(e->s_tile_range);
    dfree(e->s_counts);
    dfree(e->s_offsets);
    dfree(e->s_total);
    dfree(e->s_ctx);
    dfree(e->s_scan_sync);
    dfree(e->s_keys);
    dfree(e->s_keys2);
    if (e->s_sort_temp) (void)hipFree(e->s_sort_temp);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return GCS_OK;
}

int gcs_engine_particle_count(const gcs_engine* e, int64_t* count)
{
    if (!e || !count) return fail(GCS_EINVAL, "null argument");
    *count = e->n;
    return GCS_OK;
}

int gcs_engine_precision(const gcs_engine* e, int32_t* bits)
{
    if (!e || !bits) return fail(GCS_EINVAL, "null argument");
    *bits = e->prec;
    return GCS_OK;
}

int gcs_add_neighbor_softcore(gcs_engine* e, const gcs_softcore_params* p, int32_t* handle)
{
    if (!e || !p) return fail(GCS_EINVAL, "null argument");
    if (!(p->a_diameter > 0) || !(p->neighbor_distance > 0) || (p->mix && !(p->b_diameter > 0)))
        return fail(GCS_EINVAL, "soft-core diameters and neighbor distance must be positive");
    FieldRec* f = new_field(e, F_SOFTCORE);
    f->sc = *p;
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_neighbor_softwell(gcs_engine* e, const gcs_softwell_params* p, const int64_t* targets, int64_t n_targets,
                              int32_t* handle)
{
    if (!e || !p || (n_targets > 0 && !targets)) return fail(GCS_EINVAL, "null argument");
    if (p->exponent != 6) return fail(GCS_EINVAL, "softwell exponent must be 6");
    if (!(p->decay_distance > 0)) return fail(GCS_EINVAL, "softwell decay distance must be positive");
    for (int64_t k = 0; k < n_targets; ++k)
        if (!valid_index(e, targets[k])) return fail(GCS_EINVAL, "softwell target out of range");
    FieldRec* f = new_field(e, F_SOFTWELL);
    f->sw = *p;
    f->idx.assign(targets, targets + n_targets);
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_bonded_pairwise(gcs_engine* e, const gcs_bond_params* p, const int64_t* ranges, int64_t n_ranges,
                            int32_t stride, const int64_t* pairs, int64_t n_pairs, int32_t* handle)
{
    if (!e || !p) return fail(GCS_EINVAL, "null argument");
    if ((n_ranges > 0 && !ranges) || (n_pairs > 0 && !pairs)) return fail(GCS_EINVAL, "null topology array");
    if (n_ranges > 0 && stride < 1) return fail(GCS_EINVAL, "range stride must be >= 1");
    if (p->potential != GCS_POT_SEMISPRING && p->potential != GCS_POT_HARMONIC && p->potential != GCS_POT_SPRING)
        return fail(GCS_EINVAL, "bond potential must be semispring, harmonic or spring");
    std::vector<int64_t> idx;
    for (int64_t r = 0; r < n_ranges; ++r) {
        const int64_t b = ranges[2 * r], en = ranges[2 * r + 1];
        if (b < 0 || en > e->n || b > en) return fail(GCS_EINVAL, "bonded range out of bounds");
        for (int64_t k = b; k + stride < en; ++k) {
            idx.push_back(k);
            idx.push_back(k + stride);
        }
    }
    for (int64_t q = 0; q < n_pairs; ++q) {
        if (!valid_index(e, pairs[2 * q]) || !valid_index(e, pairs[2 * q + 1]))
            return fail(GCS_EINVAL, "bonded pair out of range");
        if (pairs[2 * q] == pairs[2 * q + 1]) return fail(GCS_EINVAL, "bonded pair joins a particle to itself");
        idx.push_back(pairs[2 * q]);
        idx.push_back(pairs[2 * q + 1]);
    }
    FieldRec* f = new_field(e, F_BONDED);
    f->bond = *p;
    f->idx = std::move(idx);
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_bonded_triplewise(gcs_engine* e, double bending_energy, const int64_t* ranges, int64_t n_ranges,
                              int32_t* handle)
{
    if (!e || (n_ranges > 0 && !ranges)) return fail(GCS_EINVAL, "null argument");
    std::vector<int64_t> idx;
    for (int64_t r = 0; r < n_ranges; ++r) {
        const int64_t b = ranges[2 * r], en = ranges[2 * r + 1];
        if (b < 0 || en > e->n || b > en) return fail(GCS_EINVAL, "bending range out of bounds");
        for (int64_t k = b; k + 2 < en; ++k) idx.push_back(k);
    }
    FieldRec* f = new_field(e, F_BENDING);
    f->energy = bending_energy;
    f->idx = std::move(idx);
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_ellipsoid_inward(gcs_engine* e, const gcs_wall_params* p, int32_t* handle)
{
    if (!e || !p) return fail(GCS_EINVAL, "null argument");
    if (!(p->a_diameter > 0) || (p->mix && !(p->b_diameter > 0))) return fail(GCS_EINVAL, "wall diameters must be positive");
    FieldRec* f = new_field(e, F_WALL_IN);
    f->wall = *p;
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_ellipsoid_outward(gcs_engine* e, double spring, const double center[3], int32_t* handle)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    FieldRec* f = new_field(e, F_WALL_OUT);
    f->spring = spring;
    for (int k = 0; k < 3; ++k) f->center[k] = center ? center[k] : 0.0;
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_point_source(gcs_engine* e, const gcs_point_source_params* p, int32_t* handle)
{
    if (!e || !p) return fail(GCS_EINVAL, "null argument");
    if (p->potential < GCS_POT_SEMISPRING || p->potential > GCS_POT_FORCE_FLUX)
        return fail(GCS_EINVAL, "unknown point-source potential");
    FieldRec* f = new_field(e, F_POINT);
    f->point = *p;
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_add_kinetochore_fiber(gcs_engine* e, const double pole[3], const gcs_kinetochore_spec* specs, int64_t n_specs,
                              int32_t* handle)
{
    if (!e || !pole || (n_specs > 0 && !specs)) return fail(GCS_EINVAL, "null argument");
    for (int64_t q = 0; q < n_specs; ++q) {
        if (!valid_index(e, specs[q].particle_index)) return fail(GCS_EINVAL, "kinetochore particle out of range");
        if (!(specs[q].mobility > 0)) return fail(GCS_EINVAL, "kinetochore mobility must be positive");
    }
    FieldRec* f = new_field(e, F_KFIBER);
    for (int k = 0; k < 3; ++k) f->pole[k] = pole[k];
    f->specs.assign(specs, specs + n_specs);
    if (handle) *handle = f->handle;
    return GCS_OK;
}

int gcs_remove_forcefield(gcs_engine* e, int32_t handle)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    for (size_t k = 0; k < e->fields.size(); ++k)
        if (e->fields[k].handle == handle) {
            e->fields.erase(e->fields.begin() + (long)k);
            e->dirty = true;
            return GCS_OK;
        }
    return fail(GCS_EINVAL, "no force field with that handle");
}

int gcs_engine_set_positions(gcs_engine* e, const double* xyz, int64_t n)
{
    if (e) e->dom_cont = false;  // a decomposed run re-primes after any outside change
    if (!e || !xyz) return fail(GCS_EINVAL, "null argument");
    if (int rc = flush_contacts(e)) return rc;
    e->chain_valid = e->dense_chain = false;
    if (n != e->n) return fail(GCS_EINVAL, "position count does not match the particle count");
    HIPCHK(hipSetDevice(e->device));
    if (e->prec == 64) {
        std::vector<double4> h(n);
        for (int64_t i = 0; i < n; ++i) h[i] = make_double4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], 0.0);
        HIPCHK(hipMemcpyAsync(e->dpos[e->parity], h.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        return GCS_OK;
    }
    std::vector<float4> h(n);
    for (int64_t i = 0; i < n; ++i)
        h[i] = make_float4((float)xyz[3 * i], (float)xyz[3 * i + 1], (float)xyz[3 * i + 2], 0.f);
    HIPCHK(hipMemcpyAsync(e->pos[e->parity], h.data(), n * sizeof(float4), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

// A cell scan whose look-back gave up waiting (kernels.hip lookback_sum, counted in DevCtx::scan_stall) leaves wrong
// cell lists behind: the synchronising reads (positions, samples, context) enqueue the count's copy before their
// synchronisation and fail once it is non-zero, so a run that went through such a scan is never read as valid
namespace {
void enqueue_stall_read(gcs_engine* e, int* dst)
{
    (void)hipMemcpyAsync(dst, (const char*)e->ctx + offsetof(DevCtx, scan_stall), sizeof(int), hipMemcpyDeviceToHost,
                         e->stream);
}
int stall_failure()
{
    return fail(GCS_ESTATE, "a multi-block cell scan's look-back stalled (DevCtx::scan_stall): the cell lists, and the "
                            "run that used them, are void");
}
}  // namespace

int gcs_engine_get_positions(gcs_engine* e, double* xyz, int64_t n)
{
    if (!e || !xyz) return fail(GCS_EINVAL, "null argument");
    if (n != e->n) return fail(GCS_EINVAL, "position count does not match the particle count");
    HIPCHK(hipSetDevice(e->device));
    int stalls = 0;
    enqueue_stall_read(e, &stalls);
    if (e->prec == 64) {
        std::vector<double4> h(n);
        HIPCHK(hipMemcpyAsync(h.data(), e->dpos[e->parity], n * sizeof(double4), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        if (stalls) return stall_failure();
        for (int64_t i = 0; i < n; ++i) {
            xyz[3 * i] = h[i].x;
            xyz[3 * i + 1] = h[i].y;
            xyz[3 * i + 2] = h[i].z;
        }
        return GCS_OK;
    }
    std::vector<float4> h(n);
    HIPCHK(hipMemcpyAsync(h.data(), e->pos[e->parity], n * sizeof(float4), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (stalls) return stall_failure();
    for (int64_t i = 0; i < n; ++i) {
        xyz[3 * i] = h[i].x;
        xyz[3 * i + 1] = h[i].y;
        xyz[3 * i + 2] = h[i].z;
    }
    return GCS_OK;
}

int gcs_engine_get_context(gcs_engine* e, gcs_context* c)
{
    if (!e || !c) return fail(GCS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    DevCtx d;
    HIPCHK(hipMemcpyAsync(&d, e->ctx, sizeof(d), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (d.scan_stall) return stall_failure();
    c->step = d.step;
    c->time = d.time;
    c->core_scale = d.cs;
    c->bond_scale = d.bs;
    for (int k = 0; k < 3; ++k) {
        c->wall_semiaxes[k] = d.wall[k];
        c->inward_reaction[k] = d.react_in[k];
        c->outward_reaction[k] = d.react_out[k];
    }
    c->last_timestep = d.dt_used;
    return GCS_OK;
}

int gcs_engine_set_context(gcs_engine* e, const gcs_context* c)
{
    if (e) e->dom_cont = false;  // a decomposed run re-primes after any outside change
    if (!e || !c) return fail(GCS_EINVAL, "null argument");
    if (int rc = flush_contacts(e)) return rc;
    e->chain_valid = e->dense_chain = false;
    HIPCHK(hipSetDevice(e->device));
    DevCtx d;
    HIPCHK(hipMemcpyAsync(&d, e->ctx, sizeof(d), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    d.step = c->step;
    d.time = c->time;
    d.cs = c->core_scale;
    d.bs = c->bond_scale;
    for (int k = 0; k < 3; ++k) {
        d.wall[k] = c->wall_semiaxes[k];
        d.react_in[k] = c->inward_reaction[k];
        d.react_out[k] = c->outward_reaction[k];
    }
    d.dt_used = c->last_timestep;
    HIPCHK(hipMemcpyAsync(e->ctx, &d, sizeof(d), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_set_schedule(gcs_engine* e, const gcs_schedule* s)
{
    if (e) e->dom_cont = false;  // a decomposed run re-primes after any outside change
    if (!e || !s) return fail(GCS_EINVAL, "null argument");
    e->chain_valid = e->dense_chain = false;
    if ((s->update_scales && (!(s->core_scale_tau > 0) || !(s->bond_scale_tau > 0))))
        return fail(GCS_EINVAL, "scale time constants must be positive");
    HIPCHK(hipSetDevice(e->device));
    e->sched = *s;
    int rc = upload_sched(e);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_apply_schedule(gcs_engine* e, int64_t step)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    e->chain_valid = e->dense_chain = false;
    int rc = prepare(e);
    if (rc) return rc;
    long long st = step;
    if ((rc = set_ctx_field(e, offsetof(DevCtx, step), &st, sizeof(st)))) return rc;
    launch_prime(e->stream, e->ctx, e->fa, 0.f, e->ncell_max, e->dsched);
    launch_tail(e->stream, e->ctx, e->fa, 0, 0, 0, 1, e->ncell_max, e->dsched);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_set_noise(gcs_engine* e, const double* normals, int64_t steps)
{
    if (!e || (steps > 0 && !normals)) return fail(GCS_EINVAL, "null argument");
    if (steps < 0) return fail(GCS_EINVAL, "negative step count");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    dfree(e->noise);
    dfree(e->dnoise);
    const size_t cnt = (size_t)steps * (size_t)e->n * 3;
    int rc;
    std::vector<float> h(e->prec == 64 ? 0 : cnt);
    if (e->prec == 64) {  // the normals as given
        if ((rc = dalloc(&e->dnoise, cnt))) return rc;
        HIPCHK(hipMemcpyAsync(e->dnoise, normals, cnt * sizeof(double), hipMemcpyHostToDevice, e->stream));
    } else {
        for (size_t k = 0; k < cnt; ++k) h[k] = (float)normals[k];
        if ((rc = dalloc(&e->noise, cnt))) return rc;
        HIPCHK(hipMemcpyAsync(e->noise, h.data(), cnt * sizeof(float), hipMemcpyHostToDevice, e->stream));
    }
    long long zero = 0;
    if ((rc = set_ctx_field(e, offsetof(DevCtx, noise_cursor), &zero, sizeof(zero)))) return rc;
    HIPCHK(hipStreamSynchronize(e->stream));
    e->noise_steps = steps;
    e->noise_cursor = 0;
    drop_graph(e);
    return GCS_OK;
}

namespace {
// the persistent small-system step (kernels.hip k_pstep): fixed-timestep runs of <= kPMax particles, undecomposed,
// unless a step shape was asked for (GCS_OPT_FUSED_STEP) or the option is off
bool small_path(const gcs_engine* e, bool spacestep)
{
    return e->small_opt != 0 && !e->fused_explicit && !spacestep && !e->dom && e->n >= 1 && e->n <= kPMax;
}
constexpr int kPDebugWords = 1024 + 64 * 128;  // GCS_DEBUG_PSTEP: kernels.hip k_pstep's stamps
constexpr int kPChunk = 2048;  // steps per cooperative launch (a launch then lasts ~10 ms)

int run_small(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps)
{
    int rc;
    if ((rc = flush_contacts(e))) return rc;
    if ((rc = begin_run(e, cfg, first_step))) return rc;
    if (!e->psync && (rc = dalloc(&e->psync, kPSyncWords))) return rc;
    if (!e->pstall) {
        if ((rc = dalloc(&e->pstall, 1)) || (rc = dalloc(&e->pkeep, 1))) return rc;
        HIPCHK(hipMemsetAsync(e->pstall, 0, sizeof(int), e->stream));
    }
    ForceArgs a = e->fa;
    a.psync = e->psync;
    a.pstall = e->pstall;
    a.pstep_skip = -1;
    // GCS_DEBUG_PSTEP_SKIP=<workgroup>:<step> (tests): that workgroup does not publish its hand-off of that step of
    // the run's first launch, so every workgroup stalls -- the run must fail, with the context and positions as before
    if (const char* sk = std::getenv("GCS_DEBUG_PSTEP_SKIP")) {
        int wg = -1, st = -1;
        if (std::sscanf(sk, "%d:%d", &wg, &st) == 2 && wg >= 0 && st >= 0 && st < 65536) a.pstep_skip = (wg << 16) | st;
    }
    // GCS_DEBUG_PSTEP=<file>: workgroup 0's phase stamps of the first 64 steps of the call's first launch
    const char* dbg_path = std::getenv("GCS_DEBUG_PSTEP");
    unsigned long long* dbg = nullptr;
    if (dbg_path) {
        HIPCHK(hipMalloc(&dbg, kPDebugWords * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(dbg, 0, kPDebugWords * sizeof(unsigned long long), e->stream));
        a.dbg_times = dbg;
    }
    // GCS_DEBUG_PSTEP_OFF=<mask>: timing probes only (wrong physics): drop bonds 1, bending 2, tethers 4, point
    // sources 8, walls 16, droplet 32 from the particle-local terms
    if (const char* off = std::getenv("GCS_DEBUG_PSTEP_OFF")) {
        const int m = std::atoi(off);
        if (m & 1) a.has_bonds = 0;
        if (m & 2) a.has_bend = 0;
        if (m & 4) a.has_tether = 0;
        if (m & 8) a.n_point = 0;
        if (m & 16) a.has_wall_in = a.has_wall_out = 0;
        if (m & 32) a.sw_n = 0;
    }
    for (int64_t done = 0; done < steps;) {
        const int len = (int)std::min<int64_t>(kPChunk, steps - done);
        HIPCHK(hipMemsetAsync(e->psync, 0, kPSyncWords * sizeof(unsigned), e->stream));
        launch_pstep_guard(e->stream, e->ctx, e->pkeep, e->pstall, 0);
        if (launch_pstep(e->stream, e->ctx, a, len, e->sched_flags != 0 ? 1 : 0))
            return fail(GCS_EHIP, "the persistent small-system step could not be launched cooperatively");
        e->rstats.eager_steps += len;
        done += len;
        a.dbg_times = nullptr;
        a.pstep_skip = -1;
    }
    // a stalled hand-off fails the run: the context goes back to the failing launch's start (its positions are
    // intact: a launch writes only the other parity), the stall word is cleared for the next run
    launch_pstep_guard(e->stream, e->ctx, e->pkeep, e->pstall, 1);
    int stalled = 0;
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&stalled, e->pstall, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (stalled) {
        HIPCHK(hipMemsetAsync(e->pstall, 0, sizeof(int), e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->chain_valid = false;
        if (dbg) (void)hipFree(dbg);
        return fail(GCS_ESTATE, "the persistent small-system step stalled: a workgroup's hand-off did not arrive "
                                "(the run is void; the context and positions are those before the failing launch)");
    }
    if (dbg) {
        std::vector<unsigned long long> h(kPDebugWords);
        HIPCHK(hipMemcpyAsync(h.data(), dbg, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipFree(dbg));
        if (FILE* f = std::fopen(dbg_path, "wb")) {
            std::fwrite(h.data(), sizeof(h[0]), h.size(), f);
            std::fclose(f);
        }
    }
    end_run(e, cfg, first_step, steps);
    e->chain_valid = false;  // no cell or neighbour lists of these positions
    if (steps & 1) e->parity ^= 1;
    if (cfg->noise == GCS_NOISE_INJECTED) e->noise_cursor += steps;
    return GCS_OK;
}
}  // namespace

int gcs_engine_run(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps)
{
    if (e) e->dom_cont = false;  // a decomposed run re-primes after any outside change
    if (!e || !cfg) return fail(GCS_EINVAL, "null argument");
    if (steps < 0) return fail(GCS_EINVAL, "negative step count");
    if (!(cfg->timestep > 0)) return fail(GCS_EINVAL, "timestep must be positive");
    if (cfg->noise < GCS_NOISE_PHILOX || cfg->noise > GCS_NOISE_NONE) return fail(GCS_EINVAL, "unknown noise mode");
    if (cfg->noise == GCS_NOISE_INJECTED && e->noise_cursor + steps > e->noise_steps)
        return fail(GCS_ESTATE, "not enough injected noise for the requested steps");
    if (steps == 0) return prepare(e);
    const bool spacestep = cfg->spacestep > 0;
    int rc = choose_shape(e, cfg, first_step);
    if (rc) return rc;
    // (the fp64 engine's fixed-timestep step is the list step when the system admits it -- a neighbor soft-core field,
    // <= 256 (a, b) pair classes, < 2^24 particles -- and otherwise its cell-list step: enqueue_step, prec 64)
    if (small_path(e, spacestep)) return run_small(e, cfg, first_step, steps);
    if (!list_path(e, spacestep) || spacestep)  // (contact updates are fused into fixed-timestep list steps only)
        if ((rc = flush_contacts(e))) return rc;
    // the list skin of the run's first step (skin_level); a change from the last run's re-primes and rebuilds
    const int lv0 = list_path(e, spacestep) ? skin_level(e, first_step) : e->skin_level_pm;
    const bool lv_changed = lv0 != e->skin_level_pm;
    e->skin_level_pm = lv0;
    if ((rc = begin_run(e, cfg, first_step))) return rc;
    if (lv_changed && list_path(e, spacestep)) {
        launch_prime(e->stream, e->ctx, list_args(e), 0.f, e->ncell_max, e->dsched);
        e->l_need_build = true;
    }

    const int G = e->graph_steps;
    GraphKey key = run_key(e, cfg, spacestep);
    int64_t done = 0;
    if (list_path(e, spacestep)) {
        // rebuilds at the steps k with (first_step + k) % M == 0 and at a run start without continuity, so a run
        // split into chunks rebuilds where the whole run does (bitwise identical).  Every stretch of up to G steps
        // is replayed from a graph captured once per (first step mod M, starting parity, length): a run of any
        // length, from any step, replays graphs (only the forced rebuild of a run start and a pending contact
        // update run eagerly)
        // the host knows every step's position-buffer parity (the kernels' slot loads then need no context read);
        // a captured graph bakes its steps' parities in
        auto par = [&](int64_t k) { return e->parity ^ (int)(k & 1); };
        while (done < steps) {
            const int64_t st = first_step + done;
            const int lv = skin_level(e, st);
            if (lv != e->skin_level_pm) {
                // the skin changes at this step (the core scale grew): the grid at the new list radius, a rebuild,
                // the period for the new skin, graphs under the new key
                e->skin_level_pm = lv;
                e->list_every = auto_list_every(e, cfg->temperature, cfg->timestep);
                launch_prime(e->stream, e->ctx, list_args(e), 0.f, e->ncell_max, e->dsched);
                e->l_need_build = true;
                key = run_key(e, cfg, spacestep);
            }
            const int M = e->list_every;
            const int phase = (int)((((st + e->list_phase) % M) + M) % M);
            // the contact update the host asked for after the last step: counted by this stretch's first step, its
            // distance set in the context (so the stretch's graph does not depend on it)
            const bool ct = e->c_pending > 0;
            if (ct) {
                const float d = (float)e->c_pending;
                // the products the predicates form: fp32 (k_contact_insert) and fp64
                launch_set_contact(e->stream, e->ctx, d * d, e->c_pending * e->c_pending);
                e->c_pending = 0;
                e->rstats.fused_contact_steps++;
            }
            const gcs_bd_config* rx = spacestep ? cfg : nullptr;  // the relaxation step
            if (e->l_need_build || G == 0) {
                // a run start's rebuild, or no graphs
                enqueue_list_step(e, e->l_need_build || phase == 0, list_flags(e, st) | 16, ct ? 1.0 : 0.0, par(done),
                                  rx);  // (16: a stretch's last step writes the particle-order copy, kLFlagPos)
                e->l_need_build = false;
                ++done;
                e->rstats.eager_steps++;
                continue;
            }
            int len = (int)std::min<int64_t>(G, steps - done);
            for (int k = 1; k < len; ++k)  // a stretch ends where the skin changes
                if (skin_level(e, st + k) != lv) {
                    len = k;
                    break;
                }
            const int p0 = par(done);
            hipGraphExec_t x = nullptr;
            // cache slot: rebuild phase, and whether the first step counts contacts
            rc = cached_graph(e, key, phase | (ct ? 1 << 20 : 0), p0, len, [&]() {
                for (int k = 0; k < len; ++k)
                    enqueue_list_step(e, (phase + k) % M == 0, list_flags(e, st + k) | (k == len - 1 ? 16 : 0),
                                      (ct && k == 0) ? 1.0 : 0.0,
                                      p0 ^ (k & 1), rx);
            }, &x);
            if (rc || (rc = launch_graph(e, x))) return rc;
            e->rstats.graph_steps += len;
            done += len;
        }
    }
    // other step shapes: every step is the same launch sequence (the context carries the parity)
    while (G > 0 && done < steps) {
        const int len = (int)std::min<int64_t>(G, steps - done);
        hipGraphExec_t x = nullptr;
        rc = cached_graph(e, key, 0, 0, len, [&]() {
            for (int k = 0; k < len; ++k) enqueue_step(e, spacestep, cfg->spacestep, cfg->timestep);
        }, &x);
        if (rc || (rc = launch_graph(e, x))) return rc;
        e->rstats.graph_steps += len;
        done += len;
    }
    for (; done < steps; ++done) {
        enqueue_step(e, spacestep, cfg->spacestep, cfg->timestep);
        e->rstats.eager_steps++;
    }
    HIPCHK(hipGetLastError());
    end_run(e, cfg, first_step, steps);
    if (spacestep) e->chain_dt = -1.0;  // ctx->dt_used holds an adapted timestep: the next run rewrites it
    if (steps & 1) e->parity ^= 1;
    if (cfg->noise == GCS_NOISE_INJECTED) e->noise_cursor += steps;
    return GCS_OK;
}

int gcs_engine_synchronize(gcs_engine* e)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_compute_forces(gcs_engine* e, double* forces, int64_t n)
{
    if (!e || !forces) return fail(GCS_EINVAL, "null argument");
    if (n != e->n) return fail(GCS_EINVAL, "force array size does not match the particle count");
    e->chain_valid = e->dense_chain = false;
    int rc = prepare(e);
    if (rc) return rc;
    launch_prime(e->stream, e->ctx, e->fa, 0.f, e->ncell_max, e->dsched);
    enqueue_cells(e);
    if (e->prec == 64) {
        launch_eval64(e->stream, kModeForce, e->ctx, e->fa);
        launch_red64(e->stream, e->ctx, e->fa, -1.0, 0.0, nullptr);  // reactions, drift, neighbours (dt untouched)
        HIPCHK(hipGetLastError());
        std::vector<double4> h(n);
        HIPCHK(hipMemcpyAsync(h.data(), e->dforce_out, n * sizeof(double4), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        for (int64_t i = 0; i < n; ++i) {
            forces[3 * i] = h[i].x;
            forces[3 * i + 1] = h[i].y;
            forces[3 * i + 2] = h[i].z;
        }
        return GCS_OK;
    }
    launch_force(e->stream, kModeForce, e->waves, e->ctx, e->fa, false);
    launch_tail(e->stream, e->ctx, e->fa, force_grid(e->n), 0, 0, 0, e->ncell_max, e->dsched);
    HIPCHK(hipGetLastError());
    std::vector<float4> h(n);
    HIPCHK(hipMemcpyAsync(h.data(), e->force_out, n * sizeof(float4), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int64_t i = 0; i < n; ++i) {
        forces[3 * i] = h[i].x;
        forces[3 * i + 1] = h[i].y;
        forces[3 * i + 2] = h[i].z;
    }
    return GCS_OK;
}

int gcs_engine_compute_energy(gcs_engine* e, double* total, double* per_kind)
{
    if (!e || !total) return fail(GCS_EINVAL, "null argument");
    e->chain_valid = e->dense_chain = false;
    int rc = prepare(e);
    if (rc) return rc;
    launch_prime(e->stream, e->ctx, e->fa, 0.f, e->ncell_max, e->dsched);
    enqueue_cells(e);
    if (e->prec == 64)
        launch_eval64(e->stream, kModeEnergy, e->ctx, e->fa);
    else
        launch_force(e->stream, kModeEnergy, e->waves, e->ctx, e->fa, false);
    HIPCHK(hipGetLastError());
    const int fb = e->prec == 64 ? eval64_blocks(e->n) : force_grid(e->n);
    std::vector<double> h((size_t)fb * kEnergyKinds);
    HIPCHK(hipMemcpyAsync(h.data(), e->part_energy, h.size() * sizeof(double), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    double pk[kEnergyKinds] = {0};
    for (int b = 0; b < fb; ++b)
        for (int k = 0; k < kEnergyKinds; ++k) pk[k] += h[(size_t)b * kEnergyKinds + k];
    double t = 0;
    for (int k = 0; k < kEnergyKinds; ++k) t += pk[k];
    *total = t;
    if (per_kind)
        for (int k = 0; k < kEnergyKinds; ++k) per_kind[k] = pk[k];
    return GCS_OK;
}

int gcs_engine_search_neighbors(gcs_engine* e, const double* points, int64_t n, double distance, uint32_t* pairs,
                                int64_t capacity, int64_t* count)
{
    if (!e || !count || (capacity > 0 && !pairs)) return fail(GCS_EINVAL, "null argument");
    if (!(distance > 0)) return fail(GCS_EINVAL, "search distance must be positive");
    e->chain_valid = e->dense_chain = false;
    if (!points && n != e->n) return fail(GCS_EINVAL, "point count does not match the particle count");
    if (n < 0 || n > (int64_t)1 << 30) return fail(GCS_EINVAL, "bad point count");
    *count = 0;
    if (n < 2) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    int rc;
    if ((rc = ensure_search(e, n))) return rc;
    const int ni = (int)n;
    const float4* src = e->s_pts;
    const double4* src64 = nullptr;  // fp64 engine: the points in fp64, the fp64 predicate
    if (points) {
        if (e->prec == 64) {
            dfree(e->s_pts64);
            if ((rc = dalloc(&e->s_pts64, n))) return rc;
            std::vector<double4> h(n);
            for (int64_t i = 0; i < n; ++i) h[i] = make_double4(points[3 * i], points[3 * i + 1], points[3 * i + 2], 0.0);
            HIPCHK(hipMemcpyAsync(e->s_pts64, h.data(), n * sizeof(double4), hipMemcpyHostToDevice, e->stream));
            src64 = e->s_pts64;
        } else {
            std::vector<float4> h(n);
            for (int64_t i = 0; i < n; ++i)
                h[i] = make_float4((float)points[3 * i], (float)points[3 * i + 1], (float)points[3 * i + 2], 0.f);
            HIPCHK(hipMemcpyAsync(e->s_pts, h.data(), n * sizeof(float4), hipMemcpyHostToDevice, e->stream));
        }
        HIPCHK(hipStreamSynchronize(e->stream));
    } else {
        src = e->pos[e->parity];
        if (e->prec == 64) src64 = e->dpos[e->parity];
    }
    if ((rc = enqueue_search_cells(e, src, src64, ni, distance))) return rc;
    launch_search_count(e->stream, e->s_ctx, ni, e->s_spos, e->s_sidx, e->s_scell, e->s_cstart, e->s_counts, src64,
                        distance);
    launch_exclusive_scan_small(e->stream, e->s_counts, e->s_offsets, ni, e->s_total);
    HIPCHK(hipGetLastError());
    int total = 0;
    HIPCHK(hipMemcpyAsync(&total, e->s_total, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    *count = total;
    if (total > capacity) return fail(GCS_ECAPACITY, "pair buffer too small; *count holds the required size");
    if (total == 0) return GCS_OK;
    if (total > e->s_key_cap) {
        dfree(e->s_keys);
        dfree(e->s_keys2);
        if (e->s_sort_temp) (void)hipFree(e->s_sort_temp);
        e->s_sort_temp = nullptr;
        e->s_key_cap = 0;
        if ((rc = dalloc(&e->s_keys, total)) || (rc = dalloc(&e->s_keys2, total))) return rc;
        e->s_sort_bytes = sort_u64_temp_bytes(total);
        HIPCHK(hipMalloc(&e->s_sort_temp, std::max<size_t>(e->s_sort_bytes, 16)));
        e->s_key_cap = total;
    }
    launch_search_emit(e->stream, e->s_ctx, ni, e->s_spos, e->s_sidx, e->s_scell, e->s_cstart, e->s_offsets, e->s_keys,
                       src64, distance);
    size_t bytes = sort_u64_temp_bytes(total);
    if (bytes > e->s_sort_bytes) {
        (void)hipFree(e->s_sort_temp);
        HIPCHK(hipMalloc(&e->s_sort_temp, bytes));
        e->s_sort_bytes = bytes;
    }
    sort_u64_keys(e->stream, e->s_keys, e->s_keys2, total, e->s_sort_temp, e->s_sort_bytes);
    HIPCHK(hipGetLastError());
    std::vector<unsigned long long> h(total);
    HIPCHK(hipMemcpyAsync(h.data(), e->s_keys2, total * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int k = 0; k < total; ++k) {
        pairs[2 * k] = (uint32_t)(h[k] >> 32);
        pairs[2 * k + 1] = (uint32_t)h[k];
    }
    return GCS_OK;
}

int gcs_engine_contacts_update(gcs_engine* e, double distance)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    if (!(distance > 0)) return fail(GCS_EINVAL, "contact distance must be positive");
    if (e->n < 2) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    int rc;
    if (!e->c_keys) {
        int bits = e->c_bits_opt;
        if (bits <= 0) {
            // >= 256 slots per particle, at most 2^28 (3 GB): a C2 window of the reference's cadence (10 samples x
            // 50 updates) holds ~2.9 million distinct pairs, 18 % of C2's 2^24 slots.  Round 6, 300,000 steps of
            // the interphase stage with the contact map (profiles/r06_contact_bits.txt): 2^25 slots 28.97k
            // steps/s, 2^24 29.45k, 2^23 29.30k -- the table's random atomics stay closer to the caches, and each
            // window's read compacts a smaller table (9.0 -> 5.8 ms); at 2^23 the probe chains start to cost
            bits = 12;
            while (bits < 28 && ((int64_t)1 << bits) < 256 * (int64_t)e->n) ++bits;
        }
        const size_t slots = (size_t)1 << bits;
        if ((rc = dalloc(&e->c_keys, slots)) || (rc = dalloc(&e->c_counts, slots)) || (rc = dalloc(&e->c_flags, 2)))
            return rc;
        e->c_bits = bits;
        HIPCHK(hipMemsetAsync(e->c_keys, 0xff, slots * sizeof(unsigned long long), e->stream));
        HIPCHK(hipMemsetAsync(e->c_counts, 0, slots * sizeof(unsigned), e->stream));
        HIPCHK(hipMemsetAsync(e->c_flags, 0, 2 * sizeof(int), e->stream));
    }
    if ((rc = flush_contacts(e))) return rc;
    if (list_path(e, false) && e->chain_valid) {
        // after a list-step run: the next list step counts the pairs from its start positions (= these), inside
        // its pair loop (contact distance < cutoff: every such pair is in the lists or the exact search)
        e->c_pending = distance;
    } else if ((rc = contacts_insert_now(e, distance))) {
        return rc;
    }
    e->c_updates++;
    return GCS_OK;
}

int gcs_engine_contacts_clear(gcs_engine* e)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    // a pending (deferred) update followed by a clear leaves an empty table: dropping it equals counting it first
    e->c_pending = 0;
    e->c_updates = 0;
    if (!e->c_keys) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    const size_t slots = (size_t)1 << e->c_bits;
    HIPCHK(hipMemsetAsync(e->c_keys, 0xff, slots * sizeof(unsigned long long), e->stream));
    HIPCHK(hipMemsetAsync(e->c_counts, 0, slots * sizeof(unsigned), e->stream));
    HIPCHK(hipMemsetAsync(e->c_flags, 0, 2 * sizeof(int), e->stream));
    return GCS_OK;
}

int gcs_engine_contacts_read(gcs_engine* e, uint32_t* ijc, int64_t capacity, int64_t* count)
{
    if (!e || !count || (capacity > 0 && !ijc)) return fail(GCS_EINVAL, "null argument");
    if (int rc = flush_contacts(e)) return rc;
    *count = 0;
    if (!e->c_keys) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    const long long slots = (long long)1 << e->c_bits;
    int rc;
    HIPCHK(hipMemsetAsync(e->c_flags + 1, 0, sizeof(int), e->stream));
    int flags[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(flags, e->c_flags, sizeof(flags), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (flags[0]) return fail(GCS_ECAPACITY, "contact map overflowed its hash table: raise GCS_OPT_CONTACT_BITS");
    // count the occupied slots, then compact into scratch of that size and radix-sort (key, count) by key; the
    // scratch (12 B + 12 B + 12 B per distinct pair) stays allocated for the next read, grown when a window holds more
    // pairs (not sized to the table: at the 2^28-slot cap that would be 3 GB)
    launch_contact_occupied(e->stream, e->c_keys, slots, e->c_flags + 1);
    int total = 0;
    HIPCHK(hipMemcpyAsync(&total, e->c_flags + 1, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    *count = total;
    if (total > capacity) return fail(GCS_ECAPACITY, "contact buffer too small; *count holds the required size");
    if (total == 0) return GCS_OK;
    if (total > e->c_sorted_cap) {
        dfree(e->c_ck);
        dfree(e->c_cv);
        dfree(e->c_ck2);
        dfree(e->c_cv2);
        dfree(e->c_rows);
        e->c_sorted_cap = 0;
        const size_t cap = (size_t)total + (size_t)total / 4;  // headroom for the next windows
        if ((rc = dalloc(&e->c_ck, cap)) || (rc = dalloc(&e->c_cv, cap)) || (rc = dalloc(&e->c_ck2, cap)) ||
            (rc = dalloc(&e->c_cv2, cap)) || (rc = dalloc(&e->c_rows, 3 * cap)))
            return rc;
        e->c_sorted_cap = (int64_t)cap;
    }
    HIPCHK(hipMemsetAsync(e->c_flags + 1, 0, sizeof(int), e->stream));
    launch_contact_compact(e->stream, e->c_keys, e->c_counts, slots, e->c_ck, e->c_cv, e->c_flags + 1);
    const size_t bytes = std::max<size_t>(sort_pairs_u64_u32_temp_bytes(total), 16);
    if (bytes > e->c_temp_bytes) {
        if (e->c_temp) (void)hipFree(e->c_temp);
        e->c_temp = nullptr;
        e->c_temp_bytes = 0;
        HIPCHK(hipMalloc(&e->c_temp, bytes));
        e->c_temp_bytes = bytes;
    }
    // keys are i << 32 | j with i, j < N: the radix passes stop at 32 + bit length of N - 1
    int nbits = 1;
    while (nbits < 32 && ((int64_t)1 << nbits) < e->n) ++nbits;
    sort_pairs_u64_u32(e->stream, e->c_ck, e->c_ck2, e->c_cv, e->c_cv2, total, e->c_temp, e->c_temp_bytes,
                       32 + nbits);
    launch_contact_emit(e->stream, e->c_ck2, e->c_cv2, total, e->c_rows);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ijc, e->c_rows, 3 * (size_t)total * sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_sample_positions(gcs_engine* e, float* xyz, int64_t n, int32_t fraction_bits)
{
    if (!e || !xyz) return fail(GCS_EINVAL, "null argument");
    if (n != e->n) return fail(GCS_EINVAL, "position count does not match the particle count");
    if (fraction_bits < 1 || fraction_bits > 23) return fail(GCS_EINVAL, "fraction_bits must be in [1, 23]");
    HIPCHK(hipSetDevice(e->device));
    int rc;
    if (!e->q_out && (rc = dalloc(&e->q_out, 3 * (size_t)e->n))) return rc;
    if (!e->q_host) HIPCHK(hipHostMalloc(&e->q_host, 3 * (size_t)e->n * sizeof(float), hipHostMallocDefault));
    if (e->prec == 64)
        launch_quantize(e->stream, e->dpos[e->parity], e->q_out, e->n, fraction_bits);
    else
        launch_quantize(e->stream, e->pos[e->parity], e->q_out, e->n, fraction_bits);
    HIPCHK(hipGetLastError());
    int stalls = 0;
    enqueue_stall_read(e, &stalls);
    HIPCHK(hipMemcpyAsync(e->q_host, e->q_out, 3 * (size_t)n * sizeof(float), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (stalls) return stall_failure();
    std::memcpy(xyz, e->q_host, 3 * (size_t)n * sizeof(float));
    return GCS_OK;
}

// ---- spatial domain decomposition (C5) ----

namespace {
float finite_f(double v) { return (float)std::min(std::max(v, -3.0e38), 3.0e38); }
DomBox make_box(const double* lohi)
{
    DomBox b;
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = finite_f(lohi[k]);
        b.hi[k] = finite_f(lohi[3 + k]);
    }
    return b;
}
// a domain's region: its (fp32) box extended by the (fp32) halo.  Every engine derives its own region and its
// peers' with this one formula, so a particle is inside a region bit-identically for the domain that bins by it
// and for the owner that decides whether to send (a 1-ulp disagreement would leave a binned ghost stale)
DomBox region_of(const DomBox& b, float halo)
{
    DomBox r;
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = finite_f((double)b.lo[k] - (double)halo);
        r.hi[k] = finite_f((double)b.hi[k] + (double)halo);
    }
    return r;
}
}  // namespace

int gcs_engine_set_domain(gcs_engine* e, const double* box, double halo, const double* peer_boxes, int32_t npeer,
                          int32_t index, int32_t ndomains)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    if (!(halo > 0)) {  // off
        e->dom = false;
        e->dom_cont = false;
        return GCS_OK;
    }
    if (!box) return fail(GCS_EINVAL, "null argument");
    for (int k = 0; k < 3; ++k)
        if (!(box[k] < box[3 + k])) return fail(GCS_EINVAL, "domain box must have lo < hi on every axis");
    if (npeer < 0 || npeer > kMaxPeers || (npeer > 0 && !peer_boxes)) return fail(GCS_EINVAL, "bad peer list");
    if (ndomains < 1 || ndomains > kMaxDomains || index < 0 || index >= ndomains)
        return fail(GCS_EINVAL, "bad domain index / count");
    HIPCHK(hipSetDevice(e->device));
    int rc;
    if (!e->dom_regions && (rc = dalloc(&e->dom_regions, kMaxPeers))) return rc;
    if (!e->dom_flags && (rc = dalloc(&e->dom_flags, 1))) return rc;
    DomBox h[kMaxPeers] = {};
    for (int p = 0; p < npeer; ++p) h[p] = region_of(make_box(peer_boxes + 6 * p), (float)halo);
    HIPCHK(hipMemcpyAsync(e->dom_regions, h, sizeof(h), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    drop_domain_graph(e);  // the captured chunk holds the box and the peer count by value
    if (e->dom_red && e->dom_ndom != ndomains) {
        // the allreduce buffer holds one slot per domain: set up again (gcs_engine_domain_buffers)
        dfree(e->dom_send);
        dfree(e->dom_recv);
        dfree(e->dom_red);
        dfree(e->dom_glob);
        e->dom_nred = 0;
        e->dom_cap = 0;
    }
    e->dom = true;
    e->dom_box = make_box(box);
    e->dom_halo = (float)halo;
    e->dom_npeer = npeer;
    e->dom_index = index;
    e->dom_ndom = ndomains;
    e->dom_cont = false;
    return GCS_OK;
}

int gcs_engine_set_domain_shared(gcs_engine* e, const int64_t* idx, int32_t count)
{
    if (!e || (count > 0 && !idx)) return fail(GCS_EINVAL, "null argument");
    if (count < 0) return fail(GCS_EINVAL, "negative count");
    HIPCHK(hipSetDevice(e->device));
    std::vector<int> h(count), flag(e->n, 0);
    for (int k = 0; k < count; ++k) {
        if (!valid_index(e, idx[k])) return fail(GCS_EINVAL, "shared particle index out of range");
        h[k] = (int)idx[k];
        flag[h[k]] = k + 1;  // (nonzero: shared; k + 1: its row in the allreduce buffer's shared block)
    }
    drop_domain_graph(e);
    if (e->dom_red && kDomainRed + 3 * count + e->dom_ndom != e->dom_nred) {
        // the allreduce buffer holds the shared positions: its size changes, so the exchange buffers must be
        // set up again (gcs_engine_domain_buffers) before the next decomposed run
        dfree(e->dom_send);
        dfree(e->dom_recv);
        dfree(e->dom_red);
        dfree(e->dom_glob);
        e->dom_nred = 0;
        e->dom_cap = 0;
    }
    dfree(e->dom_shared_idx);
    dfree(e->dom_shared_flag);
    e->dom_nshared = 0;
    int rc;
    if ((rc = dalloc(&e->dom_shared_idx, std::max(count, 1))) || (rc = dalloc(&e->dom_shared_flag, e->n))) return rc;
    if (count > 0)
        HIPCHK(hipMemcpyAsync(e->dom_shared_idx, h.data(), count * sizeof(int), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->dom_shared_flag, flag.data(), e->n * sizeof(int), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->dom_nshared = count;
    return GCS_OK;
}

int gcs_engine_stream(gcs_engine* e, void** stream)
{
    if (!e || !stream) return fail(GCS_EINVAL, "null argument");
    *stream = (void*)e->stream;
    return GCS_OK;
}

namespace {
// the decomposed step's argument block: the list step's (dom_list) or the tile step's, with the domain geometry, the
// reduction layout (dom_red: the caller's buffer) and the flags
bool dom_list_ok(const gcs_engine* e);
// The ghosts a decomposed step BINS: the list step needs a particle's partners within its list radius (cutoff at
// cs = 1 + skin) of the box, plus the displacement since the build, so it bins the ghosts within list radius + one
// more skin (the motion check flags cutoff + largest displacement beyond it); the exchange halo itself is the
// chain bonds' reach (C5: 0.54 against a list radius of 0.21), which only the bonded partners need, and they are
// read by index from the position buffers the unpack refreshes, binned or not.  The tile step bins the whole halo.
float dom_bin_halo(const gcs_engine* e)
{
    if (!dom_list_ok(e)) return e->dom_halo;
    return std::min(e->dom_halo, e->fa.pf.pair_dist + 2.f * list_skin_max(e));
}

ForceArgs domain_args(const gcs_engine* e, double* red = nullptr)
{
    ForceArgs a = e->dom_list ? list_args(e) : e->fa;
    a.dom_on = 1;
    a.dom = e->dom_box;
    a.dom_halo = e->dom_halo;
    a.dom_bin_halo = dom_bin_halo(e);
    a.bucket_p = nullptr;
    a.dom_red = red;
    a.dom_dbase = kDomainRed + 3 * e->dom_nshared;
    a.dom_index = e->dom_index;
    a.dom_ndom = e->dom_ndom;
    a.dom_flags = e->dom_flags;
    a.islot = e->islot;
    return a;
}

DomBox dom_region(const gcs_engine* e) { return region_of(e->dom_box, dom_bin_halo(e)); }

// the decomposed run takes the list step when the engine would (list step selected, lists admitted) and the halo
// holds the list radius: a partner within the cutoff of an owned particle must have been binned at the build
// (cutoff + skin at cs = 1; the tail checks cutoff + largest displacement every step, kDomFlagMotion)
bool dom_list_ok(const gcs_engine* e)
{
    return list_path(e, false) && e->fa.has_pair && e->dom_halo >= e->fa.pf.pair_dist + list_skin_max(e);
}

// the list-step half of a decomposed step before the allreduce: on a rebuild step the cells of this domain's region
// (owned + ghosts) and the lists, then k_lstep<..., DOM> (owned slots; local reduction -> red), then the shared
// particles' new positions into red
void enqueue_dom_list_step(gcs_engine* e, int64_t st, double* red, bool fused_pack = false)
{
    const int lv = skin_level(e, st);
    if (lv != e->skin_level_pm) {
        // the skin changes at this step (skin_level): the grid at the new list radius over this domain's local box
        // (padded by the binning halo, sized for the largest skin), a rebuild, the period for the new skin.  Never
        // inside a capture: gcs_engine_domain_run runs a stretch with a change eagerly
        e->skin_level_pm = lv;
        e->list_every = auto_list_every(e, e->fa.pd.temperature, e->fa.pd.timestep);
        launch_dom_grid(e->stream, e->ctx, domain_args(e, red));
        e->l_need_build = true;
    }
    ForceArgs a = domain_args(e, red);
    if (fused_pack) {  // the engine's bands (header rows zeroed by the last unpack) and reduction buffer
        a.dom_bands = e->dom_send;
        a.dom_bstride = e->dom_cap + 1;
        a.dom_cap = e->dom_cap;
        a.dom_npeer = e->dom_npeer;
        a.dom_regions = e->dom_regions;
        a.dom_shared = e->dom_shared_flag;
    }
    if (e->l_need_build || (st + e->list_phase) % e->list_every == 0) {
        const DomBox reg = dom_region(e);
        enqueue_count(e, &reg, e->islot);
        dbg_sync(e, "dom: k_cell_count");
        enqueue_scan(e, false);
        dbg_sync(e, "dom: cell scan");
        launch_cell_scatter(e->stream, e->n, e->cell_of, e->slot, e->cstart, e->tmp, e->count);
        dbg_sync(e, "dom: k_cell_scatter");
        enqueue_cell_order(e, true, e->islot);
        dbg_sync(e, "dom: k_cell_sort");
        launch_list_build(e->stream, e->ctx, a);
        dbg_sync(e, "dom: k_lbuild");
        e->l_need_build = false;
    }
    e->dom_flags_step = list_flags(e, st) | 8;  // 8: kLFlagDomain
    launch_list_step(e->stream, e->ctx, a, e->dom_flags_step);
    dbg_sync(e, "dom: k_lstep<DOM>");
    if (!fused_pack) launch_domain_shared_out(e->stream, e->ctx, a, e->dom_shared_idx, e->dom_nshared, red);
}

// after the allreduce: the tail from the global sums, the shared particles in, the send bands' headers zeroed
void enqueue_dom_list_finish(gcs_engine* e, const double* glob, void* bands, int npeer)
{
    // (with the engine's reduction buffer: its shared block is zeroed for the next step's fused pack)
    launch_list_domain_tail(e->stream, e->ctx, domain_args(e, e->dom_red), glob, e->dom_flags_step & ~8,
                            e->dom_shared_idx, e->dom_nshared, bands, npeer, e->dom_cap + 1);
    dbg_sync(e, "dom: k_ldom_tail");
}
}  // namespace

// fused: the engine's own bands and reduction buffer take the step's band pack and shared particles from
// k_lstep<..., DOM> itself (gcs_engine_domain_step_host; the pack then only copies); otherwise the separate pack
static int domain_step_impl(gcs_engine* e, const gcs_bd_config* cfg, int64_t step, double* dev_reaction, bool fused)
{
    if (!e || !cfg || !dev_reaction) return fail(GCS_EINVAL, "null argument");
    if (!e->dom) return fail(GCS_ESTATE, "gcs_engine_set_domain first");
    if (cfg->spacestep > 0) return fail(GCS_EINVAL, "decomposed runs use a fixed timestep");
    if (cfg->noise == GCS_NOISE_INJECTED) return fail(GCS_EINVAL, "decomposed runs draw Philox noise");
    if (int rc = flush_contacts(e)) return rc;
    HIPCHK(hipSetDevice(e->device));
    if (!(e->dom_cont && e->dom_next == step)) {
        int rc = prepare(e);
        if (rc) return rc;
        e->dom_list = dom_list_ok(e);
        if (e->prec == 64 && !e->dom_list)
            return fail(GCS_ESTATE, "an fp64 decomposed run takes the list step: it needs a neighbor soft-core field "
                                    "and a halo of at least the list radius (cutoff x (1 + skin))");
        if (e->dom_list && !e->islot && (rc = dalloc(&e->islot, e->n))) return rc;
        drop_domain_graph(e);  // captured for the other step shape, or another rebuild phase
        if ((rc = begin_run(e, cfg, step))) return rc;
        // both position buffers hold the start state: a domain writes only what it owns or receives, so the
        // buffer the first step writes must already carry every other particle's copy
        if (e->prec == 64)
            HIPCHK(hipMemcpyAsync(e->dpos[e->parity ^ 1], e->dpos[e->parity], (size_t)e->n * sizeof(double4),
                                  hipMemcpyDeviceToDevice, e->stream));
        else
            HIPCHK(hipMemcpyAsync(e->pos[e->parity ^ 1], e->pos[e->parity], (size_t)e->n * sizeof(float4),
                                  hipMemcpyDeviceToDevice, e->stream));
        // the fused pack's starting state: empty send bands, an empty shared block in the reduction buffer
        if (e->dom_send) launch_band_headers_zero(e->stream, e->dom_send, e->dom_npeer, e->dom_cap + 1, e->prec);
        if (e->dom_red) HIPCHK(hipMemsetAsync(e->dom_red, 0, (size_t)e->dom_nred * sizeof(double), e->stream));
        dbg_sync(e, "dom: run start (prime, copies)");
    }
    e->chain_valid = e->dense_chain = false;
    e->dom_next = step + 1;
    e->dom_fused = fused && e->dom_list && e->dom_send && dev_reaction == e->dom_red;
    if (e->dom_list) {
        enqueue_dom_list_step(e, step, dev_reaction, e->dom_fused);
        HIPCHK(hipGetLastError());
        return GCS_OK;
    }
    const ForceArgs a = domain_args(e);
    const DomBox reg = dom_region(e);
    enqueue_count(e, &reg);
    enqueue_scan(e, false);
    enqueue_sort(e);
    launch_force(e->stream, kModeStep, e->waves, e->ctx, a, false);
    launch_tail_reduce(e->stream, e->ctx, a, step_grid(e), dev_reaction);
    launch_domain_shared_out(e->stream, e->ctx, a, e->dom_shared_idx, e->dom_nshared, dev_reaction);
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

int gcs_engine_domain_step(gcs_engine* e, const gcs_bd_config* cfg, int64_t step, double* dev_reaction)
{
    return domain_step_impl(e, cfg, step, dev_reaction, false);
}

int gcs_engine_domain_finish(gcs_engine* e, const double* dev_reaction)
{
    if (!e || !dev_reaction) return fail(GCS_EINVAL, "null argument");
    if (!e->dom) return fail(GCS_ESTATE, "gcs_engine_set_domain first");
    HIPCHK(hipSetDevice(e->device));
    if (e->dom_list) {
        enqueue_dom_list_finish(e, dev_reaction, nullptr, 0);
    } else {
        ForceArgs a = domain_args(e);
        a.ext_react = dev_reaction;
        const int sb = step_grid(e);
        launch_tail(e->stream, e->ctx, a, sb, sb, 1, e->sched_flags != 0, e->ncell_max, e->dsched);
        launch_domain_shared_in(e->stream, a, e->dom_shared_idx, e->dom_nshared, dev_reaction);
    }
    HIPCHK(hipGetLastError());
    e->parity ^= 1;
    e->dom_cont = true;
    return GCS_OK;
}

int gcs_engine_domain_pack(gcs_engine* e, void* dev_out, int32_t* dev_counts, int32_t cap, int32_t* dev_flags)
{
    if (!e || (e->dom_npeer > 0 && (!dev_out || !dev_counts)) || !dev_flags) return fail(GCS_EINVAL, "null argument");
    if (!e->dom) return fail(GCS_ESTATE, "gcs_engine_set_domain first");
    if (cap < 1) return fail(GCS_EINVAL, "band capacity must be positive");
    HIPCHK(hipSetDevice(e->device));
    if (e->dom_npeer > 0) HIPCHK(hipMemsetAsync(dev_counts, 0, e->dom_npeer * sizeof(int), e->stream));
    launch_domain_pack(e->stream, e->ctx, domain_args(e), e->dom_regions, e->dom_npeer, dev_out, dev_counts,
                       cap, dev_flags, e->dom_shared_flag, 0, 1, e->dom_list ? 1 : 0);
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

int gcs_engine_domain_unpack(gcs_engine* e, const void* dev_in, const int32_t* dev_counts, int32_t nbuf, int32_t cap)
{
    if (!e || (nbuf > 0 && (!dev_in || !dev_counts))) return fail(GCS_EINVAL, "null argument");
    if (nbuf <= 0) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    launch_domain_unpack(e->stream, domain_args(e), dev_in, dev_counts, nbuf, cap, 0, 1,
                         e->dom_list ? 1 : 0, e->dom_send, e->dom_send ? e->dom_npeer : 0, e->dom_cap + 1);
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

// ---- engine-owned exchange: bands with the count in their header row, the reaction buffer, the flags --------------

int gcs_engine_domain_buffers(gcs_engine* e, int32_t cap, int32_t* nred)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    if (!e->dom) return fail(GCS_ESTATE, "gcs_engine_set_domain first");
    if (cap < 1) return fail(GCS_EINVAL, "band capacity must be positive");
    HIPCHK(hipSetDevice(e->device));
    dfree(e->dom_send);
    dfree(e->dom_recv);
    dfree(e->dom_red);
    dfree(e->dom_glob);
    const size_t rows = (size_t)std::max(e->dom_npeer, 1) * (cap + 1);
    const int nr = kDomainRed + 3 * e->dom_nshared + e->dom_ndom;
    int rc;
    const size_t rb = band_record_bytes(e->prec);
    if ((rc = dalloc(&e->dom_send, rows * rb)) || (rc = dalloc(&e->dom_recv, rows * rb)) || (rc = dalloc(&e->dom_red, nr)) ||
        (rc = dalloc(&e->dom_glob, nr)))
        return rc;
    if (!e->dom_flags && (rc = dalloc(&e->dom_flags, 1))) return rc;
    HIPCHK(hipMemsetAsync(e->dom_send, 0, rows * rb, e->stream));
    HIPCHK(hipMemsetAsync(e->dom_recv, 0, rows * rb, e->stream));
    HIPCHK(hipMemsetAsync(e->dom_red, 0, nr * sizeof(double), e->stream));
    HIPCHK(hipMemsetAsync(e->dom_glob, 0, nr * sizeof(double), e->stream));
    HIPCHK(hipMemsetAsync(e->dom_flags, 0, sizeof(int), e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->dom_cap = cap;
    e->dom_nred = nr;
    if (nred) *nred = nr;
    drop_domain_graph(e);
    return GCS_OK;
}

namespace {

// pack this step's bands into the send buffer (header rows zeroed first unless the tail did, counts land in them)
void enqueue_band_pack(gcs_engine* e, bool headers_zeroed = false)
{
    const int stride = e->dom_cap + 1;
    const size_t rb = band_record_bytes(e->prec);
    if (!headers_zeroed) launch_band_headers_zero(e->stream, e->dom_send, e->dom_npeer, stride, e->prec);
    launch_domain_pack(e->stream, e->ctx, domain_args(e), e->dom_regions, e->dom_npeer, e->dom_send + rb,
                       reinterpret_cast<int*>(e->dom_send), e->dom_cap, e->dom_flags, e->dom_shared_flag, stride,
                       stride * (int)(rb / sizeof(int)), e->dom_list ? 1 : 0);
}

void enqueue_band_unpack(gcs_engine* e)
{
    const int stride = e->dom_cap + 1;
    if (e->dom_npeer > 0)  // (and the send bands' headers zeroed for the next step's fused pack)
        launch_domain_unpack(e->stream, domain_args(e), e->dom_recv + band_record_bytes(e->prec),
                             reinterpret_cast<const int*>(e->dom_recv), e->dom_npeer, e->dom_cap, stride,
                             stride * (int)(band_record_bytes(e->prec) / sizeof(int)), e->dom_list ? 1 : 0, e->dom_send,
                             e->dom_npeer, stride);
    dbg_sync(e, "dom: k_domain_unpack");
}

// one grouped send/recv of every peer's band (the count in its header row)
int enqueue_band_exchange(gcs_engine* e)
{
    if (e->dom_npeer == 0) return GCS_OK;
    const RcclApi* r = rccl();
    const size_t bytes = band_record_bytes(e->prec) * (e->dom_cap + 1);  // one band: header row + records
    NCCLCHK(r->groupStart());
    for (int p = 0; p < e->dom_npeer; ++p) {
        NCCLCHK(r->send(e->dom_send + (size_t)p * bytes, bytes, ncclUint8, e->dom_peer_rank[p], e->nccl, e->stream));
        NCCLCHK(r->recv(e->dom_recv + (size_t)p * bytes, bytes, ncclUint8, e->dom_peer_rank[p], e->nccl, e->stream));
    }
    NCCLCHK(r->groupEnd());
    return GCS_OK;
}

// one decomposed step after its start (gcs_engine_domain_step primed the run): the domain kernels, the reaction
// allreduce, the tail, the bands to and from every peer (one grouped send/recv per peer, the count in the band)
int enqueue_rccl_step(gcs_engine* e, const gcs_bd_config* cfg, int64_t step)
{
    const RcclApi* r = rccl();
    if (e->dom_list) {
        // list step: k_lstep<DOM> (+ rebuild) with the band pack and the shared particles fused, allreduce, exchange,
        // tail + shared in + unpack (+ the send headers zeroed): 2 launches and 2 collectives per step
        enqueue_dom_list_step(e, step, e->dom_red, true);
        NCCLCHK(r->allReduce(e->dom_red, e->dom_glob, e->dom_nred, ncclDouble, ncclSum, e->nccl, e->stream));
        if (int rc = enqueue_band_exchange(e)) return rc;
        // the tail and the unpack in one launch (k_ldom_finish; the exchange does not depend on the tail)
        const int stride = e->dom_cap + 1;
        const size_t rb = band_record_bytes(e->prec);
        launch_list_domain_finish(e->stream, e->ctx, domain_args(e, e->dom_red), e->dom_glob, e->dom_flags_step & ~8,
                                  e->dom_shared_idx, e->dom_nshared, e->dom_recv + rb,
                                  reinterpret_cast<const int*>(e->dom_recv), e->dom_npeer, e->dom_cap, stride,
                                  stride * (int)(rb / sizeof(int)), e->dom_npeer > 0 ? e->dom_send : nullptr,
                                  e->dom_npeer, stride);
        HIPCHK(hipGetLastError());
        (void)cfg;
        return GCS_OK;
    }
    const ForceArgs a = domain_args(e);
    const DomBox reg = dom_region(e);
    enqueue_count(e, &reg);
    enqueue_scan(e, false);
    enqueue_sort(e);
    launch_force(e->stream, kModeStep, e->waves, e->ctx, a, false);
    launch_tail_reduce(e->stream, e->ctx, a, step_grid(e), e->dom_red);
    launch_domain_shared_out(e->stream, e->ctx, a, e->dom_shared_idx, e->dom_nshared, e->dom_red);
    NCCLCHK(r->allReduce(e->dom_red, e->dom_glob, e->dom_nred, ncclDouble, ncclSum, e->nccl, e->stream));
    ForceArgs f = a;
    f.ext_react = e->dom_glob;
    const int sb = step_grid(e);
    launch_tail(e->stream, e->ctx, f, sb, sb, 1, e->sched_flags != 0, e->ncell_max, e->dsched);
    launch_domain_shared_in(e->stream, f, e->dom_shared_idx, e->dom_nshared, e->dom_glob);
    enqueue_band_pack(e);
    if (int rc = enqueue_band_exchange(e)) return rc;
    enqueue_band_unpack(e);
    HIPCHK(hipGetLastError());
    (void)cfg;
    (void)step;
    return GCS_OK;
}

}  // namespace

int gcs_rccl_unique_id(uint8_t* id)
{
    if (!id) return fail(GCS_EINVAL, "null argument");
    const RcclApi* r = rccl();
    if (!r) return fail(GCS_EHIP, "librccl.so.1 could not be opened");
    ncclUniqueId u;
    NCCLCHK(r->getUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return GCS_OK;
}

int gcs_engine_domain_rccl(gcs_engine* e, const uint8_t* id, int32_t nranks, int32_t rank, const int32_t* peer_ranks)
{
    if (!e || !id || (e->dom_npeer > 0 && !peer_ranks)) return fail(GCS_EINVAL, "null argument");
    if (!e->dom_send) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(GCS_EINVAL, "bad rank");
    const RcclApi* r = rccl();
    if (!r) return fail(GCS_EHIP, "librccl.so.1 could not be opened");
    for (int p = 0; p < e->dom_npeer; ++p) {
        if (peer_ranks[p] < 0 || peer_ranks[p] >= nranks || peer_ranks[p] == rank) return fail(GCS_EINVAL, "bad peer rank");
        e->dom_peer_rank[p] = peer_ranks[p];
    }
    HIPCHK(hipSetDevice(e->device));
    drop_domain_graph(e);  // its collectives name the old communicator
    if (e->nccl) {
        (void)r->commDestroy(e->nccl);
        e->nccl = nullptr;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    NCCLCHK(r->commInitRank(&e->nccl, nranks, u, rank));
    e->nccl_ranks = nranks;
    return GCS_OK;
}

int gcs_engine_domain_run(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps)
{
    if (!e || !cfg) return fail(GCS_EINVAL, "null argument");
    if (!e->nccl) return fail(GCS_ESTATE, "gcs_engine_domain_rccl first");
    if (!e->dom_red || !e->dom_send) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    if (steps < 0) return fail(GCS_EINVAL, "negative step count");
    int64_t k = 0, k0 = 0;
    int rc;
    if (steps > 0 && !(e->dom_cont && e->dom_next == first_step)) {
        // the run's first step primes through the step entry point (begin_run, both position buffers)
        if ((rc = gcs_engine_domain_step(e, cfg, first_step, e->dom_red))) return rc;
        const RcclApi* r = rccl();
        NCCLCHK(r->allReduce(e->dom_red, e->dom_glob, e->dom_nred, ncclDouble, ncclSum, e->nccl, e->stream));
        if ((rc = gcs_engine_domain_finish(e, e->dom_glob))) return rc;
        enqueue_band_pack(e);
        if ((rc = enqueue_band_exchange(e))) return rc;
        enqueue_band_unpack(e);
        k = k0 = 1;  // gcs_engine_domain_finish flipped the host parity of this step
    }
    // the rest: G-step chunks captured once into a graph (kernels and collectives), the remainder eagerly.  The list
    // step rebuilds at steps = 0 (mod M): its chunks are whole periods, captured for the rebuild phase they start at.
    // A step that changes the list skin (skin_level; a few times while the core scale grows: a new grid, a rebuild,
    // the period of the new skin) runs eagerly, as do the steps of a chunk that would hold one; the graph is then
    // captured again for the new skin, period and phase
    while (k < steps) {
        const int64_t st = first_step + k;
        const bool change = e->dom_list && skin_level(e, st) != e->skin_level_pm;
        const int M = e->dom_list ? e->list_every : 1;
        const int G = e->graph_steps > 0 ? (e->graph_steps + M - 1) / M * M : 0;
        bool whole = !change && G > 0 && steps - k >= G;
        for (int q = 1; whole && e->dom_list && q < G; ++q) whole = skin_level(e, st + q) == e->skin_level_pm;
        if (!whole) {
            if ((rc = enqueue_rccl_step(e, cfg, st))) return rc;
            e->rstats.eager_steps++;
            ++k;
            continue;
        }
        const int phase = e->dom_list ? (int)((st + e->list_phase) % M) : 0;
        // (geometry, buffers, communicator and options drop the graph when they change: drop_domain_graph)
        const bool same = e->dgexec && e->dg_steps == G && std::memcmp(&e->dg_cfg, cfg, sizeof(*cfg)) == 0 &&
                          e->dg_version == e->topo_version && e->dg_sched_flags == e->sched_flags &&
                          e->dg_phase == phase && e->dg_skin == e->skin_level_pm;
        if (!same) {
            drop_domain_graph(e);
            HIPCHK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
            for (int q = 0; q < G; ++q) {
                if ((rc = enqueue_rccl_step(e, cfg, st + q))) {
                    hipGraph_t g = nullptr;
                    (void)hipStreamEndCapture(e->stream, &g);
                    if (g) (void)hipGraphDestroy(g);
                    return rc;
                }
            }
            HIPCHK(hipStreamEndCapture(e->stream, &e->dgraph));
            HIPCHK(hipGraphInstantiate(&e->dgexec, e->dgraph, nullptr, nullptr, 0));
            e->dg_steps = G;
            e->dg_cfg = *cfg;
            e->dg_version = e->topo_version;
            e->dg_sched_flags = e->sched_flags;
            e->dg_phase = phase;
            e->dg_skin = e->skin_level_pm;
            e->rstats.graphs_captured++;
        }
        if ((rc = launch_graph(e, e->dgexec))) return rc;
        e->rstats.graph_steps += G;
        k += G;
    }
    if ((steps - k0) & 1) e->parity ^= 1;
    if (steps > 0) {
        e->dom_cont = true;
        e->dom_next = first_step + steps;
    }
    e->chain_valid = e->dense_chain = false;
    return GCS_OK;
}

// ---- host-staged transport (any process layout, e.g. several processes on one device): one step's halves ------

int gcs_engine_domain_step_host(gcs_engine* e, const gcs_bd_config* cfg, int64_t step, double* red, int32_t nred)
{
    if (!e || !red) return fail(GCS_EINVAL, "null argument");
    if (!e->dom_red) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    if (nred != e->dom_nred) return fail(GCS_EINVAL, "reaction buffer size does not match");
    int rc = domain_step_impl(e, cfg, step, e->dom_red, true);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(red, e->dom_red, nred * sizeof(double), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_domain_finish_host(gcs_engine* e, const double* glob, int32_t nred)
{
    if (!e || !glob) return fail(GCS_EINVAL, "null argument");
    if (!e->dom_glob) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    if (nred != e->dom_nred) return fail(GCS_EINVAL, "reaction buffer size does not match");
    HIPCHK(hipMemcpyAsync(e->dom_glob, glob, nred * sizeof(double), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));  // glob is the caller's
    return gcs_engine_domain_finish(e, e->dom_glob);
}

int gcs_engine_domain_pack_host(gcs_engine* e, void* bands)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    if (!e->dom_send) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    HIPCHK(hipSetDevice(e->device));
    if (!e->dom_fused) enqueue_band_pack(e);  // (a fused step packed its bands already)
    HIPCHK(hipGetLastError());
    if (!bands) return GCS_OK;  // packed on the device only (in-process transport: gcs_engine_domain_receive)
    if (e->dom_npeer > 0)
        HIPCHK(hipMemcpyAsync(bands, e->dom_send, (size_t)e->dom_npeer * (e->dom_cap + 1) * band_record_bytes(e->prec),
                              hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_domain_unpack_host(gcs_engine* e, const void* bands)
{
    if (!e || (e->dom_npeer > 0 && !bands)) return fail(GCS_EINVAL, "null argument");
    if (!e->dom_recv) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    if (e->dom_npeer == 0) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpyAsync(e->dom_recv, bands, (size_t)e->dom_npeer * (e->dom_cap + 1) * band_record_bytes(e->prec),
                          hipMemcpyHostToDevice, e->stream));
    enqueue_band_unpack(e);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));  // bands is the caller's
    return GCS_OK;
}

int gcs_engine_domain_receive(gcs_engine* dst, int32_t dst_slot, gcs_engine* src, int32_t src_slot)
{
    if (!dst || !src) return fail(GCS_EINVAL, "null argument");
    if (!dst->dom_recv || !src->dom_send) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    if (dst->dom_cap != src->dom_cap) return fail(GCS_EINVAL, "band capacities differ");
    if (dst_slot < 0 || dst_slot >= dst->dom_npeer || src_slot < 0 || src_slot >= src->dom_npeer)
        return fail(GCS_EINVAL, "bad band slot");
    if (dst->device != src->device) return fail(GCS_EINVAL, "in-process bands move within one device");
    if (dst->prec != src->prec) return fail(GCS_EINVAL, "band records differ in precision");
    HIPCHK(hipSetDevice(dst->device));
    hipEvent_t ev, done;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev, src->stream));
    HIPCHK(hipStreamWaitEvent(dst->stream, ev, 0));
    const size_t rows = (size_t)dst->dom_cap + 1;
    const size_t rb = band_record_bytes(dst->prec);
    HIPCHK(hipMemcpyAsync(dst->dom_recv + (size_t)dst_slot * rows * rb, src->dom_send + (size_t)src_slot * rows * rb,
                          rows * rb, hipMemcpyDeviceToDevice, dst->stream));
    // and src's stream waits for the copy: its unpack zeroes the band's header row for the next step's fused pack
    HIPCHK(hipEventRecord(done, dst->stream));
    HIPCHK(hipStreamWaitEvent(src->stream, done, 0));
    HIPCHK(hipEventDestroy(ev));
    HIPCHK(hipEventDestroy(done));
    return GCS_OK;
}

int gcs_engine_domain_unpack_received(gcs_engine* e)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    if (!e->dom_recv) return fail(GCS_ESTATE, "gcs_engine_domain_buffers first");
    HIPCHK(hipSetDevice(e->device));
    enqueue_band_unpack(e);
    HIPCHK(hipGetLastError());
    return GCS_OK;
}

int gcs_engine_domain_flags(gcs_engine* e, int32_t* flags)
{
    if (!e || !flags) return fail(GCS_EINVAL, "null argument");
    *flags = 0;
    if (!e->dom_flags) return GCS_OK;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpyAsync(flags, e->dom_flags, sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return GCS_OK;
}

int gcs_engine_profile(gcs_engine* e, const gcs_bd_config* cfg, int64_t first_step, int64_t steps, gcs_profile* out)
{
    if (!e || !cfg || !out) return fail(GCS_EINVAL, "null argument");
    if (steps <= 0) return fail(GCS_EINVAL, "profile needs at least one step");
    if (cfg->spacestep > 0) return fail(GCS_EINVAL, "profile covers the fixed-timestep path only");
    if (cfg->noise == GCS_NOISE_INJECTED && e->noise_cursor + steps > e->noise_steps)
        return fail(GCS_ESTATE, "not enough injected noise for the requested steps");
    if (int rc = flush_contacts(e)) return rc;
    int rc = begin_run(e, cfg, first_step);
    if (rc) return rc;
    std::vector<hipEvent_t> ev((size_t)steps * 5 + 2, nullptr);
    // GCS_DEBUG_TIMES=<file>: per-block timings of the last profiled force launch (see k_force)
    const char* dbg_path = std::getenv("GCS_DEBUG_TIMES");
    unsigned long long* dbg = nullptr;
    const size_t dbg_n = (size_t)step_grid(e) * 8 + 2 * (size_t)rebuild_blocks(e->ncell_max);
    if (dbg_path) HIPCHK(hipMalloc(&dbg, dbg_n * sizeof(unsigned long long)));
    // GCS_DEBUG_BUILD=<file>: k_lbuild's per-workgroup stamps of the last list build in the profiled steps
    const char* dbgb_path = std::getenv("GCS_DEBUG_BUILD");
    unsigned long long* dbgb = nullptr;
    const size_t dbgb_n = (size_t)force_grid(e->n) * 8;
    if (dbgb_path) {
        HIPCHK(hipMalloc(&dbgb, dbgb_n * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(dbgb, 0, dbgb_n * sizeof(unsigned long long), e->stream));
    }
    for (auto& x : ev) HIPCHK(hipEventCreate(&x));
    const int fb = step_grid(e);
    HIPCHK(hipEventRecord(ev[0], e->stream));
    const bool rebuild = rebuild_path(e, false), lst = list_path(e, false);
    // per step: [1] cells [2] force [3] unfused: tail [4] - [5]
    // (rebuild: [1] - [2] force [3] rebuild + tail [4] - [5]; list: [1] cells + list build on rebuild steps
    // [2] list step incl. its tail [3] - [4] - [5])
    for (int64_t k = 0; k < steps; ++k) {
        HIPCHK(hipEventRecord(ev[1 + 5 * k], e->stream));
        if (dbg && k == steps - 1) e->fa.dbg_times = dbg;
        if (lst) {
            const bool build = e->l_need_build || ((first_step + k + e->list_phase) % e->list_every) == 0;
            e->l_need_build = false;
            ForceArgs la = list_args(e);
            if (build) {
                la.dbg_build = dbgb;
                enqueue_count(e);
                enqueue_scan(e, false);
                launch_cell_scatter(e->stream, e->n, e->cell_of, e->slot, e->cstart, e->tmp, e->count);
                enqueue_cell_order(e, true);
                launch_list_build(e->stream, e->ctx, la);
                la.dbg_build = nullptr;
            }
            HIPCHK(hipEventRecord(ev[2 + 5 * k], e->stream));
            ForceArgs lk = la;
            lk.par_hint = e->parity ^ (int)(k & 1);  // as gcs_engine_run launches it
            launch_list_step(e->stream, e->ctx, lk, list_flags(e, first_step + k) | 4 | (k == steps - 1 ? 16 : 0));
            e->fa.dbg_times = nullptr;
            for (int q = 3; q <= 5; ++q) HIPCHK(hipEventRecord(ev[q + 5 * k], e->stream));
            continue;
        }
        if (!rebuild) enqueue_cells(e);
        HIPCHK(hipEventRecord(ev[2 + 5 * k], e->stream));
        if (dbg && k == steps - 1) e->fa.dbg_times = dbg;

        launch_force(e->stream, kModeStep, e->waves, e->ctx, e->fa, rebuild);
        HIPCHK(hipEventRecord(ev[3 + 5 * k], e->stream));
        if (rebuild)
            launch_rebuild(e->stream, e->ctx, e->fa, e->tmp, e->rb_sync, fb, e->sched_flags != 0);
        else
            launch_tail(e->stream, e->ctx, e->fa, fb, fb, 1, e->sched_flags != 0, e->ncell_max, e->dsched);
        e->fa.dbg_times = nullptr;
        HIPCHK(hipEventRecord(ev[4 + 5 * k], e->stream));
        HIPCHK(hipEventRecord(ev[5 + 5 * k], e->stream));
    }
    HIPCHK(hipEventRecord(ev[ev.size() - 1], e->stream));
    HIPCHK(hipGetLastError());
    end_run(e, cfg, first_step, steps);
    HIPCHK(hipStreamSynchronize(e->stream));
    double cell = 0, force = 0, tail = 0;
    for (int64_t k = 0; k < steps; ++k) {
        float t[4] = {0, 0, 0, 0};
        for (int q = 0; q < 4; ++q) HIPCHK(hipEventElapsedTime(&t[q], ev[1 + q + 5 * k], ev[2 + q + 5 * k]));
        force += t[1];
        if (lst) {
            cell += t[0];  // cell list + list build (rebuild steps only)
        } else if (rebuild) {
            cell += t[2];  // rebuild kernel (its tail block runs beside the cell-list blocks)
        } else {
            cell += t[0];
            tail += t[2] + t[3];
        }
    }
    float tot = 0;
    HIPCHK(hipEventElapsedTime(&tot, ev[0], ev[ev.size() - 1]));
    if (dbg) {
        std::vector<unsigned long long> h(dbg_n);
        HIPCHK(hipMemcpyAsync(h.data(), dbg, dbg_n * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        (void)hipFree(dbg);
        if (FILE* f = std::fopen(dbg_path, "wb")) {
            std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
            std::fclose(f);
        }
    }
    if (dbgb) {
        std::vector<unsigned long long> h(dbgb_n);
        HIPCHK(hipMemcpyAsync(h.data(), dbgb, dbgb_n * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        (void)hipFree(dbgb);
        if (FILE* f = std::fopen(dbgb_path, "wb")) {
            std::fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
            std::fclose(f);
        }
    }
    for (auto& x : ev) (void)hipEventDestroy(x);
    if (steps & 1) e->parity ^= 1;
    if (cfg->noise == GCS_NOISE_INJECTED) e->noise_cursor += steps;
    DevCtx d;
    HIPCHK(hipMemcpyAsync(&d, e->ctx, sizeof(d), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    out->steps = steps;
    out->total_ms = tot;
    out->force_ms = force / (double)steps;
    out->cell_ms = cell / (double)steps;
    out->tail_ms = tail / (double)steps;
    if (std::getenv("GCS_DEBUG")) {
        int khz = 0;
        HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, e->device));
        if (khz > 0)
            std::fprintf(stderr, "gcs: grid %d x %d x %d (%d cells), ntiles %d; k_cell_scan body: cells %.2f us, "
                         "rows %.2f us; k_tail body %.2f us\n", d.grid.n[0], d.grid.n[1], d.grid.n[2], d.grid.ncell,
                         d.ntiles, 1e3 * (d.t_last[2] - d.t_last[1]) / khz, 1e3 * (d.t_last[3] - d.t_last[2]) / khz,
                         1e3 * (d.t_tail[1] - d.t_tail[0]) / khz);
        if (khz > 0 && rebuild) {
            auto us = [&](unsigned long long x, unsigned long long y) { return 1e3 * ((double)y - (double)x) / khz; };
            std::fprintf(stderr, "gcs: rebuild: tail block %.2f us\n", us(d.t_tail[0], d.t_tail[1]));
            for (int w = 0; w < 2; ++w) {
                const unsigned long long* pr = w ? d.t_cells : d.t_rows;
                std::fprintf(stderr, "gcs: rebuild %s block: start %+.2f; published %.2f, staged %.2f, "
                             "ranked %.2f, looked back %.2f, barrier %.2f, tables %.2f, copies %.2f us\n",
                             w ? "last" : "middle", us(d.t_tail[0], pr[0]), us(pr[0], pr[1]), us(pr[0], pr[2]),
                             us(pr[0], pr[4]), us(pr[0], pr[3]), us(pr[0], pr[5]), us(pr[0], pr[6]), us(pr[0], pr[7]));
            }
        }
        if (khz > 0)
            std::fprintf(stderr, "gcs: cell probes: start->loaded %.2f, sum %.2f, scan+barrier %.2f, stores %.2f, "
                         "->pass end %.2f us\n", 1e3 * (d.t_cells[0] - d.t_last[0]) / khz,
                         1e3 * (d.t_cells[1] - d.t_cells[0]) / khz, 1e3 * (d.t_cells[2] - d.t_cells[1]) / khz,
                         1e3 * (d.t_cells[3] - d.t_cells[2]) / khz, 1e3 * (d.t_last[2] - d.t_cells[3]) / khz);
        if (khz > 0)
            std::fprintf(stderr, "gcs: rows probes: cellpass->rows %.2f, rows scan %.2f, barrier %.2f, stores %.2f, "
                         "->end %.2f us\n", 1e3 * (d.t_rows[0] - d.t_last[2]) / khz,
                         1e3 * (d.t_rows[1] - d.t_rows[0]) / khz, 1e3 * (d.t_rows[2] - d.t_rows[1]) / khz,
                         1e3 * (d.t_rows[3] - d.t_rows[2]) / khz, 1e3 * (d.t_last[3] - d.t_rows[3]) / khz);
    }
    out->mean_neighbors = d.neighbors;
    return GCS_OK;
}

int gcs_engine_set_cu_mask(gcs_engine* e, const uint32_t* mask, int32_t words)
{
    if (!e || (words > 0 && !mask)) return fail(GCS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    hipStream_t s = nullptr;
    if (words > 0) {
        // a CU-masked stream has the default (blocking) flags: it orders against legacy null-stream work, so the
        // engine issues no null-stream copies (every copy is async on e->stream)
        HIPCHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask));
    } else {
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    drop_graph(e);
    (void)hipStreamDestroy(e->stream);
    e->stream = s;
    return GCS_OK;
}

int gcs_engine_get_list_stats(gcs_engine* e, gcs_list_stats* out)
{
    if (!e || !out) return fail(GCS_EINVAL, "null argument");
    HIPCHK(hipSetDevice(e->device));
    DevCtx d;
    HIPCHK(hipMemcpyAsync(&d, e->ctx, sizeof(d), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    out->active = list_path(e, false) ? 1 : 0;
    out->rebuild_every = e->list_every;
    out->builds = d.lbuilds;
    out->fallback_particle_steps = d.lfallback;
    out->skin = list_skin(e);
    out->max_displacement = d.ldisp;
    out->pair_classes = e->ntypes;
    out->capacity = e->list_cap;
    out->sync_stalls = (int64_t)d.scan_stall;
    out->deal = (int64_t)list_deal(e);
    return GCS_OK;
}

int gcs_engine_get_run_stats(gcs_engine* e, gcs_run_stats* out)
{
    if (!e || !out) return fail(GCS_EINVAL, "null argument");
    *out = e->rstats;
    out->graphs_cached = (int64_t)e->graphs.size() + (e->dgexec ? 1 : 0);
    return GCS_OK;
}

int gcs_engine_set_option(gcs_engine* e, int32_t option, int64_t value)
{
    if (!e) return fail(GCS_EINVAL, "null argument");
    e->chain_valid = e->dense_chain = false;
    if (option == GCS_OPT_CONTACT_BITS) {
        if (value != 0 && (value < 10 || value > 34)) return fail(GCS_EINVAL, "contact bits must be 0 or in [10, 34]");
        if (e->c_keys) return fail(GCS_ESTATE, "the contact map is already allocated");
        e->c_bits_opt = (int)value;
        return GCS_OK;
    }
    if (option == GCS_OPT_GRAPH_STEPS) {
        if (value < 0 || value > 4096) return fail(GCS_EINVAL, "graph steps must be in [0, 4096]");
        e->graph_steps = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_SKIN) {
        if (value < 0 || value > 4000)
            return fail(GCS_EINVAL, "list skin must be in [1, 4000] per mille of the cutoff (0: the default)");
        e->list_skin_pm = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_SKIN_BASE) {
        if (value < 0 || value > 4000)
            return fail(GCS_EINVAL, "list skin base must be in [1, 4000] per mille of the cutoff (0: the default)");
        if (e->dom && (int)value != e->list_skin_base_pm)
            return fail(GCS_ESTATE, "the list skin base sizes a decomposed engine's binning halo: set it before the "
                                    "domain");
        e->list_skin_base_pm = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_EVERY) {
        if (value < 0 || value > 4096) return fail(GCS_EINVAL, "list rebuild period must be in [0, 4096] (0 = auto)");
        e->list_every_opt = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_WAVES) {
        if (value != 2 && value != 4) return fail(GCS_EINVAL, "list waves per tile must be 2 or 4");
        e->list_waves = (int)value;
        if (!deal_valid(e->list_deal_opt, e->list_waves)) e->list_deal_opt = -1;  // back to the default
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_DEAL) {
        if (value != -1 && !deal_valid(value, e->list_waves))
            return fail(GCS_EINVAL, "list deal must be -1, 0 or (period << 60 | wave nibbles < waves per tile)");
        e->list_deal_opt = value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_FORMAT) {
        if (value < 0 || value > 2)
            return fail(GCS_EINVAL, "list format must be 0 (default: 16-bit slots, absolute up to 65,536 particles, "
                                    "plane-relative beyond), 1 (plane-relative 16-bit) or 2 (32-bit)");
        e->list_fmt_opt = (int)value;
        e->l_need_build = true;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_CAP) {
        // whole batches of 8 entries per wave segment (2 or 4 waves)
        if (value < 32 || value > 16384 || (value % (8 * kMaxListWaves)) != 0)
            return fail(GCS_EINVAL, "list capacity must be a multiple of 32 in [32, 16384]");
        e->list_cap = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_DENSE_NEIGHBORS) {
        if (value < 0) return fail(GCS_EINVAL, "dense threshold must be >= 0");
        e->dense_opt = (int)value;
        e->chain_valid = e->dense_chain = false;
        return GCS_OK;
    }
    if (option == GCS_OPT_LIST_PHASE) {
        if (value < 0 || value > 1024) return fail(GCS_EINVAL, "list phase must be in [0, 1024]");
        e->list_phase = (int)value;
        e->l_need_build = true;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_SMALL_STEP) {
        if (value != 0 && value != 1) return fail(GCS_EINVAL, "small step must be 0 or 1");
        e->small_opt = (int)value;
        return GCS_OK;
    }
    if (option == GCS_OPT_FUSED_STEP) {
        if (value != 0 && value != 2 && value != 3) return fail(GCS_EINVAL, "fused step must be 0, 2 or 3");
        if (e->prec == 64 && value == 2)
            return fail(GCS_EINVAL, "the fp64 engine runs the list step (3) or its cell-list step (0)");
        e->fused = (int)value;
        e->fused_explicit = true;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_CHUNK_ORDER) {
        if (value != 0 && value != 1) return fail(GCS_EINVAL, "chunk order must be 0 (contiguous) or 1 (strided)");
        e->fa.chunk_mode = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_SCAN_BLOCKS) {
        if (value != 0 && value != 1) return fail(GCS_EINVAL, "scan blocks must be 0 (one block) or 1 (multi-block)");
        e->scan_mb = value != 0;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_SUBTILES) {
        if (value != 1 && value != 2 && value != 4) return fail(GCS_EINVAL, "sub-tiles must be 1, 2 or 4");
        e->fa.subtiles = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_TILE_PRIORITY) {
        if (value < 0 || value > (1 << 20)) return fail(GCS_EINVAL, "tile priority step must be in [0, 2^20]");
        e->fa.prio_step = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_SPLIT_TILES) {
        if (value < 0 || value > 2) return fail(GCS_EINVAL, "split tiles must be 0, 1 or 2");
        e->fa.split = (int)value;
        drop_graph(e);
        return GCS_OK;
    }
    if (option == GCS_OPT_WAVES_PER_TILE) {
        if (value != 1 && value != 2 && value != 4 && value != 8) return fail(GCS_EINVAL, "waves per tile must be 1, 2, 4 or 8");
        e->waves = (int)value;
        e->resident = std::min(force_step_resident(e->waves), kMaxUnits);
        drop_graph(e);
        return GCS_OK;
    }
    return fail(GCS_EINVAL, "unknown option");
}

}  // extern "C"
