// kernels.hip -- CDNA4 (gfx950, wave64) kernels of the gcs engine.
//
// One Brownian-dynamics step = 6 launches on one stream (captured into a hipGraph by the host):
//   cell_count   per particle: cell of its position, slot = atomicAdd(count[cell])
//   cell_scan    1 block: exclusive scan count -> cstart, re-zero count
//   cell_scatter per particle: tmp[cstart[cell] + slot] = particle
//   cell_sort    per sorted slot: rank inside the cell by particle index (deterministic order),
//                write the cell-sorted copies spos/sb/sidx/scell
//   force        per 64-particle tile (WAVES waves): gather-form pair loop over the tile's stencil rows
//                (wave-uniform neighbour reads -> scalar loads), + bonded/bending/tether/point/wall terms,
//                + the Euler-Maruyama update; per-block reaction / bbox partials; no atomics
//   tail         1 block: reduce the partials in a fixed order (fp64), apply the interphase schedule
//                (time, core/bond scale, wall ODE), build the next step's cell grid
// Replaces: md::simulate_brownian_dynamics's force+integrator loop as driven from
// stage_interphase/simulation_driver_interphase.cpp:57-63 (force fields: simulation_driver_forcefield.cpp:9-244).
#include "engine_internal.hpp"

#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <type_traits>

#include "../../include/gcs.h"

namespace gcs {

namespace {

// 16-B L1-bypassing (sc1) load through a buffer descriptor (out-of-range offsets read 0): the single-block
// reductions read data written by other CUs once, so there is nothing to gain from L1
__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, int byte_off)
{
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
    float4 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}
__device__ __forceinline__ void st_sc1_f4(__amdgpu_buffer_rsrc_t r, int byte_off, float4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned*>(&v),
                                           r, byte_off, 0, 16);
}
__device__ __forceinline__ int4 ld_sc1_i4(__amdgpu_buffer_rsrc_t r, int byte_off)
{
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
    int4 f;
    __builtin_memcpy(&f, &v, 16);
    return f;
}
// DPP wave primitives (GFX9 row_shr / row_bcast): an inclusive scan in 6 DPP steps without LDS.  Lanes whose
// DPP source is out of range take `ident` (bound_ctrl off, old = ident).  After the sequence lane l holds
// op(x_0 .. x_l); lane 63 holds the wave total.  Fixed combination order: bitwise reproducible.
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i(int ident, int x)
{
    return __builtin_amdgcn_update_dpp(ident, x, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM>
__device__ __forceinline__ float dpp_f(float ident, float x)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ident), __float_as_int(x), CTRL, RM, 0xf, false));
}
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_d(double ident, double x)
{
    const long long o = __double_as_longlong(ident), v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)v, CTRL, RM, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(v >> 32), CTRL, RM, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
#define GCS_DPP_SCAN(DPP, OP, IDENT, X)              \
    X = OP(X, DPP<0x111, 0xf>(IDENT, X)); /* shr 1 */ \
    X = OP(X, DPP<0x112, 0xf>(IDENT, X)); /* shr 2 */ \
    X = OP(X, DPP<0x114, 0xf>(IDENT, X)); /* shr 4 */ \
    X = OP(X, DPP<0x118, 0xf>(IDENT, X)); /* shr 8 */ \
    X = OP(X, DPP<0x142, 0xa>(IDENT, X)); /* bcast 15 -> rows 1, 3 */ \
    X = OP(X, DPP<0x143, 0xc>(IDENT, X)); /* bcast 31 -> rows 2, 3 */

__device__ __forceinline__ int add_i(int a, int b) { return a + b; }
__device__ __forceinline__ int max_i(int a, int b) { return max(a, b); }
__device__ __forceinline__ int min_i(int a, int b) { return min(a, b); }
__device__ __forceinline__ double add_d(double a, double b) { return a + b; }
__device__ __forceinline__ float min_f(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ float max_f(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ double max_d(double a, double b) { return fmax(a, b); }

__device__ __forceinline__ int wave_incl_scan_dpp(int v)
{
    GCS_DPP_SCAN(dpp_i, add_i, 0, v)
    return v;
}
__device__ __forceinline__ double lane63_d(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ float lane63_f(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63)); }
__device__ __forceinline__ double wave_total_sum_d(double v)
{
    GCS_DPP_SCAN(dpp_d, add_d, 0.0, v)
    return lane63_d(v);
}
__device__ __forceinline__ double wave_total_max_d(double v)
{
    GCS_DPP_SCAN(dpp_d, max_d, -1.0e300, v)
    return lane63_d(v);
}
__device__ __forceinline__ float wave_total_min_f(float v)
{
    GCS_DPP_SCAN(dpp_f, min_f, 3.0e38f, v)
    return lane63_f(v);
}
__device__ __forceinline__ float wave_total_max_f(float v)
{
    GCS_DPP_SCAN(dpp_f, max_f, -3.0e38f, v)
    return lane63_f(v);
}

// Whole-wave reductions (all lanes active, result wave-uniform): the DPP scan above plus a readlane of lane 63 --
// six VALU steps with no LDS round trip, where a __shfl_xor butterfly is six dependent ds_bpermute waits.
__device__ __forceinline__ float add_f(float a, float b) { return a + b; }
__device__ inline float wave_sum(float v)
{
    GCS_DPP_SCAN(dpp_f, add_f, 0.f, v)
    return lane63_f(v);
}
__device__ inline double wave_sum_d(double v) { return wave_total_sum_d(v); }
__device__ inline float wave_max(float v)
{
    GCS_DPP_SCAN(dpp_f, max_f, -__builtin_huge_valf(), v)
    return lane63_f(v);
}
__device__ inline float wave_min(float v)
{
    GCS_DPP_SCAN(dpp_f, min_f, __builtin_huge_valf(), v)
    return lane63_f(v);
}

__device__ inline int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ inline float uniform_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

// ---- precision-generic scalar helpers (R = float: exactly the fp32 builtins the fp32 kernels always used) ----
template <typename R> __device__ __forceinline__ R r_sqrt(R x)
{
    if constexpr (sizeof(R) == 4) return sqrtf(x); else return sqrt(x);
}
template <typename R> __device__ __forceinline__ R r_rsqrt(R x)
{
    if constexpr (sizeof(R) == 4) return rsqrtf(x); else return rsqrt(x);
}
template <typename R> __device__ __forceinline__ R r_fma(R a, R b, R c)
{
    if constexpr (sizeof(R) == 4) return fmaf(a, b, c); else return fma(a, b, c);
}
template <typename R> __device__ __forceinline__ R r_fmax(R a, R b)
{
    if constexpr (sizeof(R) == 4) return fmaxf(a, b); else return fmax(a, b);
}
template <typename R> __device__ __forceinline__ R r_fabs(R x)
{
    if constexpr (sizeof(R) == 4) return fabsf(x); else return fabs(x);
}
template <typename R> __device__ __forceinline__ R r_atan2(R y, R x)
{
    if constexpr (sizeof(R) == 4) return atan2f(y, x); else return atan2(y, x);
}
template <typename R> __device__ __forceinline__ R wave_sum_r(R v)
{
    if constexpr (sizeof(R) == 4) return wave_sum(v); else return wave_sum_d(v);
}
// the integer a slot-ordered position record carries in .w (particle | class << 24): the float's bits in fp32, the
// low word of the double's bits in fp64


__device__ inline int wave_max_int(int v)
{
    GCS_DPP_SCAN(dpp_i, max_i, (int)0x80000000, v)
    return __builtin_amdgcn_readlane(v, 63);
}


__device__ inline int cell_index(const Grid& g, float x, float y, float z)
{
    int cx = (int)((x - g.lo[0]) * g.inv[0]);
    int cy = (int)((y - g.lo[1]) * g.inv[1]);
    int cz = (int)((z - g.lo[2]) * g.inv[2]);
    cx = min(max(cx, 0), g.n[0] - 1);
    cy = min(max(cy, 0), g.n[1] - 1);
    cz = min(max(cz, 0), g.n[2] - 1);
    return cx + g.n[0] * (cy + g.n[1] * cz);
}

// Cell grid over the box [lo, hi]; cell edge >= rc (x edge rc / fx) plus a margin, so any pair closer than rc lies
// in the same or an adjacent cell (+-fx in x).  The margin covers the binning's fp32 arithmetic: 1e-4 of the edge,
// plus, in length units, the roundings of a particle's coordinate (2^-24 |x|, the fp32 copy of an fp64 position)
// and of (x - lo) * inv (2^-24 of the extent each), for both particles of a pair, with a factor 2 to spare:
// 2.5e-7 (max(|lo|, |hi|) + 2 extent) -- which matters far from the origin and at the 1,024-cell cap.
// Particles outside the box are clamped into the border cells, which keeps that property because clamping never
// increases a per-axis cell distance.
__device__ __forceinline__ Grid make_grid(const float* lo, const float* hi, float rc, int ncell_max, int fx)
{
    Grid g;
    int n[3];
    float ext[3];
    long long total = 1;
    for (int k = 0; k < 3; ++k) {
        float e = hi[k] - lo[k];
        if (!(e > 0.f) || !(e < 3.0e38f)) e = 0.f;
        ext[k] = e;
        const float edge = (k == 0) ? rc / (float)fx : rc;
        const float mag = (e > 0.f) ? fmaxf(fabsf(lo[k]), fabsf(hi[k])) : 0.f;
        float q = (rc > 0.f) ? e / (edge * 1.0001f + 2.5e-7f * (mag + 2.f * e)) : 0.f;
        int m = (q >= 1.f) ? (int)fminf(q, 1024.f) : 1;
        n[k] = m;
        total *= m;
    }
    while (total > ncell_max) {  // halve the longest axis (no dynamic array indexing: keeps it in registers)
        if (n[0] >= n[1] && n[0] >= n[2])
            n[0] = max(1, n[0] / 2);
        else if (n[1] >= n[2])
            n[1] = max(1, n[1] / 2);
        else
            n[2] = max(1, n[2] / 2);
        total = (long long)n[0] * n[1] * n[2];
    }
    for (int k = 0; k < 3; ++k) {
        g.lo[k] = (ext[k] > 0.f) ? lo[k] : 0.f;
        g.n[k] = n[k];
        g.inv[k] = ext[k] > 0.f ? (float)n[k] / ext[k] : 0.f;
    }
    g.ncell = (int)total;
    g.fx = (n[0] > 1) ? fx : 1;
    g.rc = rc;
    g.rc2 = rc * rc;
    return g;
}

__device__ __forceinline__ void compute_grid(DevCtx* ctx, float rc, int ncell_max, int fx)
{
    ctx->grid = make_grid(ctx->bbox_lo, ctx->bbox_hi, rc, ncell_max, fx);
}

// The grid that bins the positions produced by the NEXT step: the current bbox padded by 2 % + 0.01 (particles
// move far less per step; any that leave are clamped, which is still exact) and the pair cutoff that step
// will use, i.e. with the core scale the schedule sets after step `step` (closed form of update_core_scale).
__device__ __forceinline__ Grid next_grid(const DevCtx* ctx, const ForceArgs& a, const double* sched, long long step, int ncell_max)
{
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        const float pad = 0.02f * fmaxf(ctx->bbox_hi[k] - ctx->bbox_lo[k], 0.f) + 0.01f;
        lo[k] = ctx->bbox_lo[k] - pad;
        hi[k] = ctx->bbox_hi[k] + pad;
    }
    double cs = ctx->cs;
    const int flags = (int)sched[kSchedFlags];
    if (flags & 2) {
        const double t = (flags & 1) ? (double)step * sched[kSchedDt] : ctx->time;
        cs = 1.0 - (1.0 - sched[kSchedCs0]) * exp(-(t / sched[kSchedCsTau]));
    }
    const float rc = a.has_pair ? a.pf.pair_dist * (a.pair_scaled ? (float)fmax(cs, ctx->cs) : 1.f) : 1.f;
    return make_grid(lo, hi, rc, ncell_max, kPairFx);
}

__device__ inline float pair_cutoff(const ForceArgs& a, double cs)
{
    if (!a.has_pair) return 1.f;
    return a.pf.pair_dist * (a.pair_scaled ? (float)cs : 1.f);
}
// the pair cutoff in precision R (fp32: exactly pair_cutoff)
template <typename R>
__device__ inline R pair_cutoff_r(const ForceArgs& a, double cs)
{
    if constexpr (sizeof(R) == 4) {
        return pair_cutoff(a, cs);
    } else {
        if (!a.has_pair) return 1.0;
        return a.pd.pair_dist * (a.pair_scaled ? cs : 1.0);
    }
}

// ----------------------------------------------------------------------------------------------------
// cell list

// R: the positions' precision (the bounding box is taken of their fp32 roundings, which is what the cells bin)
template <typename R>
__global__ __launch_bounds__(1024) void k_prime(DevCtx* ctx, ForceArgs a, float rc_fixed, int ncell_max,
                                                const double* __restrict__ sched)
{
    __shared__ float red[6][16];
    const real4<R>* pos = St<R>::pos(a, ctx->parity);
    float lo[3] = {3.0e38f, 3.0e38f, 3.0e38f}, hi[3] = {-3.0e38f, -3.0e38f, -3.0e38f};
    for (int i = threadIdx.x; i < a.n; i += blockDim.x) {
        const real4<R> p = pos[i];
        const float px = (float)p.x, py = (float)p.y, pz = (float)p.z;
        lo[0] = fminf(lo[0], px);
        lo[1] = fminf(lo[1], py);
        lo[2] = fminf(lo[2], pz);
        hi[0] = fmaxf(hi[0], px);
        hi[1] = fmaxf(hi[1], py);
        hi[2] = fmaxf(hi[2], pz);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int k = 0; k < 3; ++k) {
        float l = wave_min(lo[k]), h = wave_max(hi[k]);
        if (lane == 0) {
            red[k][wave] = l;
            red[3 + k][wave] = h;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = blockDim.x / 64;
        for (int k = 0; k < 3; ++k) {
            float l = red[k][0], h = red[3 + k][0];
            for (int w = 1; w < nw; ++w) {
                l = fminf(l, red[k][w]);
                h = fmaxf(h, red[3 + k][w]);
            }
            ctx->bbox_lo[k] = l;
            ctx->bbox_hi[k] = h;
        }
        float rc = rc_fixed > 0.f ? rc_fixed : pair_cutoff(a, ctx->cs) + a.list_skin;
        compute_grid(ctx, rc, ncell_max, rc_fixed > 0.f ? 1 : kPairFx);
        if (sched) ctx->grid_next = next_grid(ctx, a, sched, ctx->step + 1, ncell_max);
        ctx->ticket = 0u;
    }
}

// dom != 0: bin only the particles inside reg (a domain's box extended by its halo); islot: reset to -1 (k_cell_sort
// writes the binned particles' slots)
template <typename P>
__global__ __launch_bounds__(256) void k_cell_count(const DevCtx* __restrict__ ctx, const P* __restrict__ p0,
                                                    const P* __restrict__ p1, int n, int* __restrict__ cell_of,
                                                    int* __restrict__ slot, int* __restrict__ count, int dom,
                                                    DomBox reg, int* __restrict__ islot)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const P* pos = ctx->parity ? p1 : p0;
    const Grid g = ctx->grid;
    const P pr = pos[i];
    const float4 p = make_float4((float)pr.x, (float)pr.y, (float)pr.z, 0.f);  // fp64 positions bin by their rounding
    const int c = cell_index(g, p.x, p.y, p.z);
    if (islot) islot[i] = -1;
    if (dom && !box_has(reg, p.x, p.y, p.z)) {  // domain: outside its region, not binned
        cell_of[i] = -1;
        return;
    }
    cell_of[i] = c;
    slot[i] = atomicAdd(&count[c], 1);
}

// exclusive scan of the wave (64 lanes), returns the inclusive value
__device__ inline int wave_incl_scan(int v, int lane)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    return v;
}

// Exclusive scan count -> cstart over the grid's cells, kScanSeg consecutive cells per thread (16-B loads, the
// next iteration's issued before this one's scan) with a running carry, re-zeroing count for the next step; then
// the per-row tile table of k_force (a tile is <= 64 consecutive sorted particles of ONE row of cells).  Wave
// scans are DPP (no LDS round trips); the wave totals are double-buffered in LDS, so each iteration has one
// barrier.  Row starts are captured in LDS during the cell pass (rows <= kRowsLds), so the row pass does not
// re-read cstart.  count/cstart are padded by kScanPad so whole iterations may be touched; entries past ncell
// are zero by invariant.  Any block size that is a multiple of 64 (<= 1024).
constexpr int kRowsLds = 4096;
constexpr int kCellsLds = 16384;

// Row pass of the cell scan: tiles per row, their prefix (tile_start) and the tile table.  Row starts come from
// LDS (LDS = true) or from cstart; two instantiations so the LDS path carries no global-load wait (on gfx9
// vmcnt also counts the cell pass's stores).
template <bool LDS>
__device__ __forceinline__ void scan_rows(DevCtx* __restrict__ ctx, const int* s_rowbeg, const int* __restrict__ cstart,
                                          int nx, int nrows, int* __restrict__ tile_start,
                                          int2* __restrict__ tile_range, int (*wtot)[16], int it, int* s_tstart,
                                          const int* s_cst, int4* __restrict__ units, int budget, int ny, int nz,
                                          int gfx)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    int carry = 0;
    const int span = 4 * blockDim.x;
    if (tid == 0) ctx->t_rows[0] = wall_clock64();
    for (int base = 0; base < nrows; base += span, ++it) {
        int beg[5];  // starts of rows base + 4 tid + q, q = 0..4
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            const int r = base + 4 * tid + q;
            beg[q] = (r <= nrows) ? (LDS ? s_rowbeg[r] : cstart[r * nx]) : 0;
        }
        int c[4];
        int sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = base + 4 * tid + q;
            c[q] = (r < nrows) ? (beg[q + 1] - beg[q] + kTile - 1) / kTile : 0;
            sum += c[q];
        }
        const int incl = wave_incl_scan_dpp(sum);
        if (tid == 0) ctx->t_rows[1] = wall_clock64();
        if (lane == 63) wtot[it & 1][wave] = incl;
        __syncthreads();
        if (tid == 0) ctx->t_rows[2] = wall_clock64();
        int woff = 0, ttot = 0;
        for (int w = 0; w < nw; ++w) {
            const int t = wtot[it & 1][w];
            woff += (w < wave) ? t : 0;
            ttot += t;
        }
        int run = carry + woff + incl - sum;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int r = base + 4 * tid + q;
            if (r < nrows) {
                if (LDS) {
                    s_tstart[r] = run;
                } else {
                    tile_start[r] = run;
                    const int rb = beg[q], re = beg[q + 1];
                    for (int k = 0; k < c[q]; ++k)
                        tile_range[run + k] = make_int2(rb + k * kTile, min(re, rb + (k + 1) * kTile));
                }
            }
            run += c[q];
        }
        carry += ttot;
    }
    bool units_ok = false;
    int nunits = carry;
    if (LDS) {
        // tile-parallel table: thread t writes tiles t, t + blockDim, ... (coalesced); its row by binary search
        if (tid == 0) s_tstart[nrows] = carry;
        __syncthreads();
        auto tile_of = [&](int k, int& row, int& sb, int& se) {
            int lo = 0, hi = nrows;  // last row r with s_tstart[r] <= k (that row is non-empty)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_tstart[mid] <= k)
                    lo = mid;
                else
                    hi = mid;
            }
            const int j = k - s_tstart[lo], rb = s_rowbeg[lo], re = s_rowbeg[lo + 1];
            row = lo;
            sb = rb + j * kTile;
            se = min(re, rb + (j + 1) * kTile);
        };
        const int ntl = carry;
        const int room = budget - ntl;  // budget = resident workgroups of the force launch
        if (s_cst && units && room > 0 && ntl <= 4 * (int)blockDim.x) {
            // Heavy-tile selection for the next force launch.  A tile's pair work is its stencil's candidate count
            // (the force kernel's `total`): from the cell starts in LDS, the cells of its first and last
            // particle, x-range +-fx, 9 row segments.  Up to `budget` tiles (the workgroups that stay resident
            // beside one per tile) whose count is at least 1.25x the mean and in the top `budget` are split in
            // two units (split units first, adjacent pairs; then the others), so the densest tiles get 8 waves.
            // budget - ntiles = the workgroups that stay resident beside one per tile.
            __shared__ int s_hist[128];
            __shared__ int s_red[2][16];
            __shared__ int s_thr;
            int cost[4], srow[4], ssb[4], sse[4];
            int lmax = 0, lsum = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = 4 * tid + q;
                cost[q] = 0;
                srow[q] = ssb[q] = sse[q] = 0;
                if (k < ntl) {
                    tile_of(k, srow[q], ssb[q], sse[q]);
                    tile_range[k] = make_int2(ssb[q], sse[q]);
                    const int cb = srow[q] * nx;
                    int x0 = 0, x1 = 0;
                    for (int step = 1 << (31 - __clz(nx)); step > 0; step >>= 1) {
                        if (x0 + step < nx && s_cst[cb + x0 + step] <= ssb[q]) x0 += step;
                        if (x1 + step < nx && s_cst[cb + x1 + step] <= sse[q] - 1) x1 += step;
                    }
                    const int xlo = max(x0 - gfx, 0), xhi = min(x1 + gfx, nx - 1);
                    const int y0 = srow[q] % ny, z0 = srow[q] / ny;
                    int v = 0;
#pragma unroll
                    for (int d = 0; d < 9; ++d) {
                        const int y = y0 + d % 3 - 1, z = z0 + d / 3 - 1;
                        if (y >= 0 && y < ny && z >= 0 && z < nz) {
                            const int base = (z * ny + y) * nx;
                            v += s_cst[base + xhi + 1] - s_cst[base + xlo];
                        }
                    }
                    cost[q] = v;
                    lmax = max(lmax, v);
                    lsum += v;
                }
            }
            if (tid < 128) s_hist[tid] = 0;
            // block max and sum
            int wm = lmax, ws = lsum;
            GCS_DPP_SCAN(dpp_i, max_i, 0, wm)
            GCS_DPP_SCAN(dpp_i, add_i, 0, ws)
            if (lane == 63) {
                s_red[0][wave] = wm;
                s_red[1][wave] = ws;
            }
            __syncthreads();
            int cmax = 0;
            long long csum = 0;
            for (int w = 0; w < nw; ++w) {
                cmax = max(cmax, s_red[0][w]);
                csum += s_red[1][w];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * tid + q < ntl) atomicAdd(&s_hist[(int)(((long long)cost[q] * 128) / (cmax + 1))], 1);
            __syncthreads();
            if (wave == 0) {
                // lowest bin b whose tiles at or above it fit the room: P(b) >= ntiles - room with P the exclusive
                // prefix of the histogram (lane l holds bins 2l, 2l + 1; one DPP scan, one wave minimum)
                const int h0 = s_hist[2 * lane], h1 = s_hist[2 * lane + 1];
                int pre = h0 + h1;
                GCS_DPP_SCAN(dpp_i, add_i, 0, pre)
                const int p_lo = pre - h0 - h1, p_mid = p_lo + h0, need = ntl - room;
                int bmin = (p_lo >= need) ? 2 * lane : ((p_mid >= need) ? 2 * lane + 1 : 128);
                GCS_DPP_SCAN(dpp_i, min_i, 128, bmin)
                if (lane == 63) {
                    // cost >= thr_bin <=> bin >= bmin; never below 1.25x the mean cost
                    const int thr_bin = (int)(((long long)bmin * (cmax + 1) + 127) / 128);
                    const int floor_cost = (int)((csum * 5) / (4LL * max(ntl, 1)));
                    s_thr = max(max(thr_bin, floor_cost), 1);
                }
            }
            __syncthreads();
            const int thr = s_thr;
            int nsp = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) nsp += (4 * tid + q < ntl && cost[q] >= thr) ? 1 : 0;
            int incl = nsp;
            GCS_DPP_SCAN(dpp_i, add_i, 0, incl)
            if (lane == 63) wtot[(it + 1) & 1][wave] = incl;
            __syncthreads();
            int woff = 0, total_split = 0;
            for (int w = 0; w < nw; ++w) {
                const int t = wtot[(it + 1) & 1][w];
                woff += (w < wave) ? t : 0;
                total_split += t;
            }
            int rs = woff + incl - nsp;  // split tiles before mine
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = 4 * tid + q;
                if (k >= ntl) continue;
                if (cost[q] >= thr) {
                    units[2 * rs] = make_int4(ssb[q], sse[q], k, 0 | (2 << 8));
                    units[2 * rs + 1] = make_int4(ssb[q], sse[q], k, 1 | (2 << 8));
                    ++rs;
                } else {
                    units[2 * total_split + (k - rs)] = make_int4(ssb[q], sse[q], k, 0 | (1 << 8));
                }
            }
            units_ok = true;
            nunits = ntl + total_split;
        } else {
            for (int k = tid; k < carry; k += blockDim.x) {
                int row, sb, se;
                tile_of(k, row, sb, se);
                tile_range[k] = make_int2(sb, se);
            }
        }
    }
    if (tid == 0) {
        tile_start[nrows] = carry;
        ctx->ntiles = carry;
        ctx->units_ok = units_ok ? 1 : 0;
        ctx->nunits = nunits;
        ctx->t_rows[3] = wall_clock64();
    }
}

// Cell pass of the cell scan: SEG consecutive cells per thread (16-B loads), DPP wave scan, one barrier per pass
// (double-buffered wave totals), cstart stores, row starts (and, for the heavy-tile selection, every cell start)
// captured in LDS.  PREFETCH issues the next pass's loads before this pass's scan.
template <int SEG, bool PREFETCH>
__device__ __forceinline__ void scan_cell_pass(const int* __restrict__ count, int* __restrict__ cstart, int nc, int nx,
                                               bool rows_lds, int* s_rowbeg, bool cells_lds, int* s_cst,
                                               int (*wtot)[16], int& carry, int& it, DevCtx* ctx)
{
    static_assert(SEG % 4 == 0, "counts are loaded as int4");
    constexpr int kQ = SEG / 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int span = SEG * blockDim.x;
    const auto rc = __builtin_amdgcn_make_buffer_rsrc((void*)count, 0, nc * 4, 0x00020000);  // past nc: 0
    int4 cur[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) cur[q] = ld_sc1_i4(rc, (SEG * tid + 4 * q) * 4);
    for (int base = 0; base < nc; base += span, ++it) {
        const int i0 = base + SEG * tid;
        int4 nxt[PREFETCH ? kQ : 1];
        if (PREFETCH && base + span < nc) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) nxt[q] = ld_sc1_i4(rc, (i0 + span + 4 * q) * 4);
        }
        if (tid == 0 && it == 0) ctx->t_cells[0] = wall_clock64();
        int sum = 0;
#pragma unroll
        for (int q = 0; q < kQ; ++q) sum += cur[q].x + cur[q].y + cur[q].z + cur[q].w;
        if (tid == 0 && it == 0) ctx->t_cells[1] = wall_clock64();
        const int incl = wave_incl_scan_dpp(sum);
        if (lane == 63) wtot[it & 1][wave] = incl;
        __syncthreads();
        if (tid == 0 && it == 0) ctx->t_cells[2] = wall_clock64();
        int woff = 0, ttot = 0;
        for (int w = 0; w < nw; ++w) {
            const int t = wtot[it & 1][w];
            woff += (w < wave) ? t : 0;
            ttot += t;
        }
        const int run = carry + woff + incl - sum;
        // row boundaries (cells r * nx) are recognised as the running cell index reaches the next one
        int r = (i0 + nx - 1) / nx;
        int nb = (rows_lds && i0 < nc) ? r * nx : 0x7fffffff;
        int acc = run;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {  // (count is re-zeroed by the scatter, which knows the occupied cells)
            const int4 st = make_int4(acc, acc + cur[q].x, acc + cur[q].x + cur[q].y,
                                      acc + cur[q].x + cur[q].y + cur[q].z);
            const int c = i0 + 4 * q;
            if (c < nc) *reinterpret_cast<int4*>(cstart + c) = st;
            if (cells_lds) {
                if (c < nc) s_cst[c] = st.x;
                if (c + 1 < nc) s_cst[c + 1] = st.y;
                if (c + 2 < nc) s_cst[c + 2] = st.z;
                if (c + 3 < nc) s_cst[c + 3] = st.w;
            }
            while (nb < c + 4 && nb < nc) {  // at most a few per thread
                const int j = nb - c;
                s_rowbeg[r] = j == 0 ? st.x : (j == 1 ? st.y : (j == 2 ? st.z : st.w));
                nb += nx;
                ++r;
            }
            acc = st.w + cur[q].w;
        }
        if (tid == 0 && it == 0) ctx->t_cells[3] = wall_clock64();
        carry += ttot;
        if (PREFETCH) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) cur[q] = nxt[q];
        }
    }
}

__device__ __forceinline__ void scan_cells_body(DevCtx* __restrict__ ctx, int n, int* __restrict__ count,
                                                int* __restrict__ cstart, int* __restrict__ tile_start,
                                                int2* __restrict__ tile_range, bool use_next,
                                                int4* __restrict__ units, int resident)
{
    const Grid& g = use_next ? ctx->grid_next : ctx->grid;
    __shared__ int wtot[2][16];
    __shared__ int s_rowbeg[kRowsLds + 1];
    __shared__ int s_tstart[kRowsLds + 1];
    __shared__ int s_cst[kCellsLds + 1];  // cell starts (heavy-tile selection)
    const int nc = g.ncell, nx = g.n[0], nrows = g.n[1] * g.n[2];
    const bool rows_lds = nrows <= kRowsLds;
    const bool cells_lds = rows_lds && nc <= kCellsLds && units != nullptr && resident > 0;
    const int tid = threadIdx.x;
    int carry = 0, it = 0;
    // up to 48 Ki cells: one pass of 48 cells per thread; beyond, 16-cell passes with the next pass prefetched
    if (nc <= 48 * (int)blockDim.x)
        scan_cell_pass<48, false>(count, cstart, nc, nx, rows_lds, s_rowbeg, cells_lds, s_cst, wtot, carry, it, ctx);
    else
        scan_cell_pass<16, true>(count, cstart, nc, nx, rows_lds, s_rowbeg, cells_lds, s_cst, wtot, carry, it, ctx);
    // the binned total (= n unless a decomposed domain left particles outside its region unbinned)
    if (tid == 0) {
        cstart[nc] = carry;
        if (rows_lds) s_rowbeg[nrows] = carry;
        if (cells_lds) s_cst[nc] = carry;
        ctx->t_last[2] = wall_clock64();
    }
    __syncthreads();
    if (rows_lds)
        scan_rows<true>(ctx, s_rowbeg, cstart, nx, nrows, tile_start, tile_range, wtot, it, s_tstart,
                        cells_lds ? s_cst : nullptr, cells_lds ? units : nullptr, resident, g.n[1], g.n[2], g.fx);
    else
        scan_rows<false>(ctx, s_rowbeg, cstart, nx, nrows, tile_start, tile_range, wtot, it, s_tstart, nullptr,
                         nullptr, 0, g.n[1], g.n[2], g.fx);
}

__global__ __launch_bounds__(1024) void k_cell_scan(DevCtx* __restrict__ ctx, int n, int* __restrict__ count,
                                                    int* __restrict__ cstart, int* __restrict__ tile_start,
                                                    int2* __restrict__ tile_range, int use_next,
                                                    int4* __restrict__ units, int resident)
{
    const unsigned long long t0 = wall_clock64();
    scan_cells_body(ctx, n, count, cstart, tile_start, tile_range, use_next != 0, units, resident);
    if (threadIdx.x == 0) {
        ctx->t_last[0] = ctx->t_last[1] = t0;
        ctx->t_last[3] = wall_clock64();
    }
}

template <int kTailRows = 8>
__device__ __forceinline__ void tail_body(DevCtx* ctx, const ForceArgs& a, int fblocks, int bblocks, int advance,
                                          int apply_sched, int ncell_max, const double* __restrict__ sched, bool fused,
                                          double* red_out = nullptr);

// Multi-block cell scan (same outputs as k_cell_scan without the heavy-tile unit table).  Block b owns rows
// [b*R, b*R + R) of the grid, R = max(1, kMbCells / nx): it scans their cells (8 consecutive cells per thread,
// DPP wave scans), captures the row starts and the per-row tile counts in LDS, publishes its particle and tile
// totals as two 8-byte {tag, value} granules, then sums its predecessors' granules (one wave; every earlier
// block was dispatched first and waits only on blocks before it) and writes cstart, tile_start and the tile
// table with those offsets.  The block owning the last row writes the totals and advances the epoch word
// sync[0] (tag = epoch + 1, so granules of earlier launches never match).  Rows wider than kMbCells are scanned
// in chunks, twice (the second pass writes).  Bitwise the same tables as the single-block scan.
constexpr int kMbThreads = 256;
constexpr int kMbSeg = 8;
constexpr int kMbCells = kMbThreads * kMbSeg;
constexpr unsigned kMbSpinCap = 1u << 22;  // look-back polls before giving up (ctx->scan_stall: the host's reads fail)

typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ int mb_rows_per_block(int nx) { return max(1, kMbCells / nx); }

// block-wide exclusive scan of one int per thread; returns the exclusive prefix, `total` the block sum
__device__ __forceinline__ int mb_block_scan(int v, int (*wtot)[kMbThreads / 64], int it, int& total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan_dpp(v);
    if (lane == 63) wtot[it & 1][wave] = incl;
    __syncthreads();
    int woff = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < kMbThreads / 64; ++w) {
        const int t = wtot[it & 1][w];
        woff += (w < wave) ? t : 0;
        total += t;
    }
    return woff + incl - v;
}

// Look-back of the multi-block scans, by one wave: the sums of the {tag, value} granules 2 + 2j (particles) and
// 3 + 2j (tiles) of blocks j < b into s_off[0..1].  Each lane issues its granules kLbBatch at a time (one memory
// round trip per batch instead of one per granule) and re-polls only those not yet tagged.
constexpr int kLbBatch = 8;
__device__ __forceinline__ void lookback_sum(DevCtx* ctx, const unsigned long long* sync, int b, unsigned tag, int lane,
                                             long long* s_off)
{
    long long p = 0, t = 0;
    bool stalled = false;
    for (int base = 0; base < 2 * b; base += 64 * kLbBatch) {
        unsigned long long x[kLbBatch];
#pragma unroll
        for (int k = 0; k < kLbBatch; ++k) {
            const int j = base + 64 * k + lane;
            x[k] = (j < 2 * b) ? __hip_atomic_load((gu64*)(sync + 2 + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : ((unsigned long long)tag << 32);
        }
#pragma unroll
        for (int k = 0; k < kLbBatch; ++k) {
            const int j = base + 64 * k + lane;
            unsigned spins = 0;
            while ((unsigned)(x[k] >> 32) != tag && ++spins < kMbSpinCap)
                x[k] = __hip_atomic_load((gu64*)(sync + 2 + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            stalled |= (unsigned)(x[k] >> 32) != tag;
            if (j & 1)
                t += (unsigned)x[k];
            else
                p += (unsigned)x[k];
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        p += __shfl_xor(p, o);
        t += __shfl_xor(t, o);
    }
    if (__any(stalled) && lane == 0) atomicAdd(&ctx->scan_stall, 1);
    if (lane == 0) {
        s_off[0] = p;
        s_off[1] = t;
    }
}

__global__ __launch_bounds__(kMbThreads) void k_cell_scan_mb(DevCtx* __restrict__ ctx, int n,
                                                              const int* __restrict__ count, int* __restrict__ cstart,
                                                              int* __restrict__ tile_start,
                                                              int2* __restrict__ tile_range, int use_next,
                                                              unsigned long long* __restrict__ sync)
{
    const Grid& g = use_next ? ctx->grid_next : ctx->grid;
    const int nx = g.n[0], nrows = g.n[1] * g.n[2], nc = g.ncell;
    const int rpb = mb_rows_per_block(nx);
    const int nb = (nrows + rpb - 1) / rpb;
    const int b = blockIdx.x;
    if (b >= nb) return;
    __shared__ int wtot[2][kMbThreads / 64];
    __shared__ int s_rowbeg[kMbCells + 1];  // block-local row starts (rows per block <= kMbCells)
    __shared__ long long s_off[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned tag = (unsigned)sync[0] + 1u;
    const int r0 = b * rpb, r1 = min(nrows, r0 + rpb), nr = r1 - r0;
    const int c0 = r0 * nx, c1 = r1 * nx;
    const bool one_chunk = c1 - c0 <= kMbCells;
    int it = 0;

    // pass 1: cell sums, the block-local cell prefix (kept in registers for a single chunk), row starts
    int loc[kMbSeg];
    int carry = 0;
    for (int base = c0; base < c1; base += kMbCells, ++it) {
        const int i0 = base + kMbSeg * tid;
        int v[kMbSeg];
        int sum = 0;
#pragma unroll
        for (int k = 0; k < kMbSeg; ++k) {
            v[k] = (i0 + k < c1) ? count[i0 + k] : 0;
            sum += v[k];
        }
        int ttot;
        int acc = carry + mb_block_scan(sum, wtot, it, ttot);
        int nbnd = ((i0 - c0 + nx - 1) / nx) * nx + c0;  // first row boundary at or after i0
#pragma unroll
        for (int k = 0; k < kMbSeg; ++k) {
            loc[k] = acc;
            if (i0 + k == nbnd && nbnd < c1) {
                s_rowbeg[(nbnd - c0) / nx] = acc;
                nbnd += nx;
            }
            acc += v[k];
        }
        carry += ttot;
    }
    if (tid == 0) {
        s_rowbeg[nr] = carry;
        __hip_atomic_store((gu64*)(sync + 2 + 2 * b), ((unsigned long long)tag << 32) | (unsigned)carry,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();

    // tiles per row (<= kTile consecutive sorted particles of one row each) and their block-local prefix
    const int rpt = (nr + kMbThreads - 1) / kMbThreads;  // rows per thread, contiguous
    const int q0 = min(nr, tid * rpt), q1 = min(nr, q0 + rpt);
    int tsum = 0;
    for (int q = q0; q < q1; ++q) tsum += (s_rowbeg[q + 1] - s_rowbeg[q] + kTile - 1) / kTile;
    int ttiles;
    const int texcl = mb_block_scan(tsum, wtot, it, ttiles);
    ++it;
    if (tid == 0)
        __hip_atomic_store((gu64*)(sync + 3 + 2 * b), ((unsigned long long)tag << 32) | (unsigned)ttiles,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // look-back: one wave sums the granules of blocks 0 .. b-1 (even words particles, odd words tiles)
    if (wave == 0) lookback_sum(ctx, sync, b, tag, lane, s_off);
    __syncthreads();
    const int poff = (int)s_off[0], toff = (int)s_off[1];

    // pass 2: cstart (from registers, or a second chunked scan), tile_start and the tile table
    if (one_chunk) {
        const int i0 = c0 + kMbSeg * tid;
#pragma unroll
        for (int k = 0; k < kMbSeg; ++k)
            if (i0 + k < c1) cstart[i0 + k] = poff + loc[k];
    } else {
        carry = poff;
        for (int base = c0; base < c1; base += kMbCells, ++it) {
            const int i0 = base + kMbSeg * tid;
            int v[kMbSeg];
            int sum = 0;
#pragma unroll
            for (int k = 0; k < kMbSeg; ++k) {
                v[k] = (i0 + k < c1) ? count[i0 + k] : 0;
                sum += v[k];
            }
            int ttot;
            int acc = carry + mb_block_scan(sum, wtot, it, ttot);
#pragma unroll
            for (int k = 0; k < kMbSeg; ++k) {
                if (i0 + k < c1) cstart[i0 + k] = acc;
                acc += v[k];
            }
            carry += ttot;
        }
    }
    int tile = toff + texcl;  // this thread's rows' first tile
    for (int q = q0; q < q1; ++q) {
        const int rb = poff + s_rowbeg[q], re = poff + s_rowbeg[q + 1];
        tile_start[r0 + q] = tile;
        for (int s = rb; s < re; s += kTile) tile_range[tile++] = make_int2(s, min(re, s + kTile));
    }
    if (b == nb - 1 && tid == 0) {
        const int ntl = toff + ttiles;
        cstart[nc] = poff + carry;  // the binned total (see scan_cells_body)
        tile_start[nrows] = ntl;
        ctx->ntiles = ntl;
        ctx->units_ok = 0;
        ctx->nunits = ntl;
        __hip_atomic_store((gu64*)sync, (unsigned long long)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Rebuild step (GCS_OPT_FUSED_STEP 2): everything between two force kernels in ONE launch.  Block 0 runs the
// step's tail (tail_body: reductions, schedule, wall, grid <- grid_next).  Blocks 1.. rebuild the cell list the
// force kernel filed into its per-cell buckets, each owning rows of the grid (R = max(1, kRbCells / nx) rows):
// the count scan, row starts and tiles of k_cell_scan_mb with the same look-back, and the cell-sorted copies
// (spos / sb / sidx / scell) of its cells, members ordered by particle index inside each cell (as k_cell_sort).
// A bucket entry carries the whole sorted record (new position, pair factors, particle), so the copies need no
// gathers.  Up to kRbPcap particles per block the records are staged and ranked through registers + LDS;
// denser blocks, or rows wider than kRbCells, stage the entry ids in `tmp` (same result).  The grid, parity
// and step come from the rb_* copies the force kernel stashed, so block 0 may advance the live ones meanwhile.
constexpr int kRbThreads = 256;
constexpr int kRbSeg = 1;
constexpr int kRbCells = kRbThreads * kRbSeg;
constexpr int kRbPcap = 2048;

// a member's record: bucket slot j < kBucketCap of cell c, or overflow entry k (src = -(k + 1))
__device__ __forceinline__ void rb_load(const ForceArgs& a, int c, int j, int src, float4& p, int& i, float& b)
{
    if (src >= 0) {
        const size_t e = (size_t)c * kBucketCap + j;
        p = a.bucket_p[e];
        const int2 q = a.bucket_q[e];
        i = q.x;
        b = __int_as_float(q.y);
    } else {
        p = a.ovf_p[-src - 1];
        const int4 q = a.ovf_q[-src - 1];
        i = q.x;
        b = __int_as_float(q.y);
    }
}

__device__ __forceinline__ void rb_store(const ForceArgs& a, int d, int i, int c, float4 p, float b)
{
    const_cast<float4*>(a.spos)[d] = p;
    const_cast<float*>(a.sb)[d] = b;
    const_cast<int*>(a.sidx)[d] = i;
    const_cast<int*>(a.scell)[d] = c;
}

// overflow entries filed under cell c, in list order: put(q, -(k + 1)) for the q-th one (q from kBucketCap)
template <typename Put>
__device__ __forceinline__ void rb_overflow(const ForceArgs& a, int novf, int c, Put put)
{
    int q = kBucketCap;
    for (int k = 0; k < novf; ++k)
        if (a.ovf_q[k].z == c) put(q++, -(k + 1));
}

__global__ __launch_bounds__(kRbThreads) void k_rebuild(DevCtx* __restrict__ ctx, ForceArgs a, int* __restrict__ tmp,
                                                        unsigned long long* __restrict__ sync, int fblocks,
                                                        int apply_sched)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // GCS_DEBUG_TIMES: per-block {start, end} after the force kernel's 8 words per force block
    unsigned long long* const dbg = (a.dbg_times && tid == 0) ? a.dbg_times + 8 * fblocks + 2 * blockIdx.x : nullptr;
    if (dbg) dbg[0] = wall_clock64();
    if (blockIdx.x == 0) {
        const long long st = ctx->rb_step;
        const unsigned long long t0 = wall_clock64();
        tail_body(ctx, a, fblocks, fblocks, 1, apply_sched, a.ncell_max, a.sched, true);
        if (tid == 0) {
            a.ovf_n[(st + 1) & 1] = 0;  // the next force kernel's overflow counter (last read one step ago)
            ctx->t_tail[0] = t0;
            ctx->t_tail[1] = wall_clock64();
            if (dbg) dbg[1] = ctx->t_tail[1];
        }
        return;
    }
    const Grid& g = ctx->rb_grid;
    const int nx = g.n[0], nrows = g.n[1] * g.n[2], nc = g.ncell;
    const int rpb = max(1, kRbCells / nx);
    const int nb = (nrows + rpb - 1) / rpb;
    const int b = blockIdx.x - 1;
    if (b >= nb) {
        if (dbg) dbg[1] = wall_clock64();
        return;
    }
    // GCS_DEBUG probes: the middle block in t_rows, the last in t_cells (start, published, looked back, end)
    unsigned long long* const probe =
        (tid == 0 && (b == nb / 2 || b == nb - 1)) ? (b == nb / 2 ? ctx->t_rows : ctx->t_cells) : nullptr;
    if (probe) probe[0] = wall_clock64();
    const int novf = a.ovf_n[ctx->rb_step & 1];
    __shared__ int wtot[2][kRbThreads / 64];
    __shared__ int s_rowbeg[kRbCells + 1];  // block-local row starts
    __shared__ int s_cst[kRbCells + 1];     // block-local cell starts (single chunk)
    __shared__ int s_mcell[kRbPcap];        // LDS path: block-local cell of each staged slot
    __shared__ int s_src[kRbPcap];          // LDS path: overflow source of slots past kBucketCap; then slot order
    __shared__ float4 s_rp[kRbPcap];        // LDS path: staged records (LDS-DMA): position + a factor
    __shared__ int s_ri[kRbPcap];           //   particle
    __shared__ int s_rb[kRbPcap];           //   b factor bits
    __shared__ long long s_off[2];
    const unsigned tag = (unsigned)sync[0] + 1u;
    const int r0 = b * rpb, r1 = min(nrows, r0 + rpb), nr = r1 - r0;
    const int c0 = r0 * nx, c1 = r1 * nx;
    const bool one_chunk = c1 - c0 <= kRbCells;
    int it = 0;

    // pass 1: cell counts -> block-local cell starts (registers + LDS), row starts
    int v[kRbSeg], loc[kRbSeg];
    int carry = 0;
    for (int base = c0; base < c1; base += kRbCells, ++it) {
        const int i0 = base + kRbSeg * tid;
        int sum = 0;
#pragma unroll
        for (int k = 0; k < kRbSeg; ++k) {
            v[k] = (i0 + k < c1) ? a.count[i0 + k] : 0;
            sum += v[k];
        }
        int ttot;
        int acc = carry + mb_block_scan(sum, wtot, it, ttot);
        int nbnd = ((i0 - c0 + nx - 1) / nx) * nx + c0;  // first row boundary at or after i0
#pragma unroll
        for (int k = 0; k < kRbSeg; ++k) {
            loc[k] = acc;
            if (one_chunk && i0 + k < c1) s_cst[i0 + k - c0] = acc;
            if (i0 + k == nbnd && nbnd < c1) {
                s_rowbeg[(nbnd - c0) / nx] = acc;
                nbnd += nx;
            }
            acc += v[k];
        }
        carry += ttot;
    }
    const int P = carry;  // particles of this block's cells
    if (tid == 0) {
        s_rowbeg[nr] = P;
        if (one_chunk) s_cst[c1 - c0] = P;
        __hip_atomic_store((gu64*)(sync + 2 + 2 * b), ((unsigned long long)tag << 32) | (unsigned)P,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool lds = one_chunk && P <= kRbPcap;
    if (lds) {
        // slot -> cell map (and the overflow sources) by each cell's owner; counts re-zeroed for the next binning
        const int i0 = c0 + kRbSeg * tid;
#pragma unroll
        for (int k = 0; k < kRbSeg; ++k) {
            const int c = i0 + k;
            if (c < c1 && v[k] > 0) {
                a.count[c] = 0;
                const int ls = loc[k];
#pragma unroll
                for (int j = 0; j < kBucketCap; ++j)
                    if (j < v[k]) s_mcell[ls + j] = c - c0;
                if (v[k] > kBucketCap)
                    rb_overflow(a, novf, c, [&](int q, int src) {
                        s_mcell[ls + q] = c - c0;
                        s_src[ls + q] = src;
                    });
            }
        }
    }
    __syncthreads();

    // tiles per row and their block-local prefix
    const int rpt = (nr + kRbThreads - 1) / kRbThreads;
    const int q0 = min(nr, tid * rpt), q1 = min(nr, q0 + rpt);
    int tsum = 0;
    for (int q = q0; q < q1; ++q) tsum += (s_rowbeg[q + 1] - s_rowbeg[q] + kTile - 1) / kTile;
    int ttiles;
    const int texcl = mb_block_scan(tsum, wtot, it, ttiles);
    ++it;
    if (tid == 0)
        __hip_atomic_store((gu64*)(sync + 3 + 2 * b), ((unsigned long long)tag << 32) | (unsigned)ttiles,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (probe) probe[1] = wall_clock64();

    // LDS path: every record straight into LDS (LDS-DMA, no VGPR round trip), then each member's rank in its
    // cell (by particle index) -> the slot order s_src[cell start + rank] = staged slot; all in rolled loops (this
    // code runs once per step per CU: its instruction fetch is part of the critical path)
    if (lds) {
        typedef __attribute__((address_space(1))) void gvoid;
        typedef __attribute__((address_space(3))) void lvoid;
        for (int s0 = wave * 64; s0 < P; s0 += kRbThreads) {
            const int s = s0 + lane;
            if (s < P) {
                const int lc = s_mcell[s], j = s - s_cst[lc];
                const float4* gp;
                const int* gq;
                if (j < kBucketCap) {
                    const size_t e = (size_t)(c0 + lc) * kBucketCap + j;
                    gp = a.bucket_p + e;
                    gq = reinterpret_cast<const int*>(a.bucket_q + e);
                } else {
                    const int k = -s_src[s] - 1;
                    gp = a.ovf_p + k;
                    gq = reinterpret_cast<const int*>(a.ovf_q + k);
                }
                __builtin_amdgcn_global_load_lds((gvoid*)gp, (lvoid*)(s_rp + s0), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((gvoid*)gq, (lvoid*)(s_ri + s0), 4, 0, 0);
                __builtin_amdgcn_global_load_lds((gvoid*)(gq + 1), (lvoid*)(s_rb + s0), 4, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (probe) probe[2] = wall_clock64();
        for (int s = tid; s < P; s += kRbThreads) {
            const int i = s_ri[s], lc = s_mcell[s];
            const int ls = s_cst[lc], le = s_cst[lc + 1];
            int r = 0;
            for (int t = ls; t < le; t += 4) {  // 4 independent LDS reads per round (clamped, masked)
                const int x0 = s_ri[t], x1 = s_ri[min(t + 1, le - 1)], x2 = s_ri[min(t + 2, le - 1)],
                          x3 = s_ri[min(t + 3, le - 1)];
                r += (x0 < i) + ((t + 1 < le) & (x1 < i)) + ((t + 2 < le) & (x2 < i)) + ((t + 3 < le) & (x3 < i));
            }
            s_src[ls + r] = s;
        }
        if (probe) probe[4] = wall_clock64();
    }

    // look-back: one wave sums the granules of blocks 0 .. b-1 (even words particles, odd words tiles)
    if (wave == 0) lookback_sum(ctx, sync, b, tag, lane, s_off);
    if (probe) probe[3] = wall_clock64();
    __syncthreads();
    const int poff = (int)s_off[0], toff = (int)s_off[1];
    if (probe) probe[5] = wall_clock64();

    // cstart, tile_start, tile table
    if (one_chunk) {
        const int i0 = c0 + kRbSeg * tid;
#pragma unroll
        for (int k = 0; k < kRbSeg; ++k)
            if (i0 + k < c1) a.cstart_w[i0 + k] = poff + loc[k];
    } else {
        carry = poff;
        for (int base = c0; base < c1; base += kRbCells, ++it) {
            const int i0 = base + kRbSeg * tid;
            int w[kRbSeg];
            int sum = 0;
#pragma unroll
            for (int k = 0; k < kRbSeg; ++k) {
                w[k] = (i0 + k < c1) ? a.count[i0 + k] : 0;
                sum += w[k];
            }
            int ttot;
            int acc = carry + mb_block_scan(sum, wtot, it, ttot);
#pragma unroll
            for (int k = 0; k < kRbSeg; ++k) {
                if (i0 + k < c1) a.cstart_w[i0 + k] = acc;
                acc += w[k];
            }
            carry += ttot;
        }
    }
    int tile = toff + texcl;
    for (int q = q0; q < q1; ++q) {
        const int rb = poff + s_rowbeg[q], re = poff + s_rowbeg[q + 1];
        a.tile_start_w[r0 + q] = tile;
        for (int s = rb; s < re; s += kTile) a.tile_range_w[tile++] = make_int2(s, min(re, s + kTile));
    }
    if (b == nb - 1 && tid == 0) {
        const int ntl = toff + ttiles;
        a.cstart_w[nc] = a.n;
        a.tile_start_w[nrows] = ntl;
        ctx->ntiles = ntl;
        ctx->units_ok = 0;
        ctx->nunits = ntl;
        __hip_atomic_store((gu64*)sync, (unsigned long long)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    if (probe) probe[6] = wall_clock64();
    // cell-sorted copies: the member of rank r (by particle index) in its cell goes to slot cell start + r
    if (lds) {
        // coalesced: sorted slot poff + t takes the staged record s_src[t]
        for (int t = tid; t < P; t += kRbThreads) {
            const int src = s_src[t];
            rb_store(a, poff + t, s_ri[src], c0 + s_mcell[src], s_rp[src], __int_as_float(s_rb[src]));
        }
    } else {
        // global staging: tmp[slot] = the record's source (bucket entry j of its cell, or -(overflow index + 1))
        __syncthreads();  // this block's cstart entries are visible to all its threads
        const int pend = poff + P;
        for (int c = c0 + tid; c < c1; c += kRbThreads) {
            const int cs = a.cstart_w[c], ce = (c + 1 < c1) ? a.cstart_w[c + 1] : pend;
            const int m = min(ce - cs, kBucketCap);
            for (int j = 0; j < m; ++j) tmp[cs + j] = j;
            if (ce - cs > kBucketCap) rb_overflow(a, novf, c, [&](int q, int src) { tmp[cs + q] = src; });
        }
        __syncthreads();
        for (int s = poff + tid; s < pend; s += kRbThreads) {
            int lo = c0, hi = c1;  // last cell c with cstart[c] <= s (it is non-empty)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (a.cstart_w[mid] <= s)
                    lo = mid;
                else
                    hi = mid;
            }
            const int cs = a.cstart_w[lo], ce = (lo + 1 < c1) ? a.cstart_w[lo + 1] : pend;
            float4 p;
            float bf;
            int i;
            rb_load(a, lo, s - cs, tmp[s], p, i, bf);
            int r = 0;
            for (int t = cs; t < ce; ++t) {
                float4 pt;
                float bt;
                int it2;
                rb_load(a, lo, t - cs, tmp[t], pt, it2, bt);
                r += (it2 < i) ? 1 : 0;
            }
            rb_store(a, cs + r, i, lo, p, bf);
        }
        __syncthreads();  // every count read above
        for (int c = c0 + tid; c < c1; c += kRbThreads) a.count[c] = 0;
    }
    if (probe) probe[7] = wall_clock64();
    if (dbg) dbg[1] = wall_clock64();
}

__global__ __launch_bounds__(256) void k_cell_scatter(int n, const int* __restrict__ cell_of, const int* __restrict__ slot,
                                                      const int* __restrict__ cstart, int* __restrict__ tmp,
                                                      int* __restrict__ count)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = cell_of[i];
    if (c < 0) return;  // not binned (domain decomposition)
    tmp[cstart[c] + slot[i]] = i;
    count[c] = 0;  // every occupied cell has a particle here: count is all-zero again for the next binning
}

// R: the positions' precision.  spos / sb are fp32 always (the list build and the tile step read them: in fp64 the
// roundings of the fp64 positions, which only place particles in cells and candidates in lists -- every pair force
// and pair test of the fp64 step reads psort); psort / skmu are in the positions' precision
template <typename R>
__global__ __launch_bounds__(256) void k_cell_sort(const DevCtx* __restrict__ ctx, const real4<R>* __restrict__ p0,
                                                   const real4<R>* __restrict__ p1, const real4<R>* __restrict__ kmu,
                                                   int n, const int* __restrict__ tmp, const int* __restrict__ cell_of,
                                                   const int* __restrict__ cstart, int* __restrict__ sidx,
                                                   int* __restrict__ scell, float4* __restrict__ spos,
                                                   float* __restrict__ sb, int pair_mix,
                                                   const int* __restrict__ ptype, real4<R>* __restrict__ psort0,
                                                   real4<R>* __restrict__ psort1, real4<R>* __restrict__ skmu,
                                                   int2* __restrict__ sbrow, const int* __restrict__ boff,
                                                   int* __restrict__ islot, float4* __restrict__ fsort0,
                                                   float4* __restrict__ fsort1, const int* __restrict__ brev,
                                                   int* __restrict__ bslot, const int* __restrict__ swt,
                                                   int* __restrict__ swslot)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    if (s >= cstart[ctx->grid.ncell]) {  // binned particles only (all of them, undecomposed)
        // a decomposed build bins fewer slots than the step launches (n): the step's slot loads still read these
        // slots' records (only `act` masks what it does with them), so they must hold a harmless record -- not
        // what the memory held before (a recycled allocation: a bond row of garbage sends the local-terms wave's
        // gathers anywhere; the round-5 decomposed-test fault).  Particle 0, no bonds, no target
        if (psort0) {
            const real4<R> z = mk4<R>(R(0), R(0), R(0), wpack<R>(0));
            psort0[s] = z;
            psort1[s] = z;
            if (fsort0) fsort0[s] = fsort1[s] = make_float4(0.f, 0.f, 0.f, 0.f);
            skmu[s] = mk4<R>(R(0), R(0), R(0), R(0));
            sbrow[s] = make_int2(0, 0);
        }
        return;
    }
    const real4<R>* pos = ctx->parity ? p1 : p0;
    const int i = tmp[s];
    const int c = cell_of[i];
    const int b = cstart[c], e = cstart[c + 1];
    int r = 0;
    for (int t = b; t < e; ++t) r += (tmp[t] < i) ? 1 : 0;
    const int d = b + r;
    const real4<R> p = pos[i];
    const real4<R> k = kmu ? kmu[i] : mk4<R>(R(1), R(1), R(0), R(0));
    sidx[d] = i;
    scell[d] = c;
    // the pair field's factors: (a, b) when it mixes A/B (interphase), (1, 0) for plain softcore<2,3>
    spos[d] = make_float4((float)p.x, (float)p.y, (float)p.z, pair_mix ? (float)k.y : 1.f);
    sb[d] = pair_mix ? (float)k.z : 0.f;
    if (psort0) {  // list path: the current positions in slot order, .w = particle | class << 24; the slot's
                   // constants and bond CSR row (the list step reads them by slot, not behind the particle index)
        // both parities: the step writes the next parity of the slots it integrates and the unpack both of the
        // ghosts it receives, so a decomposed ghost that misses a record (its band over capacity, or it left the
        // exchange region) keeps this build's record, never what the memory held before
        const real4<R> rec = mk4<R>(p.x, p.y, p.z, wpack<R>(i | (ptype[i] << kListIndexBits)));
        psort0[d] = rec;
        psort1[d] = rec;
        if (fsort0)  // fp64: the list step's prefilter copy (put_slot)
            fsort0[d] = fsort1[d] = make_float4((float)p.x, (float)p.y, (float)p.z, 0.f);
        skmu[d] = k;
        const int2 row = boff ? make_int2(boff[i], boff[i + 1]) : make_int2(0, 0);
        sbrow[d] = row;
        if (islot) islot[i] = d;
        // the slot-indexed partners (ForceArgs::bslot): every entry pointing at this particle -- the reverse of
        // each of its own entries (the CSR holds both directions) -- and its droplet target row learn its slot
        if (bslot)
            for (int q = row.x; q < row.y; ++q) bslot[brev[q]] = d;
        if (swslot) {
            const int t = swt[i];
            if (t >= 0) swslot[t] = d;
        }
    }
}

// ----------------------------------------------------------------------------------------------------
// Brownian step helpers

// Philox4x32-10 normals of particle i at `step` (the oracle's gcso_philox_normals, oracle/rng.c): counter (i, step_lo,
// step_hi, 'GCS1'), key (seed_lo, seed_hi), u = ((r >> 8) + 0.5) 2^-24 (exact in both precisions), Box-Muller on
// (u0, u1) -> x, y and (u2, u3) -> z, evaluated in R
template <typename R>
__device__ inline void philox_normal3(unsigned seed_lo, unsigned seed_hi, long long step, int i, R& n0, R& n1, R& n2)
{
    unsigned c[4] = {(unsigned)i, (unsigned)(unsigned long long)step, (unsigned)((unsigned long long)step >> 32),
                     0x47435331u};
    philox4x32_10(c, seed_lo, seed_hi);
    const R k24 = R(1) / R(16777216);
    R u0 = ((R)(c[0] >> 8) + R(0.5)) * k24;
    R u1 = ((R)(c[1] >> 8) + R(0.5)) * k24;
    R u2 = ((R)(c[2] >> 8) + R(0.5)) * k24;
    R u3 = ((R)(c[3] >> 8) + R(0.5)) * k24;
    R s1, c1, s2, c2, r1, r2;
    if constexpr (sizeof(R) == 4) {
        r1 = sqrtf(-2.0f * logf(u0));
        r2 = sqrtf(-2.0f * logf(u2));
        sincospif(2.0f * u1, &s1, &c1);
        sincospif(2.0f * u3, &s2, &c2);
    } else {
        r1 = sqrt(-2.0 * log(u0));
        r2 = sqrt(-2.0 * log(u2));
        sincospi(2.0 * u1, &s1, &c1);
        sincospi(2.0 * u3, &s2, &c2);
    }
    n0 = r1 * c1;
    n1 = r1 * s1;
    n2 = r2 * c2;
}

template <typename R>
__device__ inline void noise3_at(const ForceArgs& a, long long step, long long cursor, int i, R& n0, R& n1, R& n2)
{
    // the noise of the step after `step` (the context's last completed step), injected noise at `cursor`
    if (a.noise_mode == GCS_NOISE_PHILOX) {
        philox_normal3<R>(a.seed_lo, a.seed_hi, step + 1, i, n0, n1, n2);
    } else if (a.noise_mode == GCS_NOISE_INJECTED) {
        long long cur = cursor;
        if (cur >= a.noise_steps) cur = a.noise_steps - 1;  // host checks the budget before launching
        const R* p = St<R>::noise(a) + (cur * (long long)a.n + i) * 3;
        n0 = p[0];
        n1 = p[1];
        n2 = p[2];
    } else {
        n0 = n1 = n2 = R(0);
    }
}
template <typename R>
__device__ inline void noise3(const ForceArgs& a, const DevCtx* ctx, int i, R& n0, R& n1, R& n2)
{
    noise3_at<R>(a, ctx->step, ctx->noise_cursor, i, n0, n1, n2);
}

// spring-type potential at separation vector r (|r|^2 = r2): returns force coefficient c (F = c r) and U
template <typename R>
__device__ inline R spring_coef(int type, R K, R l, R r2, R& U)
{
    if (type == kHarmonic) {
        U = R(0.5) * K * r2;
        return -K;
    }
    R d = r_sqrt(r2);
    if ((type == kSemispring && d <= l) || d <= R(0)) {
        U = (type == kSpring && d <= R(0)) ? R(0.5) * K * l * l : R(0);
        return R(0);
    }
    R dl = d - l;
    U = R(0.5) * K * dl * dl;
    return -K * dl / d;
}

// ----------------------------------------------------------------------------------------------------
// force / step kernel

// Particle-local terms of particle i at (xi, yi, zi): bonded CSR (chain/loop/nucleolar bonds, droplet),
// cosine bending, kinetochore fibers, point sources and the ellipsoid walls (+ their reactions), in precision R.
// BB: bonded entries whose loads are issued together (a row of the CSR is a chain of dependent loads per entry
// otherwise: the nucleolar particles' ~20 droplet and bond partners made it the longest path of a step)
// A lane's constants of the particle-local terms, loaded once per launch by k_pstep (whose lanes keep their particle
// and share for a whole launch): its first bonded entry, its bending triple's eps, its tether row and first tether
template <typename R>
struct LocalPre {
    int2 enb;      // the first bonded entry of the lane's share (its CSR index: erange.x + lq)
    real4<R> bv;
    R beps;        // bend eps of the triple that starts at i - lq (lq < 3)
    int tb, te;    // the particle's tether row
    TetherT<R> tt; // its entry tb + lq
};
template <int MODE, int BB = 1, typename R = float, bool PL = false>
__device__ inline void local_terms(const DevCtx* __restrict__ ctx, const ForceArgs& a, int i, R xi, R yi, R zi,
                                   real4<R> km, R& fx, R& fy, R& fz, R* en, R* rin, R* rout,
                                   int2 erange = make_int2(-1, -1), const real4<R>* posv = nullptr, int lq = 0,
                                   int nq = 1, const LocalPre<R>* pre = nullptr)
{
    static_assert(!PL || BB == 1, "the preloaded first entry assumes one bonded entry per batch");
    // lq / nq: this lane's share when nq lanes hold the same particle (k_pstep): bonded entries, droplet targets,
    // bending roles and tethers strided over them, the point sources and walls on lq == 0; the caller sums the lanes
    const int n = a.n;
    const FieldPrm<R>& P = St<R>::prm(a);
    // the step-start positions of the partners: the context's buffer, or posv (PL: k_pstep's LDS image, selected
    // statically so the compiler sees the LDS pointer and reads it with ds_read, not with flat loads that also count
    // against vmcnt)
    // (not PL: posv = the slot-order positions when the partners are slot-indexed, a.bslot / a.swslot)
    const real4<R>* __restrict__ posc = (PL || posv) ? posv : St<R>::pos(a, ctx->parity);
    const int* __restrict__ bsl = PL ? nullptr : a.bslot;
    const R cs = (R)ctx->cs;
    const R bs = (R)ctx->bs;
    R e_sw = 0, e_bond = 0, e_bend = 0, e_win = 0, e_wout = 0, e_pt = 0, e_kf = 0;
    if (a.has_bonds) {
        // erange: the particle's CSR row when the caller already has it (the list step's slot-ordered copy)
        const int eb = erange.x >= 0 ? erange.x : a.boff[i], ee = erange.x >= 0 ? erange.y : a.boff[i + 1];
        const real4<R>* __restrict__ bval = St<R>::bval(a);
        auto bond = [&](const int2 e, const real4<R>& bv, const real4<R>& pj) {
            const int type = e.y & 15;
            const R rx = xi - pj.x, ry = yi - pj.y, rz = zi - pj.z;
            const R r2 = r_fma(rz, rz, r_fma(ry, ry, rx * rx));
            R c = 0, U = 0;
            if (type == kSoftwell) {
                if (r2 < bv.z) {
                    const R u6 = r2 * bv.y;
                    const R den = R(1) + u6 * u6 * u6;
                    c = R(-6) * bv.x * u6 * u6 * bv.y / (den * den);
                    e_sw += R(-0.5) * bv.x / den;
                }
            } else {
                R K = bv.x, l = bv.y;
                if (e.y >> 4) {  // scaled by the bond scale
                    K = K * (R(1) / (bs * bs));
                    l = l * bs;
                }
                c = spring_coef<R>(type, K, l, r2, U);
                e_bond += R(0.5) * U;
            }
            fx = r_fma(c, rx, fx);
            fy = r_fma(c, ry, fy);
            fz = r_fma(c, rz, fz);
        };
        int q0 = eb + lq * BB;
        if constexpr (PL) {  // the lane's first entry from the launch's preload
            if (q0 < ee) bond(pre->enb, pre->bv, posc[pre->enb.x]);
            q0 += nq;
        }
        for (; q0 < ee; q0 += nq * BB) {
          int2 enb[BB];
          real4<R> bvb[BB], pjb[BB];
#pragma unroll
          for (int u = 0; u < BB; ++u) {
              // (a batch's padding entries gather particle 0, never used: not `i`, which a lane that integrates
              // nothing may hold unchecked -- a decomposed ghost's stale record)
              enb[u] = (q0 + u < ee) ? a.bent[q0 + u] : make_int2(0, kSemispring);
              bvb[u] = (q0 + u < ee) ? bval[q0 + u] : mk4<R>(R(0), R(0), R(0), R(0));
          }
#pragma unroll
          for (int u = 0; u < BB; ++u) pjb[u] = posc[bsl ? ((q0 + u < ee) ? bsl[q0 + u] : 0) : enb[u].x];
#pragma unroll
          for (int u = 0; u < BB; ++u) {
            if (q0 + u >= ee) break;
            bond(enb[u], bvb[u], pjb[u]);
          }
        }
    }

    if (a.sw_n > 0) {
        // the droplet (simulation_driver_forcefield.cpp:164-185: softwell among the nucleolar targets, cut off at
        // apply_cutoff): every target interacts with every other; a wave holding a target loads all targets' positions
        // once (lane t: target t) and walks them by shuffles, in target order.  With nq lanes per particle lane lq
        // takes targets lq, lq + nq, ...; every lane runs the same trip count, so each shuffle's source lane is still
        // in the loop (lanes leaving after different counts read targets from lanes that had left)
        const bool tgt = km.w != R(0);
        if (__ballot(tgt)) {
            const int m = a.sw_n;
            const int jt = (__lane_id() < m) ? a.sw_idx[__lane_id()] : 0;
            const real4<R> pt = posc[(!PL && a.swslot) ? ((__lane_id() < m) ? a.swslot[__lane_id()] : 0) : jt];
            for (int t0 = 0; t0 < m; t0 += nq) {
                const int t = min(t0 + lq, 63);
                const int j = __shfl(jt, t);
                const R px = __shfl(pt.x, t), py = __shfl(pt.y, t), pz = __shfl(pt.z, t);
                const R rx = xi - px, ry = yi - py, rz = zi - pz;
                const R r2 = r_fma(rz, rz, r_fma(ry, ry, rx * rx));
                if (tgt && t0 + lq < m && j != i && r2 < P.sw_la) {
                    const R u6 = r2 * P.sw_kb;
                    const R den = R(1) + u6 * u6 * u6;
                    const R c = R(-6) * P.sw_ka * u6 * u6 * P.sw_kb / (den * den);
                    e_sw += R(-0.5) * P.sw_ka / den;
                    fx = r_fma(c, rx, fx);
                    fy = r_fma(c, ry, fy);
                    fz = r_fma(c, rz, fz);
                }
            }
        }
    }

    if (a.has_bend) {
        const R* __restrict__ bend = St<R>::bend(a);
        for (int role = lq; role < 3; role += nq) {
            const int k0 = i - role;
            if (k0 < 0 || k0 + 2 >= n) continue;
            const R eps = (PL && role == lq) ? pre->beps : bend[k0];
            if (eps == R(0)) continue;
            real4<R> q0 = (role == 0) ? mk4<R>(xi, yi, zi, R(0)) : posc[k0];
            real4<R> q1 = (role == 1) ? mk4<R>(xi, yi, zi, R(0)) : posc[k0 + 1];
            real4<R> q2 = (role == 2) ? mk4<R>(xi, yi, zi, R(0)) : posc[k0 + 2];
            const R r1x = q1.x - q0.x, r1y = q1.y - q0.y, r1z = q1.z - q0.z;
            const R r2x = q2.x - q1.x, r2y = q2.y - q1.y, r2z = q2.z - q1.z;
            const R n1 = r1x * r1x + r1y * r1y + r1z * r1z;
            const R n2 = r2x * r2x + r2y * r2y + r2z * r2z;
            if (!(n1 > R(0)) || !(n2 > R(0))) continue;
            const R inv12 = r_rsqrt(n1 * n2);
            const R cv = (r1x * r2x + r1y * r2y + r1z * r2z) * inv12;
            const R i1 = cv / n1, i2 = cv / n2;
            const R d1x = r2x * inv12 - i1 * r1x, d1y = r2y * inv12 - i1 * r1y, d1z = r2z * inv12 - i1 * r1z;
            const R d2x = r1x * inv12 - i2 * r2x, d2y = r1y * inv12 - i2 * r2y, d2z = r1z * inv12 - i2 * r2z;
            if (role == 0) {
                fx -= eps * d1x; fy -= eps * d1y; fz -= eps * d1z;
                e_bend += eps * (R(1) - cv);
            } else if (role == 2) {
                fx += eps * d2x; fy += eps * d2y; fz += eps * d2z;
            } else {
                fx += eps * (d1x - d2x); fy += eps * (d1y - d2y); fz += eps * (d1z - d2z);
            }
        }
    }

    if (a.has_tether) {
        const int tb = PL ? pre->tb : a.toff[i], te = PL ? pre->te : a.toff[i + 1];
        const TetherT<R>* __restrict__ tent = St<R>::tent(a);
        for (int q = tb + lq; q < te; q += nq) {
            const TetherT<R> t = (PL && q == tb + lq) ? pre->tt : tent[q];
            const R rx = xi - t.px, ry = yi - t.py, rz = zi - t.pz;
            R U;
            const R c = spring_coef<R>(kSpring, t.k, t.l, rx * rx + ry * ry + rz * rz, U);
            e_kf += U;
            fx = r_fma(c, rx, fx);
            fy = r_fma(c, ry, fy);
            fz = r_fma(c, rz, fz);
        }
    }

#pragma unroll
    for (int q = 0; q < kMaxPointSources; ++q) {
        if (q >= a.n_point || lq != 0) break;
        PointSrcT<R> p = P.point[q];
        // opaque to the optimizer: keeps the (rarely used, mitotic-only) point-source constants from being hoisted
        // to the kernel entry, where they would be spilled to scratch by every wave
        asm volatile("" : "+v"(p.b), "+v"(p.f), "+v"(p.k), "+v"(p.l));
        const R rx = xi - p.px, ry = yi - p.py, rz = zi - p.pz;
        const R r2 = rx * rx + ry * ry + rz * rz;
        R c, U;
        if (p.type == GCS_POT_FORCE_FLUX) {
            // common/potentials/force_flux_potential.hpp:24-37
            const R r1 = r_sqrt(r2), b2 = p.b * p.b;
            c = (r1 > R(0)) ? p.f * b2 / (b2 * r1 + r1 * r2) : R(0);
            U = p.f * p.b * r_atan2(p.b, r1);
        } else {
            c = spring_coef<R>(p.type == GCS_POT_SEMISPRING ? kSemispring : (p.type == GCS_POT_HARMONIC ? kHarmonic : kSpring),
                               p.k, p.l, r2, U);
        }
        e_pt += U;
        fx = r_fma(c, rx, fx);
        fy = r_fma(c, ry, fy);
        fz = r_fma(c, rz, fz);
    }

    if ((a.has_wall_in || a.has_wall_out) && lq == 0) {
        // Sampson distance to the ellipsoid (DESIGN.md "ellipsoid wall"): rho = |r o 1/ax|,
        // g = r o 1/ax^2, d = |1 - rho| rho / |g|, normal n = g / |g|
        const R ax = (R)ctx->wall[0], ay = (R)ctx->wall[1], az = (R)ctx->wall[2];
        const R cx = a.has_wall_in ? P.win.cx : P.wout_cx;
        const R cy = a.has_wall_in ? P.win.cy : P.wout_cy;
        const R cz = a.has_wall_in ? P.win.cz : P.wout_cz;
        const R rx = xi - cx, ry = yi - cy, rz = zi - cz;
        const R qx = rx / ax, qy = ry / ay, qz = rz / az;
        const R gx = qx / ax, gy = qy / ay, gz = qz / az;
        const R g2 = gx * gx + gy * gy + gz * gz;
        if (g2 > R(0)) {
            const R rho = r_sqrt(qx * qx + qy * qy + qz * qz);
            const R ginv = r_rsqrt(g2);
            const R d = r_fabs(R(1) - rho) * rho * ginv;
            const R nx_ = gx * ginv, ny_ = gy * ginv, nz_ = gz * ginv;
            if (a.has_wall_in && rho < R(1)) {
                const WallInT<R>& w = P.win;
                const R sc = w.scaled ? cs : R(1);
                const R A = w.mix ? R(0.5) * (km.y + w.wall_a) : R(1);
                const R B = w.mix ? R(0.5) * (km.z + w.wall_b) : R(0);
                const R d2 = d * d;
                const R sa = w.a_sig * sc, sbw = w.b_sig * sc;
                const R k2a = R(1) / (sa * sa), k2b = R(1) / (sbw * sbw);
                const R ua = d2 * k2a, t = d2 * k2b;
                R coef = 0, U = 0;
                if (ua < R(1)) {
                    const R ga = R(1) - ua;
                    coef += A * R(6) * w.a_eps * k2a * ga * ga;
                    U += A * w.a_eps * ga * ga * ga;
                }
                if (t < R(1) && B != R(0)) {
                    const R t2 = t * t;
                    const R gb = R(1) - t2 * t2;
                    coef += B * R(24) * w.b_eps * k2b * gb * gb * t2 * t;
                    U += B * w.b_eps * gb * gb * gb;
                }
                const R wx = -coef * d * nx_, wy = -coef * d * ny_, wz = -coef * d * nz_;
                fx += wx; fy += wy; fz += wz;
                rin[0] = r_fabs(wx); rin[1] = r_fabs(wy); rin[2] = r_fabs(wz);
                e_win += U;
            }
            if (a.has_wall_out && rho > R(1)) {
                const R wx = -P.wout_k * d * nx_, wy = -P.wout_k * d * ny_, wz = -P.wout_k * d * nz_;
                fx += wx; fy += wy; fz += wz;
                rout[0] = r_fabs(wx); rout[1] = r_fabs(wy); rout[2] = r_fabs(wz);
                e_wout += R(0.5) * P.wout_k * d * d;
            }
        }
    }

    en[1] = e_sw;
    en[2] = e_bond;
    en[3] = e_bend;
    en[4] = e_win;
    en[5] = e_wout;
    en[6] = e_pt;
    en[7] = e_kf;
}

// Gather-form pair forces on the 64 particles of one tile [s_begin, s_end) (one row of cells, lane = particle)
// from this wave's share of the tile's stencil candidates.  Stencil: the 3x3 neighbouring cell rows, x-range
// [x_first - fx, x_last + fx] (x cells are rc / fx wide).  Candidates are staged 64 at a time in LDS
// (software-pipelined), filtered in fp32 into a per-lane 64-bit hit mask, and the soft-core potential is
// evaluated for the hits only.
//
// Tile frame: coordinates are taken relative to the tile's first particle and each staged candidate record is
// {-2x', -2y', -2z', |x'|^2, kA a_j, kB b_j}, so the phase-1 test  |x_j'|^2 - 2 x_i'.x_j' < rc^2 - |x_i'|^2  is
// three fma + compare (|x'| stays within the stencil, so the form is well conditioned: an error ~1e-7 rc^2
// only moves pairs at the cutoff, where the potential and its force vanish), and phase 2 recovers
// x_i - x_j = x_i' + (-2x_j')/2 exactly from the record.  Slot kTile holds a far-away sentinel record: an
// exhausted hit mask points there and contributes exactly zero (no per-hit activity mask).
template <int MODE, int WAVES>
__device__ inline void pair_forces(const DevCtx* __restrict__ ctx, const ForceArgs& a, int wave, int lane, int s,
                                   int s_begin, int s_end, float4 pi, float bi, float& fx, float& fy, float& fz,
                                   float& acc, int* s_rowV, int* s_rowJ, float4* s_cand, int* s_candj, int& ntot,
                                   int wv, int nwv)
{
    const Grid g = ctx->grid;
    const float cs = (float)ctx->cs;
    const float scale = a.pair_scaled ? cs : 1.f;
    const float sa = a.pf.pa_sig * scale, sbb = a.pf.pb_sig * scale;
    const float k2a = 1.f / (sa * sa), k2b = 1.f / (sbb * sbb);
    // F = coef * (x_i - x_j):  A * 6 eps_a k2a ga^2  +  B * 24 eps_b k2b gb^2 t^3   (A, B = pair means)
    // energy: 1/2 (mean) x 1/2 (each pair seen from both ends) x eps (A ga^3 + B gb^3)
    const float kA = (MODE == kModeEnergy) ? 0.25f * a.pf.pa_eps : 0.5f * 6.f * a.pf.pa_eps * k2a;
    const float kB = (MODE == kModeEnergy) ? 0.25f * a.pf.pb_eps : 0.5f * 24.f * a.pf.pb_eps * k2b;
    const float rc2 = g.rc2;
    const int nx = g.n[0], ny = g.n[1], nz = g.n[2], gfx = g.fx;
    const int c0 = uniform(a.scell[s_begin]), c1 = uniform(a.scell[s_end - 1]);
    const int x0 = c0 % nx, x1 = c1 % nx, r0 = c0 / nx;
    const int y0 = r0 % ny, z0 = r0 / ny;
    const int xlo = max(x0 - gfx, 0), xhi = min(x1 + gfx, nx - 1);

    // wave-private row table: lane q < 9 holds stencil row (y0 + q%3 - 1, z0 + q/3 - 1)
    {
        int len = 0, jb = 0;
        if (lane < 9) {
            const int y = y0 + lane % 3 - 1, z = z0 + lane / 3 - 1;
            if (y >= 0 && y < ny && z >= 0 && z < nz) {
                const int base = (z * ny + y) * nx;
                jb = a.cstart[base + xlo];
                len = a.cstart[base + xhi + 1] - jb;
            }
        }
        const int incl = wave_incl_scan(len, lane);
        if (lane < 16) {
            s_rowV[lane] = incl - len;
            s_rowJ[lane] = jb;
        }
        if (lane == 15) s_rowV[16] = incl;
    }
    // tile frame and the sentinel record
    const float ox = uniform_f(pi.x), oy = uniform_f(pi.y), oz = uniform_f(pi.z);
    const float xi = pi.x - ox, yi = pi.y - oy, zi = pi.z - oz;
    const float thr = rc2 - fmaf(zi, zi, fmaf(yi, yi, xi * xi));
    const float far = 1.0e3f * fmaxf(g.rc, 1.f);
    const float4 sent0 = make_float4(-2.f * far, -2.f * far, -2.f * far, 3.f * far * far);
    if (lane == 0) {
        s_cand[2 * kTile] = sent0;
        s_cand[2 * kTile + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __builtin_amdgcn_wave_barrier();
    const int total = uniform(s_rowV[16]);
    ntot = total;
    // Wave priority by tile cost: the kernel ends with its densest tiles (block time ~ 17 us + 17.5 ns per
    // candidate on C2), while light tiles have slack.  The SIMD arbiter issues higher-priority waves first, so
    // the critical tiles progress at the light ones' expense.  (s_setprio takes an immediate.)
    if (a.prio_step > 0) {
        const int pr = total / a.prio_step;
        if (pr >= 3)
            __builtin_amdgcn_s_setprio(3);
        else if (pr == 2)
            __builtin_amdgcn_s_setprio(2);
        else if (pr == 1)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    }
    const float ahi = kA * pi.w, bhi = kB * bi;
    // Chunk c of this wave holds candidates v = first(c) + stride * lane, lane < count(c).
    //   contiguous (chunk_mode 0): the wave's share [wlo, whi) in runs of 64
    //   strided    (chunk_mode 1): chunk g of G = ceil(total / 64) takes v = g + G * lane; wave w owns the
    //   chunks g = w (mod nwv).  Every chunk then samples all stencil rows, which evens the hit counts
    //   across lanes (phase 2 runs as long as the lane with the most hits).
    // (wv, nwv): this wave's index among all the waves sharing the tile (the split parts' waves included)
    const bool strided = a.chunk_mode != 0;
    const int G = (total + kTile - 1) / kTile;
    const int wlo = (int)(((long long)total * wv) / nwv);
    const int whi = (int)(((long long)total * (wv + 1)) / nwv);
    const int nchunk = strided ? (G > wv ? (G - wv + nwv - 1) / nwv : 0) : (whi - wlo + kTile - 1) / kTile;
    const int stride = strided ? G : 1;
    auto first = [&](int c) { return strided ? wv + c * nwv : wlo + c * kTile; };
    auto count = [&](int c) {
        const int f = first(c);
        return strided ? min(kTile, (total - f + G - 1) / G) : min(kTile, whi - f);
    };

    // raw loads only (consumed one chunk later: the loads stay in flight over the current chunk)
    auto fetch = [&](int c, float4& p, float& b, int& jj) {
        const int v = first(c) + stride * lane;
        jj = -1;
        if (lane < count(c)) {
            int lo = 0;  // last stencil row starting at or before v (rows 9..15 start at `total`)
#pragma unroll
            for (int step = 8; step > 0; step >>= 1)
                if (s_rowV[lo + step] <= v) lo += step;
            jj = s_rowJ[lo] + (v - s_rowV[lo]);
            p = a.spos[jj];
            b = a.sb[jj];
        }
    };
    // two chunks in flight: the load latency (an L2 miss under load is microseconds) outlasts one chunk's work
    float4 npj, npj2;
    float nbj, nbj2;
    int njj, njj2 = -1;
    if (nchunk > 0) fetch(0, npj, nbj, njj);
    if (nchunk > 1) fetch(1, npj2, nbj2, njj2);
    for (int c = 0; c < nchunk; ++c) {
        const int cnt = uniform(count(c));
        const int cnt8 = (cnt + 7) & ~7;  // sentinel-padded to a multiple of 8
        {
            const bool real = njj >= 0;
            const float px = real ? npj.x - ox : far, py = real ? npj.y - oy : far, pz = real ? npj.z - oz : far;
            s_cand[2 * lane] = make_float4(-2.f * px, -2.f * py, -2.f * pz, fmaf(pz, pz, fmaf(py, py, px * px)));
            s_cand[2 * lane + 1] = make_float4(real ? kA * npj.w : 0.f, real ? kB * nbj : 0.f, 0.f, 0.f);
            if (MODE == kModeEnergy) s_candj[lane] = njj;
        }
        __builtin_amdgcn_wave_barrier();
        npj = npj2;
        nbj = nbj2;
        njj = njj2;
        if (c + 2 < nchunk) fetch(c + 2, npj2, nbj2, njj2);  // two chunks ahead

        // phase 1: one fma chain + compare per candidate; each lane keeps a 64-bit mask of its hits.  Within a
        // group of 8 candidates the mask byte is built as byte = 2 byte + hit (v_cmp + v_addc), so candidate
        // k0 + u lands on bit k0 + 7 - u (decoded by k = bit ^ 7).
        unsigned mlo = 0u, mhi = 0u;
        for (int k0 = 0; k0 < cnt8; k0 += 8) {
            unsigned byte = 0u;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float4 q = s_cand[2 * (k0 + u)];
                const float t = fmaf(q.x, xi, fmaf(q.y, yi, fmaf(q.z, zi, q.w)));
                if (MODE == kModeEnergy) {
                    const bool in = (t < thr) && (s_candj[k0 + u] != s);
                    byte = 2u * byte + (in ? 1u : 0u);
                } else {
                    // the self pair contributes exactly zero force (F is proportional to x_i - x_j), so the force
                    // path keeps it (one wasted slot) instead of paying a second compare per candidate
                    asm("v_cmp_gt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                        : "+v"(byte)
                        : "v"(thr), "v"(t)
                        : "vcc");
                }
            }
            if (k0 < 32)
                mlo |= byte << k0;
            else
                mhi |= byte << (k0 - 32);
        }
        if (MODE != kModeEnergy) acc += (float)(__popc(mlo) + __popc(mhi));
        // phase 2: the potential on the hits only, one 32-bit half of the mask after the other (iterations =
        // the wave's largest hit count in that half), four independent hits per iteration so their LDS reads
        // overlap.  Pop = ffbl, xor, min (exhausted -> the sentinel slot), clear lowest bit.
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            unsigned m = h ? mhi : mlo;
            const float4* base = s_cand + 2 * (h ? 32 : 0);
            const unsigned lim = h ? 32u : 64u;
            const int mh = uniform(wave_max_int(__popc(m)));
            for (int t = 0; t < mh; t += 4) {
                unsigned kk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    unsigned b;
                    asm("v_ffbl_b32 %0, %1" : "=v"(b) : "v"(m));  // 0xffffffff when m == 0
                    kk[u] = min(b ^ 7u, lim);
                    m &= m - 1u;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4 q = base[2 * kk[u]];
                    const float4 w = base[2 * kk[u] + 1];
                    const float dx = fmaf(0.5f, q.x, xi), dy = fmaf(0.5f, q.y, yi), dz = fmaf(0.5f, q.z, zi);
                    const float r2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                    const float ga = fmaxf(fmaf(-k2a, r2, 1.f), 0.f);
                    const float tt = r2 * k2b;
                    const float t2 = tt * tt;
                    const float gb = fmaxf(fmaf(-t2, t2, 1.f), 0.f);
                    const float A = ahi + w.x, B = bhi + w.y;
                    if (MODE == kModeEnergy) {
                        acc += fmaf(A, ga * ga * ga, B * (gb * gb * gb));
                    } else {
                        const float coef = fmaf(A, ga * ga, B * (gb * gb * t2 * tt));
                        fx = fmaf(coef, dx, fx);
                        fy = fmaf(coef, dy, fy);
                        fz = fmaf(coef, dz, fz);
                    }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Sub-tile pair forces (a.subtiles = NG > 1): the tile's 64 lanes form NG groups of GL = 64 / NG consecutive
// particles, each with its OWN stencil x-range (the cells of its first and last particle +-fx) and its own
// candidate stream.  At the realistic interphase density a 64-particle tile spans ~10 rc of its cell row, so a
// lane's share of the tile-wide union stencil is mostly candidates far beyond its cutoff (hit rate ~5 %); per
// group of 16 the union shrinks ~2.5x.  Chunks are 32 candidates per group (one 32-bit hit mask per lane), staged
// with FPL = 32 / GL loads per lane; phase-1 LDS reads then carry NG addresses (one broadcast per group, the groups
// on disjoint banks).  Same phase-1 test, frame (per-group origin) and phase 2 as pair_forces.
#ifndef GCS_P2_UNROLL
#define GCS_P2_UNROLL 4  // sub-tile phase 2: hits popped per lane per round (rounds = wave max of hits / this)
#endif
// Neighbour-list layout (the list step): per wave segment w of a slot s, its entries packed by 8-byte words of
// E = 8 / sizeof(LE) consecutive entries (4 16-bit or 2 32-bit slot indices), the words column-major over the slots:
// entry k of (w, s) is element E ((w cap / E + k / E) stride + s) + k % E.  A wave loads E entries of each of its 64
// slots with one 8-B load per lane (512 contiguous bytes), so a batch of 8 entries is 2 (16-bit) or 4 loads.
template <typename LE>
__device__ __forceinline__ size_t list_at(int w, int cap, int k, int s, size_t stride)
{
    constexpr int E = 8 / (int)sizeof(LE);
    return (((size_t)w * (size_t)(cap / E) + (size_t)(k / E)) * stride + (size_t)s) * E + (size_t)(k % E);
}
// ListRel16 (ForceArgs::list_fmt kListFmtRel16, the default beyond 65,536 particles): 16-bit entries p << 14 | u
// relative to the slot's plane bases lbase[s] = {b0, b1, b2}: the partner's slot is b_p + u.  p = 0, 1, 2 is the
// partner's z plane (the slot's build cell z - 1, z, z + 1) and b_p the first slot of cell (x - fx, y - 1) in that
// plane: a partner lies in the plane's rows y - 1 .. y + 1 and cells x - fx .. x + fx, so u spans at most two cell rows
// plus 2 fx + 1 cells -- below 2^14 slots even at C5's densest start (11,231: profiles/r04_c5_plane_spans.txt).  A
// partner outside [b_p, b_p + 2^14) marks the list overflowed (exact search).  Absolute slots would need 32 bits past
// 2^16 particles; an offset from the slot's own index would span a whole z layer of cells (tens of thousands).
struct ListRel16 {
    unsigned short v;
};
template <typename LE>
struct ListFmt {
    static constexpr bool rel = false;
};
template <>
struct ListFmt<ListRel16> {
    static constexpr bool rel = true;
};
constexpr int kRelBits = 14;
// the partner slot of a list entry (x: its raw bits)
template <typename LE>
__device__ __forceinline__ int list_slot(int x, int4 lb)
{
    if constexpr (ListFmt<LE>::rel) {
        const int p = x >> kRelBits;
        return (p == 0 ? lb.x : (p == 1 ? lb.y : lb.z)) + (x & ((1 << kRelBits) - 1));
    } else {
        (void)lb;
        return x;
    }
}
// entry u of a batch held as 8-byte words
template <typename LE>
__device__ __forceinline__ int list_entry(const uint2* w, int u)
{
    if constexpr (sizeof(LE) == 2) {
        const unsigned x = (u & 2) ? w[u >> 2].y : w[u >> 2].x;
        return (int)((u & 1) ? (x >> 16) : (x & 0xffffu));
    } else {
        return (int)((u & 1) ? w[u >> 1].y : w[u >> 1].x);
    }
}

// The list build's deal of candidate chunks to the waves (GCS_OPT_LIST_DEAL): chunk p of every period of T = d >> 60
// chunks goes to wave nibble p of d (0 < T <= 15; d = 0: round robin over the waves).  The wave's entries form its list
// segment, and the list step's last wave also carries the particle-local terms: a pattern that deals that wave fewer
// chunks evens the step's waves out.  Any pattern covers every chunk exactly once, in increasing order per wave, so
// the union of a slot's segments (the pair set) does not depend on it.  Scalar arithmetic (every operand uniform).
__device__ __forceinline__ int deal_wave(unsigned long long d, int p)
{
    return (int)((d >> (4 * p)) & 15ull);
}
__device__ __forceinline__ int deal_count(unsigned long long d, int T, int w, int upto)
{
    int k = 0;
    for (int p = 0; p < upto && p < T; ++p) k += deal_wave(d, p) == w ? 1 : 0;
    return k;
}
// the c-th chunk of wave w (kw = its chunks per period, > 0)
__device__ __forceinline__ int deal_nth(unsigned long long d, int T, int kw, int w, int c)
{
    int r = c % kw, p = 0;
    for (; p < T; ++p)
        if (deal_wave(d, p) == w && r-- == 0) break;
    return (c / kw) * T + p;
}

template <int MODE, int NG, typename LE = int>
__device__ inline void pair_forces_sub(const DevCtx* __restrict__ ctx, const ForceArgs& a, int lane, int s,
                                       int s_begin, int s_end, float4 pi, float bi, float& fx, float& fy, float& fz,
                                       float& acc, int* s_rowV, int* s_rowJ, float4* s_cand, int* s_candj, int& ntot,
                                       int wv, int nwv, int self = -1, bool lvalid = false, int* lcnt = nullptr,
                                       unsigned long long* lpend = nullptr, int4* plb = nullptr)
{
    // kModeList: phase 2 appends each hit (other than the particle itself) to the lane's list segment wv
    // instead of evaluating the pair force (the lists of the list step, built at the grid's rc = cutoff + skin)
    constexpr int GL = kTile / NG;  // lanes (particles) per group
    constexpr int kSub = 32;        // candidates per group chunk
    constexpr int FPL = kSub / GL;  // candidate fetches per lane per chunk
    constexpr int kRec = 2 * (kSub + 1);  // float4 per group staging area (records + sentinel)
    constexpr int kP2 = GCS_P2_UNROLL;
    static_assert(NG >= 2 && NG <= 8 && FPL >= 1, "2, 4 or 8 groups");
    const Grid g = ctx->grid;
    const float cs = (float)ctx->cs;
    const float scale = a.pair_scaled ? cs : 1.f;
    const float sa = a.pf.pa_sig * scale, sbb = a.pf.pb_sig * scale;
    const float k2a = 1.f / (sa * sa), k2b = 1.f / (sbb * sbb);
    const float kA = (MODE == kModeEnergy) ? 0.25f * a.pf.pa_eps : 0.5f * 6.f * a.pf.pa_eps * k2a;
    const float kB = (MODE == kModeEnergy) ? 0.25f * a.pf.pb_eps : 0.5f * 24.f * a.pf.pb_eps * k2b;
    const float rc2 = g.rc2;
    const int nx = g.n[0], ny = g.n[1], nz = g.n[2], gfx = g.fx;
    const int grp = lane / GL, gl = lane % GL;

    // row tables: lane (h, q) = (lane / 9, lane % 9) < 9 NG builds group h's stencil row q; groups are segments of
    // one wave scan (offset = scan - group base)
    {
        const int h = lane / 9, q = lane % 9;
        int len = 0, jb = 0;
        const int r0 = uniform(a.scell[s_begin]) / nx;  // the tile's cell row (all groups share it)
        const int y0 = r0 % ny, z0 = r0 / ny;
        if (h < NG) {
            const int hb = s_begin + h * GL, he = min(s_end, hb + GL);
            if (hb < he) {
                const int x0 = a.scell[hb] % nx, x1 = a.scell[he - 1] % nx;
                const int xlo = max(x0 - gfx, 0), xhi = min(x1 + gfx, nx - 1);
                const int y = y0 + q % 3 - 1, z = z0 + q / 3 - 1;
                if (y >= 0 && y < ny && z >= 0 && z < nz) {
                    const int base = (z * ny + y) * nx;
                    jb = a.cstart[base + xlo];
                    len = a.cstart[base + xhi + 1] - jb;
                }
            }
        }
        if constexpr (MODE == kModeList && ListFmt<LE>::rel) {
            // this lane's plane bases (ListRel16): first slot of cell (x - fx, y - 1) in planes z - 1, z, z + 1
            const int cx = a.scell[min(s, s_end - 1)] % nx;
            const int xb = max(cx - gfx, 0), yb = max(y0 - 1, 0);
            int b[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const int z = z0 + p - 1;
                b[p] = (z >= 0 && z < nz) ? a.cstart[(z * ny + yb) * nx + xb] : 0;
            }
            *plb = make_int4(b[0], b[1], b[2], 0);
        }
        int incl = len;
        GCS_DPP_SCAN(dpp_i, add_i, 0, incl)
        const int gbase = __shfl(incl, max(9 * h - 1, 0));
        const int off = incl - len - (h > 0 ? gbase : 0);
        if (h < NG) {
            s_rowV[h * 17 + q] = off;
            s_rowJ[h * 16 + q] = jb;
            if (q == 8)
                for (int t = 9; t < 17; ++t) s_rowV[h * 17 + t] = off + len;  // rows 9.. start at the group total
        }
    }
    // per-group frame origin: the group's first particle (the tile's first for empty trailing groups)
    const int olane = (s_begin + grp * GL < s_end) ? grp * GL : 0;
    const float ox = __shfl(pi.x, olane), oy = __shfl(pi.y, olane), oz = __shfl(pi.z, olane);
    const float xi = pi.x - ox, yi = pi.y - oy, zi = pi.z - oz;
    const float thr = rc2 - fmaf(zi, zi, fmaf(yi, yi, xi * xi));
    const float far = 1.0e3f * fmaxf(g.rc, 1.f);
    float4* const my_cand = s_cand + grp * kRec;
    if (gl == 0) {
        my_cand[2 * kSub] = make_float4(-2.f * far, -2.f * far, -2.f * far, 3.f * far * far);
        my_cand[2 * kSub + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __builtin_amdgcn_wave_barrier();
    const int* const rowV = s_rowV + grp * 17;
    const int* const rowJ = s_rowJ + grp * 16;
    const int total = rowV[16];  // my group's candidates
    ntot = uniform(wave_max_int(total));
    const float ahi = kA * pi.w, bhi = kB * bi;
    const int G = (total + kSub - 1) / kSub;   // my group's chunks; chunk c takes v = c + G * i
    const int Gmax = uniform(wave_max_int(G));
    // kModeList: the chunks of a deal pattern (deal_nth), otherwise wave wv takes chunks wv, wv + nwv, ...
    const unsigned long long deal = MODE == kModeList ? a.list_deal : 0ull;
    const int dT = (int)(deal >> 60);
    const int dkw = deal ? deal_count(deal, dT, wv, dT) : 0;
    const int nchunk = deal ? (dkw ? (Gmax / dT) * dkw + deal_count(deal, dT, wv, Gmax % dT) : 0)
                            : (Gmax > wv ? (Gmax - wv + nwv - 1) / nwv : 0);

    float4 np[FPL];
    float nb[FPL];
    int nj[FPL], npl[FPL];
    auto fetch = [&](int c) {
        const int cg = deal ? deal_nth(deal, dT, dkw, wv, c) : wv + c * nwv;  // chunk index within every group
#pragma unroll
        for (int f = 0; f < FPL; ++f) {
            const int i = gl + GL * f;  // slot
            const int v = cg + G * i;
            nj[f] = -1;
            if (cg < G && v < total) {
                int lo = 0;  // the stencil row of candidate v: a 4-level binary search of the row starts
#pragma unroll
                for (int step = 8; step > 0; step >>= 1)
                    if (rowV[lo + step] <= v) lo += step;
                nj[f] = rowJ[lo] + (v - rowV[lo]);
                // ListRel16: the stencil row's z plane (rows q = 0..8: z = z0 + q / 3 - 1)
                npl[f] = lo / 3;
                np[f] = a.spos[nj[f]];
                nb[f] = a.sb[nj[f]];
            }
        }
    };
    if (nchunk > 0) fetch(0);
    for (int c = 0; c < nchunk; ++c) {
#pragma unroll
        for (int f = 0; f < FPL; ++f) {
            const int i = gl + GL * f;
            const bool real = nj[f] >= 0;
            const float px = real ? np[f].x - ox : far, py = real ? np[f].y - oy : far, pz = real ? np[f].z - oz : far;
            if constexpr (MODE == kModeList) {
                // pair layout: candidates 2h, 2h+1 in float4s 2h {x, x', y, y'} and 2h+1 {z, z', w, w'}; slots at
                // float 8 * kSub / 2 (the list build's phase 2 needs only the partner's slot)
                float* const P = reinterpret_cast<float*>(my_cand);
                const int h8 = 8 * (i >> 1) + (i & 1);
                P[h8] = -2.f * px;
                P[h8 + 2] = -2.f * py;
                P[h8 + 4] = -2.f * pz;
                P[h8 + 6] = fmaf(pz, pz, fmaf(py, py, px * px));
                // the partner's slot (< 2^24) and, for ListRel16, its plane in bits 28..29
                reinterpret_cast<int*>(my_cand)[4 * kSub + i] =
                    real ? (ListFmt<LE>::rel ? (nj[f] | (npl[f] << 28)) : nj[f]) : -1;
                continue;
            }
            my_cand[2 * i] = make_float4(-2.f * px, -2.f * py, -2.f * pz, fmaf(pz, pz, fmaf(py, py, px * px)));
            my_cand[2 * i + 1] = make_float4(real ? kA * np[f].w : 0.f, real ? kB * nb[f] : 0.f, 0.f, 0.f);
            if (MODE == kModeEnergy) s_candj[grp * kSub + i] = nj[f];
        }
        __builtin_amdgcn_wave_barrier();
        if (c + 1 < nchunk) fetch(c + 1);  // next chunk in flight

        // phase 1: 32 candidates of my group -> one 32-bit hit mask (byte trick: candidate k on bit k ^ 7)
        unsigned m = 0u;
        if constexpr (MODE == kModeList) {
            // the same fma chain per candidate, two candidates per packed instruction (v_pk_fma_f32); hit = sign of
            // tv - thr (tv < thr exactly: a difference of unequal finite floats is never +0), shifted in by
            // v_alignbit: 3 VALU per candidate instead of 5, the same bits in the same places
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 X = {xi, xi}, Y = {yi, yi}, Z = {zi, zi}, T = {thr, thr};
#pragma unroll
            for (int k0 = 0; k0 < kSub; k0 += 8) {
                f2 tv[4];
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const float4 A = my_cand[k0 + 2 * h], B = my_cand[k0 + 2 * h + 1];
                    const f2 qx = {A.x, A.y}, qy = {A.z, A.w}, qz = {B.x, B.y}, qw = {B.z, B.w};
                    tv[h] = __builtin_elementwise_fma(qx, X, __builtin_elementwise_fma(qy, Y,
                                                      __builtin_elementwise_fma(qz, Z, qw)));
                }
                unsigned byte = 0u;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const f2 d = tv[h] - T;
                    byte = __builtin_amdgcn_alignbit(byte, __float_as_uint(d.x), 31u);
                    byte = __builtin_amdgcn_alignbit(byte, __float_as_uint(d.y), 31u);
                }
                m |= byte << k0;
            }
        } else
#pragma unroll
        for (int k0 = 0; k0 < kSub; k0 += 8) {
            unsigned byte = 0u;
            // the 8 distance tests first, the compare chain after: the inline asm below is a scheduling barrier,
            // so interleaving it with the LDS reads would serialise every read on its own lgkmcnt(0)
            float tv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float4 q = my_cand[2 * (k0 + u)];
                tv[u] = fmaf(q.x, xi, fmaf(q.y, yi, fmaf(q.z, zi, q.w)));
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (MODE == kModeEnergy) {
                    const bool in = (tv[u] < thr) && (s_candj[grp * kSub + k0 + u] != s);
                    byte = 2u * byte + (in ? 1u : 0u);
                } else {
                    asm("v_cmp_gt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                        : "+v"(byte)
                        : "v"(thr), "v"(tv[u])
                        : "vcc");
                }
            }
            m |= byte << k0;
        }
        if (MODE != kModeEnergy) acc += (float)__popc(m);
        // phase 2: pop ffbl, xor, min (exhausted -> the group's sentinel slot), clear
        const int mh = uniform(wave_max_int(__popc(m)));
        if constexpr (MODE == kModeList) {
            // append the hits: entries shift into the lane's pending 8-byte word (lpend: the newest in the top
            // bits), stored whole when full (list_at's layout: lanes of a wave write consecutive words of a row);
            // the caller stores the last, partial word
            constexpr int E = 8 / (int)sizeof(LE);
            constexpr int EB = 8 * (int)sizeof(LE);  // bits per entry
            unsigned long long* const lw = reinterpret_cast<unsigned long long*>(a.list);
            for (int t = 0; t < mh; ++t) {
                unsigned b;
                asm("v_ffbl_b32 %0, %1" : "=v"(b) : "v"(m));
                const unsigned k = min(b ^ 7u, (unsigned)kSub);
                m &= m - 1u;
                if (k < (unsigned)kSub && lvalid) {
                    const int er = reinterpret_cast<const int*>(my_cand)[4 * kSub + k];
                    const int e = er & 0x0fffffff;  // the partner's sorted slot
                    if (e != s) {
                        const int kk = *lcnt;
                        unsigned code = (unsigned)e;
                        bool fits = true;
                        if constexpr (ListFmt<LE>::rel) {
                            const int p = er >> 28;
                            const int u = e - (p == 0 ? plb->x : (p == 1 ? plb->y : plb->z));
                            fits = (unsigned)u < (1u << kRelBits);
                            code = ((unsigned)p << kRelBits) | (unsigned)u;
                        }
                        if (kk < a.list_cap && fits) {
                            *lpend = (*lpend >> EB) | ((unsigned long long)code << (64 - EB));
                            if (kk % E == E - 1)
                                lw[((size_t)wv * (a.list_cap / E) + kk / E) * a.list_stride + s] = *lpend;
                        }
                        *lcnt = fits ? kk + 1 : max(kk + 1, a.list_cap + 1);  // out of range: overflowed
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        for (int t = 0; t < mh; t += kP2) {
            unsigned kk[kP2];
#pragma unroll
            for (int u = 0; u < kP2; ++u) {
                unsigned b;
                asm("v_ffbl_b32 %0, %1" : "=v"(b) : "v"(m));
                kk[u] = min(b ^ 7u, (unsigned)kSub);
                m &= m - 1u;
            }
#pragma unroll
            for (int u = 0; u < kP2; ++u) {
                const float4 q = my_cand[2 * kk[u]];
                const float4 w = my_cand[2 * kk[u] + 1];
                const float dx = fmaf(0.5f, q.x, xi), dy = fmaf(0.5f, q.y, yi), dz = fmaf(0.5f, q.z, zi);
                const float r2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                const float ga = fmaxf(fmaf(-k2a, r2, 1.f), 0.f);
                const float tt = r2 * k2b;
                const float t2 = tt * tt;
                const float gb = fmaxf(fmaf(-t2, t2, 1.f), 0.f);
                const float A = ahi + w.x, B = bhi + w.y;
                if (MODE == kModeEnergy) {
                    acc += fmaf(A, ga * ga * ga, B * (gb * gb * gb));
                } else {
                    const float coef = fmaf(A, ga * ga, B * (gb * gb * t2 * tt));
                    fx = fmaf(coef, dx, fx);
                    fy = fmaf(coef, dy, fy);
                    fz = fmaf(coef, dz, fz);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// One launch = one force evaluation (+ the Euler-Maruyama update in kModeStep).  Blocks walk the tiles of the
// current cell list (grid-stride); a tile is <= 64 consecutive sorted particles of ONE row of cells
// (k_cell_scan builds the per-row tile prefix).  The WAVES waves split the tile's candidates; wave 0 then
// adds the particle-local terms and integrates.  Per-block partials (reactions, bbox, drift, neighbours,
// energies) are reduced in a fixed order by k_tail / the host: no atomics, bitwise reproducible.


// FUSED (kModeStep only): the new positions are also binned into ctx->grid_next (one wave-aggregated count
// atomic per run of equal cells), so the next step's cell list needs only scan + scatter + sort (engine.hip
// enqueue_step).
#ifndef GCS_FORCE_WAVES_PER_EU
#define GCS_FORCE_WAVES_PER_EU 5  // occupancy target of the fused force kernel (VGPR cap 512 / 5 -> 96)
#endif
#ifndef GCS_FORCE_WAVES_PER_EU_UNFUSED
// the unfused instantiations (the decomposed path's step, force/energy evaluations) at 4 -> 128 VGPRs, no spills:
// C5 decomposed (1 domain) 1.85e9 -> 1.98e9, while the fused rebuild step loses 12 % at 4 (same box, tools/force_variants.sh)
#define GCS_FORCE_WAVES_PER_EU_UNFUSED 4
#endif
template <int MODE, int WAVES, bool FUSED, int NG>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(FUSED ? GCS_FORCE_WAVES_PER_EU : GCS_FORCE_WAVES_PER_EU_UNFUSED))) void k_force(DevCtx* __restrict__ ctx, ForceArgs a)
{
    __shared__ float red[WAVES > 1 ? WAVES : 1][4][64];
    // per-wave pair-loop staging, sized for the larger of the two layouts: one 64-candidate stream (pair_forces) or
    // up to 4 sub-tile streams of 32 (pair_forces_sub)
    __shared__ int s_rowV[WAVES][4 * 17];
    __shared__ int s_rowJ[WAVES][4 * 16];
    __shared__ float4 s_cand[WAVES][4 * 2 * (32 + 1)];  // candidate records (2 x float4) + sentinel(s)
    __shared__ float4 s_locf[MODE == kModeStep ? kTile : 1];  // early local terms: force, mu
    __shared__ float4 s_locr[MODE == kModeStep ? kTile : 1];  // inward reaction, particle index
    __shared__ float4 s_loco[MODE == kModeStep ? kTile : 1];  // outward reaction
    __shared__ int s_candj[MODE == kModeEnergy ? WAVES : 1][4 * 32];
    __shared__ float s_pr[kForcePartials + kBBoxPartials];  // per-block accumulators (lane 0 of wave 0)
    __shared__ double s_pe[kEnergyKinds];
    const int lane = threadIdx.x & 63;
    const int wave = uniform((int)(threadIdx.x >> 6));
    const int ntiles = ctx->ntiles;
    if (threadIdx.x == 0) {
        for (int k = 0; k < kForcePartials; ++k) s_pr[k] = 0.f;
        for (int k = 0; k < 3; ++k) {
            s_pr[kForcePartials + k] = 3.0e38f;
            s_pr[kForcePartials + 3 + k] = -3.0e38f;
        }
        for (int k = 0; k < kEnergyKinds; ++k) s_pe[k] = 0.0;
    }

    const unsigned long long t_start = a.dbg_times ? wall_clock64() : 0ull;
    __shared__ unsigned long long s_dbg[4];  // GCS_DEBUG_TIMES: pair start, pair end (wave 0), local start, end
    // Work units: with a.split, tiles t < nsplit are split in two units (2t, 2t + 1) that take alternate halves of
    // the tile's candidate chunks (8 waves on one tile, in two workgroups); the other tiles are one unit each.
    // There are more units than resident workgroups, so the dispatcher balances the units over the CUs as they
    // free up (a tile's cost varies ~5x with the local density; whole tiles pinned 4-5 per CU left the kernel
    // waiting on the most loaded CU).  The two halves meet through a per-tile arrival counter: the second to
    // finish adds the other's partial forces (write-through stores / sc1 loads) and integrates.
    // a.split == 2: the cell scan chose the heavy tiles and wrote the unit table (ctx->units_ok)
    const bool heavy = MODE == kModeStep && a.split == 2 && a.units != nullptr && ctx->units_ok != 0;
    const int nsplit = (MODE == kModeStep && a.split == 1) ? min(ntiles, a.split_cap) : 0;
    const int nunits = heavy ? ctx->nunits : ntiles + nsplit;
    // workgroups with work: the others leave identity partials, which the tail need not read
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctx->nactive = min((int)gridDim.x, max(nunits, 1));
        if (FUSED && a.bucket_p) {  // for the rebuild kernel (its tail block advances these)
            ctx->rb_grid = ctx->grid_next;
            ctx->rb_step = ctx->step;
            ctx->rb_parity = ctx->parity;
        }
    }
    int first_tile = -1, ntot = 0;
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        int tile, part, nparts;
        int2 tr;
        if (heavy) {
            const int4 ud = a.units[u];
            tr = make_int2(ud.x, ud.y);
            tile = uniform(ud.z);
            part = uniform(ud.w & 0xff);
            nparts = uniform(ud.w >> 8);
        } else {
            tile = (u < 2 * nsplit) ? (u >> 1) : u - nsplit;
            part = (u < 2 * nsplit) ? (u & 1) : 0;
            nparts = (u < 2 * nsplit) ? 2 : 1;
            tr = a.tile_range[tile];
        }
        if (first_tile < 0) first_tile = tile;
        const int s_begin = uniform(tr.x), s_end = uniform(tr.y);
        const int s = s_begin + lane;
        const bool valid = s < s_end;
        const int sl = valid ? s : s_end - 1;
        const float4 pi = a.spos[sl];
        const float bi = a.sb[sl];
        // domain decomposition: this engine integrates the particles of its slab only; tiles of ghosts alone
        // (the halo's cell rows) are skipped whole (the same ballot in every wave: the waves share the lanes)
        // (the fused step kernels are never decomposed: compiled out there)
        const bool own = FUSED || !a.dom_on || box_has(a.dom, pi.x, pi.y, pi.z);
        if (!FUSED && a.dom_on && __ballot(valid && own) == 0ull) continue;

        float fx = 0.f, fy = 0.f, fz = 0.f, acc = 0.f;  // acc: pair energy (ENERGY) or neighbour count
        // Step launches: the particle-local terms (bonds, bending, tethers, walls, point sources; a chain of
        // dependent gathers) do not depend on the pair forces, so the last wave computes them FIRST, while the
        // other waves start the pair loop (it owns the fewest strided chunks), and parks them in LDS.  Wave 0
        // then only adds them after the block reduction instead of running that latency chain at the end.
        const bool early = (MODE == kModeStep) && (WAVES > 1) && (nparts == 1);
        if (early && wave == WAVES - 1) {
            const int i = a.sidx[sl];
            const float4 km = a.kmu[i];
            float lfx = 0.f, lfy = 0.f, lfz = 0.f, en[kEnergyKinds];
            float rin[3] = {0.f, 0.f, 0.f}, rout[3] = {0.f, 0.f, 0.f};
            local_terms<MODE>(ctx, a, i, pi.x, pi.y, pi.z, km, lfx, lfy, lfz, en, rin, rout);
            s_locf[lane] = make_float4(lfx, lfy, lfz, km.x);
            s_locr[lane] = make_float4(rin[0], rin[1], rin[2], __int_as_float(i));
            s_loco[lane] = make_float4(rout[0], rout[1], rout[2], 0.f);
        }
        if (a.dbg_times && threadIdx.x == 0 && first_tile == tile) s_dbg[0] = wall_clock64();
        if (a.has_pair) {
            int* const cj = s_candj[MODE == kModeEnergy ? wave : 0];
            if (NG > 1)
                pair_forces_sub<MODE, (NG > 1 ? NG : 2)>(ctx, a, lane, s, s_begin, s_end, pi, bi, fx, fy, fz, acc,
                                                         s_rowV[wave], s_rowJ[wave], s_cand[wave], cj, ntot,
                                                         part * WAVES + wave, nparts * WAVES);
            else
                pair_forces<MODE, WAVES>(ctx, a, wave, lane, s, s_begin, s_end, pi, bi, fx, fy, fz, acc, s_rowV[wave],
                                         s_rowJ[wave], s_cand[wave], cj, ntot, part * WAVES + wave, nparts * WAVES);
        }
        if (a.dbg_times && threadIdx.x == 0 && first_tile == tile) s_dbg[1] = wall_clock64();
        if (WAVES > 1) {
            red[wave][0][lane] = fx;
            red[wave][1][lane] = fy;
            red[wave][2][lane] = fz;
            red[wave][3][lane] = acc;
            __syncthreads();
            if (wave == 0) {
                fx = red[0][0][lane];
                fy = red[0][1][lane];
                fz = red[0][2][lane];
                acc = red[0][3][lane];
#pragma unroll
                for (int w = 1; w < WAVES; ++w) {
                    fx += red[w][0][lane];
                    fy += red[w][1][lane];
                    fz += red[w][2][lane];
                    acc += red[w][3][lane];
                }
            }
        }
        bool owner = true;  // the unit that integrates the tile (the later of two split halves)
        if (MODE == kModeStep && nparts > 1 && wave == 0) {
            const auto rp = __builtin_amdgcn_make_buffer_rsrc((void*)a.pbuf, 0, 0x7fffffff, 0x00020000);
            st_sc1_f4(rp, (u * kTile + lane) * 16, make_float4(fx, fy, fz, acc));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial is out before the arrival add
            int old = 0;
            if (lane == 0) old = atomicAdd(&a.tcnt[tile], 1);
            owner = __shfl(old, 0) == 1;
            if (owner) {
                // a + b == b + a in IEEE arithmetic: the sum does not depend on which half arrived last
                const float4 o = ld_sc1_f4(rp, ((u ^ 1) * kTile + lane) * 16);
                fx += o.x;
                fy += o.y;
                fz += o.z;
                acc += o.w;
                if (lane == 0) a.tcnt[tile] = 0;  // ready for the next launch
            }
        }
        if (wave == 0 && owner) {
            int i;
            float4 km;
            float en[kEnergyKinds];
            float rin[3] = {0.f, 0.f, 0.f}, rout[3] = {0.f, 0.f, 0.f};
            if (a.dbg_times && threadIdx.x == 0 && first_tile == tile) s_dbg[2] = wall_clock64();
            if (early) {
                const float4 lf = s_locf[lane], lr = s_locr[lane], lo = s_loco[lane];
                fx += lf.x;
                fy += lf.y;
                fz += lf.z;
                km = make_float4(lf.w, 0.f, 0.f, 0.f);  // only mu is used below
                i = __float_as_int(lr.w);
                rin[0] = lr.x;
                rin[1] = lr.y;
                rin[2] = lr.z;
                rout[0] = lo.x;
                rout[1] = lo.y;
                rout[2] = lo.z;
            } else {
                i = a.sidx[sl];
                km = a.kmu[i];
                local_terms<MODE>(ctx, a, i, pi.x, pi.y, pi.z, km, fx, fy, fz, en, rin, rout);
            }
            if (a.dbg_times && threadIdx.x == 0 && first_tile == tile) s_dbg[3] = wall_clock64();
            en[0] = acc;
            if (MODE == kModeEnergy) {
                for (int k = 0; k < kEnergyKinds; ++k) {
                    const double t = wave_sum_d(valid ? (double)en[k] : 0.0);
                    if (lane == 0) s_pe[k] += t;
                }
            } else {
                float v[kForcePartials];
                const bool act = valid && own;  // the particles this engine integrates
                v[0] = wave_sum(act ? rin[0] : 0.f);
                v[1] = wave_sum(act ? rin[1] : 0.f);
                v[2] = wave_sum(act ? rin[2] : 0.f);
                v[3] = wave_sum(act ? rout[0] : 0.f);
                v[4] = wave_sum(act ? rout[1] : 0.f);
                v[5] = wave_sum(act ? rout[2] : 0.f);
                v[6] = wave_max(act ? km.x * sqrtf(fx * fx + fy * fy + fz * fz) : 0.f);
                // the pair loop counted the particle itself
                v[7] = wave_sum(act ? acc - (a.has_pair ? 1.f : 0.f) : 0.f);
                if (lane == 0)
                    for (int k = 0; k < kForcePartials; ++k) s_pr[k] = (k == 6) ? fmaxf(s_pr[k], v[k]) : s_pr[k] + v[k];
                if (MODE == kModeForce) {
                    if (valid) a.force_out[i] = make_float4(fx, fy, fz, 0.f);
                } else {
                    // Euler-Maruyama: x += mu dt F + sqrt(2 T mu dt) xi
                    float4* __restrict__ posn = ctx->parity ? a.pos0 : a.pos1;
                    const float mu = km.x;
                    const float dt = a.pf.timestep;
                    float n0, n1, n2;
                    noise3(a, ctx, i, n0, n1, n2);
                    const float amp = sqrtf(2.f * a.pf.temperature * mu * dt);
                    const float mdt = mu * dt;
                    // ghosts (domain decomposition) keep their position: the owner's exchange refreshes both buffers
                    const float nxp = own ? pi.x + mdt * fx + amp * n0 : pi.x;
                    const float nyp = own ? pi.y + mdt * fy + amp * n1 : pi.y;
                    const float nzp = own ? pi.z + mdt * fz + amp * n2 : pi.z;
                    if (act) posn[i] = make_float4(nxp, nyp, nzp, 0.f);
                    if (FUSED) {
                        // bin the new position into the next step's grid.  Wave-aggregated: lanes are cell-sorted,
                        // so runs of equal cells are common; one atomic per run returns the run's base slot.
                        const int c = valid ? cell_index(ctx->grid_next, nxp, nyp, nzp) : -1;
                        const int cprev = __shfl_up(c, 1);
                        const bool head = valid && (lane == 0 || c != cprev);
                        const unsigned long long hm = __ballot(head);
                        const unsigned long long upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
                        const int h = 63 - __clzll(hm & upto);  // my run's head (lane 0 is always a head)
                        const unsigned long long after = hm & ~upto;
                        const int nvalid = s_end - s_begin;
                        const int run = (after ? (__ffsll((long long)after) - 1) : nvalid) - lane;
                        int base = 0;
                        if (head) base = atomicAdd(&a.count[c], run);
                        base = __shfl(base, h);
                        const int sl = base + (lane - h);
                        if (a.bucket_p) {  // rebuild step: file the particle's sorted record under its cell
                            const float4 rec = make_float4(nxp, nyp, nzp, pi.w);
                            if (valid && sl < kBucketCap) {
                                const size_t e = (size_t)c * kBucketCap + sl;
                                a.bucket_p[e] = rec;
                                a.bucket_q[e] = make_int2(i, __float_as_int(bi));
                            }
                            if (valid && sl >= kBucketCap) {
                                const int k = atomicAdd(&a.ovf_n[ctx->step & 1], 1);
                                a.ovf_p[k] = rec;
                                a.ovf_q[k] = make_int4(i, __float_as_int(bi), c, 0);
                            }
                        } else if (valid) {
                            a.cell_of[i] = c;
                            a.slot[i] = sl;
                        }
                    }
                    const float big = 3.0e38f;
                    const float l0 = wave_min(valid ? nxp : big), l1 = wave_min(valid ? nyp : big),
                                l2 = wave_min(valid ? nzp : big);
                    const float h0 = wave_max(valid ? nxp : -big), h1 = wave_max(valid ? nyp : -big),
                                h2 = wave_max(valid ? nzp : -big);
                    if (lane == 0) {
                        float* b = s_pr + kForcePartials;
                        b[0] = fminf(b[0], l0);
                        b[1] = fminf(b[1], l1);
                        b[2] = fminf(b[2], l2);
                        b[3] = fmaxf(b[3], h0);
                        b[4] = fmaxf(b[4], h1);
                        b[5] = fmaxf(b[5], h2);
                    }
                }
            }
        }
        if (WAVES > 1) __syncthreads();  // `red` is reused by the next tile
    }
    if (WAVES == 1) __syncthreads();  // (WAVES > 1 synchronised at the end of every tile)
    if (a.dbg_times && threadIdx.x == 0) {
        a.dbg_times[4 * blockIdx.x] = t_start;
        a.dbg_times[4 * blockIdx.x + 1] = wall_clock64();
        a.dbg_times[4 * blockIdx.x + 2] =
            first_tile >= 0 ? ((unsigned long long)__smid() << 32) | (unsigned)ntot : ~0ull;
        a.dbg_times[4 * blockIdx.x + 3] = first_tile >= 0 ? (unsigned long long)first_tile : ~0ull;
        for (int k = 0; k < 4; ++k) a.dbg_times[4 * gridDim.x + 4 * blockIdx.x + k] = first_tile >= 0 ? s_dbg[k] : 0ull;
    }
    if (threadIdx.x == 0) {
        if (MODE == kModeEnergy) {
            for (int k = 0; k < kEnergyKinds; ++k) a.part_energy[blockIdx.x * kEnergyKinds + k] = s_pe[k];
        } else {
            for (int k = 0; k < kForcePartials; ++k) a.part_force[blockIdx.x * kForcePartials + k] = s_pr[k];
            if (MODE == kModeStep)
                for (int k = 0; k < kBBoxPartials; ++k)
                    a.part_bbox[blockIdx.x * kBBoxStride + k] = s_pr[kForcePartials + k];
        }
    }
}

// spacestep path: update from stored forces with the adapted timestep (ctx->dt_used)
template <typename R>
__global__ __launch_bounds__(kUpdateBlock) void k_update(const DevCtx* __restrict__ ctx, ForceArgs a)
{
    __shared__ float red[6][kUpdateBlock / 64];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < a.n;
    const int il = valid ? i : a.n - 1;
    const int par = ctx->parity;
    const real4<R>* posc = St<R>::pos(a, par);
    real4<R>* posn = St<R>::pos(a, par ^ 1);
    const real4<R> p = posc[il];
    const real4<R> f = St<R>::force(a)[il];
    const R mu = St<R>::kmu(a)[il].x;
    const R dt = (R)ctx->dt_used;
    R n0, n1, n2;
    noise3<R>(a, ctx, il, n0, n1, n2);
    const R amp = r_sqrt(R(2) * St<R>::prm(a).temperature * mu * dt);
    const R mdt = mu * dt;
    const R xr = p.x + mdt * f.x + amp * n0;
    const R yr = p.y + mdt * f.y + amp * n1;
    const R zr = p.z + mdt * f.z + amp * n2;
    if (valid) posn[i] = mk4<R>(xr, yr, zr, R(0));
    const float x = (float)xr, y = (float)yr, z = (float)zr;  // the bbox of the roundings (what the cells bin)
    const float big = 3.0e38f;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float v[6] = {wave_min(valid ? x : big),  wave_min(valid ? y : big),  wave_min(valid ? z : big),
                  wave_max(valid ? x : -big), wave_max(valid ? y : -big), wave_max(valid ? z : -big)};
    if (lane == 0)
        for (int k = 0; k < 6; ++k) red[k][wave] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        float* pb = a.part_bbox + blockIdx.x * kBBoxStride;
        for (int k = 0; k < 6; ++k) {
            float r = red[k][0];
            for (int w = 1; w < kUpdateBlock / 64; ++w) r = (k < 3) ? fminf(r, red[k][w]) : fmaxf(r, red[k][w]);
            pb[k] = r;
        }
    }
}

// spacestep: dt_used = min(dt, spacestep / max_i mu_i |F_i|)   (INFERRED semantics)
__global__ __launch_bounds__(256) void k_adapt(DevCtx* ctx, ForceArgs a, int blocks, float spacestep, float timestep)
{
    __shared__ float red[4];
    float m = 0.f;
    for (int b = threadIdx.x; b < blocks; b += blockDim.x) m = fmaxf(m, a.part_force[b * kForcePartials + 6]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float mm = red[0];
        for (int w = 1; w < (int)(blockDim.x / 64); ++w) mm = fmaxf(mm, red[w]);
        double dt = timestep;
        if (spacestep > 0.f && (double)mm * dt > (double)spacestep) dt = (double)spacestep / (double)mm;
        ctx->dt_used = dt;
        ctx->max_drift = mm;
    }
}

// Fixed-order reduction of the per-block partials (per thread strided, wave butterflies, waves in index order:
// bitwise reproducible) + the device-resident interphase schedule + the next cell grid.  Any block size that
// is a multiple of 64.  fused: the step's force kernel already binned the new positions with grid_next, which
// becomes the current grid, and the grid for the following step is prepared.
template <int kTailRows>
__device__ __forceinline__ void tail_body(DevCtx* ctx, const ForceArgs& a, int fblocks, int bblocks, int advance,
                                          int apply_sched, int ncell_max, const double* __restrict__ sched, bool fused,
                                          double* red_out)
{
    __shared__ double s_red[16][8];
    __shared__ float s_bb[16][8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
    const int B = blockDim.x;
    // the schedule and the context fields the tail updates are loaded up front (uniform addresses: scalar
    // loads), so their latency overlaps the partial loads instead of forming a chain of dependent round trips
    const double s_flags = sched[kSchedFlags], s_dt = sched[kSchedDt], s_cs0 = sched[kSchedCs0],
                 s_csTau = sched[kSchedCsTau], s_bs0 = sched[kSchedBs0], s_bsTau = sched[kSchedBsTau],
                 s_k0 = sched[kSchedK0], s_k1 = sched[kSchedK0 + 1], s_k2 = sched[kSchedK0 + 2],
                 s_muW = sched[kSchedMuW];
    const long long c_step = ctx->step, c_cursor = ctx->noise_cursor;
    const int c_parity = ctx->parity;
    const double c_time = ctx->time, c_cs = ctx->cs, c_bs = ctx->bs;
    const double c_w0 = ctx->wall[0], c_w1 = ctx->wall[1], c_w2 = ctx->wall[2];
    static_assert(sizeof(Grid) % 4 == 0, "Grid is copied as 32-bit words");
    constexpr int kGridWords = (int)(sizeof(Grid) / 4);
    int c_gn[kGridWords];  // ctx->grid_next as words (constant indices only: stays in registers)
#pragma unroll
    for (int k = 0; k < kGridWords; ++k) c_gn[k] = reinterpret_cast<const int*>(&ctx->grid_next)[k];
    // Latency-shaped: the partials are rows of 8 floats; each thread takes rows tid, tid + B, ... and issues
    // kTailRows rows' 16-B sc1 loads at once (one memory round trip per kTailRows * B rows), combines its rows
    // in order, then lanes meet in wave butterflies and the waves in index order: a fixed order for a given
    // (blocks, blockDim), bitwise reproducible.  Loads past the end return 0 (buffer range check).
    const float big = 3.0e38f;
    const auto rf = __builtin_amdgcn_make_buffer_rsrc((void*)a.part_force, 0, fblocks * 32, 0x00020000);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc((void*)a.part_bbox, 0, bblocks * 32, 0x00020000);
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float bb[6] = {big, big, big, -big, -big, -big};
    float ldisp = 0.f, lfb = 0.f;  // list step: bbox row words 6, 7 (max displacement from the build, fallbacks)
    if (fblocks == bblocks && ctx->nactive > 0) {  // step launches: only the working blocks' rows
        fblocks = min(fblocks, ctx->nactive);
        bblocks = fblocks;
    }
    const int nrow = max(fblocks, bblocks);
    for (int b0 = tid; b0 < nrow; b0 += kTailRows * B) {
        float4 f0[kTailRows], f1[kTailRows], g0[kTailRows], g1[kTailRows];
#pragma unroll
        for (int j = 0; j < kTailRows; ++j) {
            const int off = (b0 + j * B) * 32;
            f0[j] = ld_sc1_f4(rf, off);
            f1[j] = ld_sc1_f4(rf, off + 16);
            g0[j] = ld_sc1_f4(rb, off);
            g1[j] = ld_sc1_f4(rb, off + 16);
        }
#pragma unroll
        for (int j = 0; j < kTailRows; ++j) {
            acc[0] += f0[j].x;
            acc[1] += f0[j].y;
            acc[2] += f0[j].z;
            acc[3] += f0[j].w;
            acc[4] += f1[j].x;
            acc[5] += f1[j].y;
            acc[6] = fmax(acc[6], (double)f1[j].z);
            acc[7] += f1[j].w;
            if (b0 + j * B < bblocks) {
                bb[0] = fminf(bb[0], g0[j].x);
                bb[1] = fminf(bb[1], g0[j].y);
                bb[2] = fminf(bb[2], g0[j].z);
                bb[3] = fmaxf(bb[3], g0[j].w);
                bb[4] = fmaxf(bb[4], g1[j].x);
                bb[5] = fmaxf(bb[5], g1[j].y);
                if (a.list_skin > 0.f) {
                    ldisp = fmaxf(ldisp, g1[j].z);
                    lfb += g1[j].w;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = (k == 6) ? wave_total_max_d(acc[k]) : wave_total_sum_d(acc[k]);
#pragma unroll
    for (int k = 0; k < 6; ++k) bb[k] = (k < 3) ? wave_total_min_f(bb[k]) : wave_total_max_f(bb[k]);
    if (a.list_skin > 0.f) {
        ldisp = wave_total_max_f(ldisp);
        lfb = (float)wave_total_sum_d((double)lfb);
    }
    if (lane == 0) {
        for (int k = 0; k < 8; ++k) s_red[wave][k] = acc[k];
        for (int k = 0; k < 6; ++k) s_bb[wave][k] = bb[k];
        s_bb[wave][6] = ldisp;
        s_bb[wave][7] = lfb;
    }
    __syncthreads();
    if (tid == 0) {
        double tot[8];
        float bb[6];
        for (int k = 0; k < 8; ++k) tot[k] = s_red[0][k];
        for (int k = 0; k < 6; ++k) bb[k] = s_bb[0][k];
        float ld = s_bb[0][6], lf = s_bb[0][7];
        for (int w = 1; w < nw; ++w) {
            for (int k = 0; k < 8; ++k) tot[k] = (k == 6) ? fmax(tot[k], s_red[w][k]) : tot[k] + s_red[w][k];
            for (int k = 0; k < 6; ++k) bb[k] = (k < 3) ? fminf(bb[k], s_bb[w][k]) : fmaxf(bb[k], s_bb[w][k]);
            ld = fmaxf(ld, s_bb[w][6]);
            lf += s_bb[w][7];
        }
        if (a.list_skin > 0.f && !red_out) {
            ctx->ldisp = ld;
            ctx->lfallback += (long long)lf;
        }
        if (red_out) {  // the decomposed step's local reduction only (k_tail_reduce): the context is untouched
            for (int k = 0; k < 8; ++k) red_out[k] = tot[k];
        } else {
        // domain decomposition: the wall sees the reaction of every domain (allreduced by the host's collective)
        if (a.ext_react)
            for (int k = 0; k < 6; ++k) tot[k] = a.ext_react[k];
        // everything below works on the values thread 0 loaded at entry (sc[], c_*): no dependent global reads
        if (fblocks > 0) {
            for (int k = 0; k < 3; ++k) {
                ctx->react_in[k] = tot[k];
                ctx->react_out[k] = tot[3 + k];
            }
            ctx->max_drift = tot[6];
            ctx->neighbors = tot[7] / (double)a.n;
        }
        if (bblocks > 0)
            for (int k = 0; k < 3; ++k) {
                ctx->bbox_lo[k] = bb[k];
                ctx->bbox_hi[k] = bb[3 + k];
            }
        long long step = c_step;
        if (advance) {
            step += 1;
            ctx->step = step;
            ctx->parity = c_parity ^ 1;
            if (a.noise_mode == GCS_NOISE_INJECTED) ctx->noise_cursor = c_cursor + 1;
        }
        double time = c_time, cs = c_cs, bs = c_bs;
        const int flags = (int)s_flags;
        if (apply_sched) {
            // stage_interphase/simulation_driver_interphase.cpp:17 (time), :67-76 (scales), :79-90 (wall)
            const double dt = s_dt;
            if (flags & 1) ctx->time = time = (double)step * dt;
            if (flags & 2) {
                ctx->cs = cs = 1.0 - (1.0 - s_cs0) * exp(-(time / s_csTau));
                ctx->bs = bs = 1.0 - (1.0 - s_bs0) * exp(-(time / s_bsTau));
            }
            if (flags & 4) {
                const double w[3] = {c_w0, c_w1, c_w2}, kw[3] = {s_k0, s_k1, s_k2};
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double net = 0.0;
                    net += tot[k] + tot[3 + k];
                    net -= kw[k] * w[k];
                    ctx->wall[k] = w[k] + dt * s_muW * net;
                }
            }
        }
        if (fused) {
            // the grid that bins the NEXT step's positions: this bbox padded by 2 % + 0.01 (particles move far
            // less per step; any that leave are clamped, which is still exact) and the pair cutoff of that step
            // (closed form of update_core_scale at step + 1)
            float lo[3], hi[3];
            for (int k = 0; k < 3; ++k) {
                const float pad = 0.02f * fmaxf(bb[3 + k] - bb[k], 0.f) + 0.01f;
                lo[k] = bb[k] - pad;
                hi[k] = bb[3 + k] + pad;
            }
            double csn = cs;
            if (apply_sched && (flags & 2)) {
                const double t = (flags & 1) ? (double)(step + 1) * s_dt : time;
                csn = 1.0 - (1.0 - s_cs0) * exp(-(t / s_csTau));
            }
            const float rc = a.has_pair ? a.pf.pair_dist * (a.pair_scaled ? (float)fmax(csn, cs) : 1.f) : 1.f;
#pragma unroll
            for (int k = 0; k < kGridWords; ++k) reinterpret_cast<int*>(&ctx->grid)[k] = c_gn[k];
            ctx->grid_next = make_grid(lo, hi, rc, ncell_max, kPairFx);
        } else {
            // the list step's cell grid (used only when the lists are rebuilt) bins at cutoff + skin
            ctx->grid = make_grid(bb, bb + 3, pair_cutoff(a, cs) + a.list_skin, ncell_max, kPairFx);
        }
        }  // !red_out
    }
    __syncthreads();
}

// the local part of a decomposed step's tail: the fixed-order partial reduction into out[8] (reaction in/out,
// max drift, neighbours); the host allreduces out[0..5] and k_tail then runs with ext_react
__global__ __launch_bounds__(256) void k_tail_reduce(DevCtx* ctx, ForceArgs a, int fblocks, double* out)
{
    tail_body(ctx, a, fblocks, fblocks, 0, 0, 0, a.sched, false, out);
}

__global__ __launch_bounds__(256) void k_tail(DevCtx* ctx, ForceArgs a, int fblocks, int bblocks, int advance,
                                              int apply_sched, int ncell_max, const double* __restrict__ sched)
{
    const unsigned long long t0 = wall_clock64();
    tail_body(ctx, a, fblocks, bblocks, advance, apply_sched, ncell_max, sched, false);
    if (threadIdx.x == 0) {
        ctx->t_tail[0] = t0;
        ctx->t_tail[1] = wall_clock64();
    }
}


// ----------------------------------------------------------------------------------------------------
// list step (GCS_OPT_FUSED_STEP 3; DESIGN.md "The list step")
//
// Neighbour lists with a skin, the md::neighbor_searcher scheme the reference's integrator relies on (SURVEY.md
// §8a row a2): every few steps the cell list is built at cutoff + skin and k_lbuild files, per particle, every
// partner within that radius; in between, one launch per step (k_lstep) evaluates the pair forces from the lists,
// the particle-local terms, the Euler-Maruyama update and, in its last workgroup, the step's tail.  A list is
// complete for the step when the particle's own displacement since the build plus the largest displacement of
// any particle plus the cutoff's growth stays inside the skin; a particle for which that is not guaranteed (or
// whose list overflowed) is evaluated exactly by a search of the build's cell list around its current position
// with radius cutoff + largest displacement.  So the pair set is exact at every step, whatever the rebuild period.

#ifndef GCS_LIST_UNROLL
#define GCS_LIST_UNROLL 8  // list entries per batch of the pair loop
#endif
#ifndef GCS_LIST_WAVES_PER_EU
#define GCS_LIST_WAVES_PER_EU 5  // k_lstep occupancy target (VGPR cap 512 / waves): 5 -> <= 96, no spills
#endif
#ifndef GCS_LIST_BOND_BATCH64
#define GCS_LIST_BOND_BATCH64 4  // the fp64 step's bond batch (each entry holds a 32-B parameter and position record)
#endif
#ifndef GCS_LIST_BOND_BATCH
#define GCS_LIST_BOND_BATCH 4  // bond CSR entries whose loads are issued together in the particle-local terms
#endif

// the contact map's pair count (contacts.hip k_contact_insert: strict fp32 predicate, Fibonacci-hashed open
// addressing, contact_count); i < j by particle index, so each pair counts once
// strict pair predicate of the neighbour search and the contact map: (dx^2 + dy^2) + dz^2 < d2, every operation
// rounded on its own (no contraction), in the positions' precision -- the oracle's gcso_search_neighbors(64)
__device__ __forceinline__ bool strict_lt(float px, float py, float pz, float qx, float qy, float qz, float d2)
{
    const float dx = __fsub_rn(px, qx), dy = __fsub_rn(py, qy), dz = __fsub_rn(pz, qz);
    const float r2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
    return r2 < d2;
}
__device__ __forceinline__ bool strict_lt(double px, double py, double pz, double qx, double qy, double qz, double d2)
{
    const double dx = __dsub_rn(px, qx), dy = __dsub_rn(py, qy), dz = __dsub_rn(pz, qz);
    const double r2 = __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
    return r2 < d2;
}

template <typename R>
__device__ __forceinline__ void list_contact(const ForceArgs& a, R d2, real4<R> p, real4<R> q, int i, int j)
{
    if (j <= i) return;
    if (!strict_lt(p.x, p.y, p.z, q.x, q.y, q.z, d2)) return;
    const unsigned long long key = ((unsigned long long)(unsigned)i << 32) | (unsigned)j;
    if (!contact_count(a.c_keys, a.c_counts, a.c_bits, key)) atomicOr(a.c_overflow, 1);
}

// The list step's context update, by thread 0 of the step's final workgroup once every partial is reduced: the
// tail_body arithmetic of one undecomposed, unfused step (reactions, bbox, step/parity/noise cursor, the schedule of
// stage_interphase/simulation_driver_interphase.cpp:17, :67-90 and the cell grid at cutoff + skin for a rebuild)
// The tail's inputs besides the partial rows (the schedule and the context), loaded by the final workgroup before
// it reduces the rows, so their round trip overlaps the rows'
struct ListTailIn {
    double s_flags, s_dt, s_cs0, s_csTau, s_bs0, s_bsTau, s_muW, s_k[3];
    long long c_step, c_cursor, c_fb;
    int c_parity;
    double c_time, c_cs, c_bs, c_w[3];
};
__device__ __forceinline__ ListTailIn list_tail_load(const DevCtx* ctx, const ForceArgs& a)
{
    const double* sched = a.sched;
    ListTailIn t;
    t.s_flags = sched[kSchedFlags];
    t.s_dt = sched[kSchedDt];
    t.s_cs0 = sched[kSchedCs0];
    t.s_csTau = sched[kSchedCsTau];
    t.s_bs0 = sched[kSchedBs0];
    t.s_bsTau = sched[kSchedBsTau];
    t.s_muW = sched[kSchedMuW];
    for (int k = 0; k < 3; ++k) t.s_k[k] = sched[kSchedK0 + k];
    t.c_step = ctx->step;
    t.c_cursor = ctx->noise_cursor;
    t.c_fb = ctx->lfallback;
    t.c_parity = ctx->parity;
    t.c_time = ctx->time;
    t.c_cs = ctx->cs;
    t.c_bs = ctx->bs;
    for (int k = 0; k < 3; ++k) t.c_w[k] = ctx->wall[k];
    return t;
}

// the launch's totals (list_totals)
struct ListTotals {
    double react[6];  // wall reactions in[3], out[3]
    double nbr;       // neighbour count (stats launches)
    long long nfb;    // fallback particles
    long long nown;   // owned particles (decomposed launches)
    float ld;         // largest displacement from the build
    float bb[6];      // bbox lo[3], hi[3] (bbox launches)
    double drift;     // largest mu |F| (relaxation force launches)
};

// launch flags of k_lstep
constexpr int kLFlagSched = 1;  // apply the device schedule (gcs_schedule)
constexpr int kLFlagBBox = 2;   // the next step rebuilds: reduce the bounding box of the new positions -> its cell grid
constexpr int kLFlagStats = 4;  // reduce the neighbour count (diagnostics: ctx->neighbors)
constexpr int kLFlagDomain = 8;  // decomposed (k_lstep<..., DOM>): owned slots only, local reduction -> a.dom_red
// write the particle-order copy of the new positions (always when the partners are particle-indexed, a.bslot ==
// nullptr; otherwise the step before a rebuild -- k_cell_count bins it -- and the last step of a stretch, which the
// host reads or other kernels take up)
constexpr int kLFlagPos = 16;

// the schedule's closed forms of the next step (time, core and bond scale): they need no totals, so k_pstep
// evaluates them while the step's totals are still landing and hands them to list_tail_apply (the same expressions)
struct TailSched {
    double time, cs, bs;
};
__device__ __forceinline__ TailSched list_tail_sched(const ListTailIn& in)
{
    TailSched s{in.c_time, in.c_cs, 0.0};
    const int sf = (int)in.s_flags;
    if (sf & 1) s.time = (double)(in.c_step + 1) * in.s_dt;
    if (sf & 2) {
        s.cs = 1.0 - (1.0 - in.s_cs0) * exp(-(s.time / in.s_csTau));
        s.bs = 1.0 - (1.0 - in.s_bs0) * exp(-(s.time / in.s_bsTau));
    }
    return s;
}
__device__ void list_tail_apply(DevCtx* ctx, const ForceArgs& a, const ListTailIn& in, const ListTotals& t, int flags,
                                const TailSched* pre = nullptr)
{
    const long long step = in.c_step + 1;
    for (int k = 0; k < 3; ++k) {
        ctx->react_in[k] = t.react[k];
        ctx->react_out[k] = t.react[3 + k];
    }
    if (flags & kLFlagStats) ctx->neighbors = t.nbr / (double)a.n;
    ctx->ldisp = t.ld;
    ctx->lfallback = in.c_fb + t.nfb;
    ctx->step = step;
    ctx->parity = in.c_parity ^ 1;
    if (a.noise_mode == GCS_NOISE_INJECTED) ctx->noise_cursor = in.c_cursor + 1;
    double time = in.c_time, cs = in.c_cs;
    if (flags & kLFlagSched) {
        const int sf = (int)in.s_flags;
        const double dt = in.s_dt;
        const TailSched s = pre ? *pre : list_tail_sched(in);
        if (sf & 1) ctx->time = time = s.time;
        if (sf & 2) {
            ctx->cs = cs = s.cs;
            ctx->bs = s.bs;
        }
        if (sf & 4) {
            for (int k = 0; k < 3; ++k) {
                double net = 0.0;
                net += t.react[k] + t.react[3 + k];
                net -= in.s_k[k] * in.c_w[k];
                ctx->wall[k] = in.c_w[k] + dt * in.s_muW * net;
            }
        }
    }
    if (flags & kLFlagBBox) {  // the grid the next step's rebuild bins with (cutoff at the new core scale + skin)
        for (int k = 0; k < 3; ++k) {
            ctx->bbox_lo[k] = t.bb[k];
            ctx->bbox_hi[k] = t.bb[3 + k];
        }
        ctx->grid = make_grid(t.bb, t.bb + 3, pair_cutoff(a, cs) + a.list_skin, a.ncell_max, kPairFx);
    }
}

// The list step's launch accumulators (a.lticket + kListAccBase, one 128-B line per slot; identities between
// launches), one set per group of workgroups g = b % 8 (a device-scope atomic word takes ~11 ns per arrival: a
// single set would queue all ~1000 workgroups of a C2 launch on each word).  Integer atomics only: the totals do
// not depend on the arrival order, so runs stay bitwise reproducible.
//   0-5   wall reactions in[3], out[3]   high words: h = floor(r 2^20), int64, added
//   6     neighbour count                integer, added (stats launches)
//   7     max displacement from the build (>= 0): float bits, atomic max
//   8     fallback particles             integer, added
//   9-11  bbox lo, 12-14 bbox hi         order-preserving integer image of the float, atomic min / max (bbox launches)
//   15    owned particles                integer, added (decomposed launches)
//   16-21 wall reactions, low words      l = round((r 2^20 - h) 2^32) in [0, 2^32], added: r = (h + l 2^-32) 2^-20
//                                        exactly up to 2^-52 per term (the fp64 step's reactions keep fp64 resolution)
//   22    largest mu |F| (relaxation force launches): the fp64 bits of a value >= 0, atomic max
//   23    a reaction whose fixed-point image would not fit (non-finite or >= 2^41): the totals carry a NaN reaction,
//         as a float sum would
constexpr int kAccReactLo = 16;
constexpr int kAccDrift = 22;
constexpr int kAccWords = kListAccSlots + 1;  // slots + the overflow flag, per group
__device__ __forceinline__ unsigned ordered_bits(float v)
{
    const unsigned b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float from_ordered(unsigned o)
{
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}
__device__ __forceinline__ unsigned long long* acc_slot(unsigned* base, int k)
{
    return reinterpret_cast<unsigned long long*>(base + 32 * k);
}
// fold one value into slot k of a group's accumulators (one lane per slot)
// (v: the slot's value; an fp32 value converts exactly, and slots 6..15 only ever receive fp32 or integer values)
__device__ __forceinline__ void acc_fold(unsigned* base, int k, double v)
{
    unsigned long long* w = acc_slot(base, k);
    unsigned* w32 = reinterpret_cast<unsigned*>(w);
    if (k < 6) {
        const double sv = v * 0x1p20;
        if (fabs(sv) < 0x1p61) {
            const double h = floor(sv);
            const long long l = __double2ll_rn((sv - h) * 0x1p32);
            __hip_atomic_fetch_add(w, (unsigned long long)(long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(acc_slot(base, kAccReactLo + k), (unsigned long long)l, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_fetch_or(reinterpret_cast<unsigned*>(acc_slot(base, kListAccSlots)), 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (k == 6 || k == 8 || k == 15) {
        __hip_atomic_fetch_add(w, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (k == kAccDrift) {
        __hip_atomic_fetch_max(w, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (k == 7) {
        __hip_atomic_fetch_max(w32, __float_as_uint((float)v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (k < 12) {
        __hip_atomic_fetch_min(w32, ordered_bits((float)v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_fetch_max(w32, ordered_bits((float)v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// the final workgroup (all threads): read every group's accumulators (device-coherent loads), combine them (integer
// sums, min, max: independent of the order) and reset them for the next launch; thread 0 gets the totals
__device__ void list_totals(unsigned* base, int ngroups, ListTotals& t)
{
    __shared__ unsigned long long s_acc[8 * kAccWords];
    const int tid = threadIdx.x;
    for (int q = tid; q < ngroups * kAccWords; q += blockDim.x) {
        unsigned long long* w = acc_slot(base, q);
        s_acc[q] = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w, list_acc_identity(q % kAccWords), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tid != 0) return;
    // two passes over the groups (slots 0..15, then the low reaction words and the flag), so no more than 16 words
    // and their operands are live at once
    unsigned long long v[kAccReactLo];
    for (int k = 0; k < kAccReactLo; ++k) v[k] = s_acc[k];
    for (int g = 1; g < ngroups; ++g) {
        const unsigned long long* x = s_acc + g * kAccWords;
        for (int k = 0; k < kAccReactLo; ++k) {
            if (k <= 6 || k == 8 || k == 15) v[k] += x[k];
            else if (k >= 9 && k < 12) v[k] = min((unsigned)v[k], (unsigned)x[k]);
            else v[k] = max((unsigned)v[k], (unsigned)x[k]);
        }
    }
    unsigned long long lo[6], bad = 0, drift = 0;
    for (int k = 0; k < 6; ++k) lo[k] = 0;
    for (int g = 0; g < ngroups; ++g) {
        const unsigned long long* x = s_acc + g * kAccWords;
        for (int k = 0; k < 6; ++k) lo[k] += x[kAccReactLo + k];
        drift = max(drift, x[kAccDrift]);
        bad |= x[kListAccSlots];
    }
    t.drift = __longlong_as_double((long long)drift);
    for (int k = 0; k < 6; ++k)
        t.react[k] = (bad & 1ull) ? __longlong_as_double(0x7ff8000000000000ll)
                                  : (double)(long long)v[k] * 0x1p-20 + (double)(long long)lo[k] * 0x1p-52;
    t.nbr = (double)v[6];
    t.ld = __uint_as_float((unsigned)v[7]);
    t.nfb = (long long)v[8];
    t.nown = (long long)v[15];
    for (int k = 0; k < 6; ++k) t.bb[k] = from_ordered((unsigned)v[9 + k]);
}

#ifndef GCS_LBUILD_GROUPS
#define GCS_LBUILD_GROUPS 2  // k_lbuild: candidate groups per tile (2: 32 lanes each, 4: 16 lanes each)
#endif
#ifndef GCS_XCD_REMAP
#define GCS_XCD_REMAP 1  // 1: the list kernels give each XCD a contiguous range of tiles (see xcd_block)
#endif
// Workgroups are dispatched to the 8 XCDs round-robin (b % 8), each XCD with its own L2.  Tiles are spatially
// ordered (slots sorted by cell), so handing XCD x the contiguous tile range x * G / 8 ... instead of every 8th
// tile keeps the pair partners an XCD gathers within its own slab: each L2 fetches about 1/8 of the positions
// instead of all of them.  A bijection of [0, G) (G need not be a multiple of 8); the dispatch order only affects
// speed, never which tiles are processed.
// Only for the 16-bit absolute lists (<= 65,536 particles: C1, C2, C4's trajectories): there every L2 would otherwise
// fetch the whole position array, and the slabs win (same box, C2 fp64 4 trajectories 4.51-4.54 vs 4.39e9, single
// 1.91 vs 1.83; fp32 6.14 vs 5.95).  Beyond (C5's plane-relative lists) the slabs lose: 1.92 vs 2.12e9 at C5 fp64,
// k_lstep 223 vs 201 us, although the L2s fetch less (393 vs 508 MB per launch) -- a slab of a non-uniform system
// is a non-uniform share of the work, and the round-robin dispatch runs at the pace of the XCD with the densest slab
// (profiles/r06s_c5_l2_*.txt, r06t_xcd_remap_c2.txt)
template <typename LE>
__device__ __forceinline__ int xcd_block(int b, int G)
{
#if GCS_XCD_REMAP
    if constexpr (sizeof(LE) == 2 && !ListFmt<LE>::rel) {
        const int x = b & 7, k = b >> 3, q = G >> 3, r = G & 7;
        return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
    }
#endif
    (void)G;
    return b;
}

#ifndef GCS_LBUILD_WAVES_PER_EU
#define GCS_LBUILD_WAVES_PER_EU 8  // k_lbuild occupancy target: 8 -> <= 64 VGPRs (65 without it: 7 waves/SIMD)
#endif
// LE: list entry type (unsigned short when every slot index fits 16 bits: half the list traffic)
template <typename LE, int kListWaves>
__global__ __launch_bounds__(64 * kListWaves) __attribute__((amdgpu_waves_per_eu(GCS_LBUILD_WAVES_PER_EU))) void k_lbuild(DevCtx* __restrict__ ctx, ForceArgs a)
{
    __shared__ int s_rowV[kListWaves][4 * 17];
    __shared__ int s_rowJ[kListWaves][4 * 16];
    __shared__ float4 s_cand[kListWaves][GCS_LBUILD_GROUPS * 2 * (32 + 1)];
    __shared__ int s_ovf[kListWaves][64];
    const int lane = threadIdx.x & 63;
    const int wave = uniform((int)(threadIdx.x >> 6));
    const int ntiles = ctx->ntiles;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // read by the list steps that follow (next launches); every block here reads ctx->grid only
        ctx->lgrid = ctx->grid;
        ctx->lrc_b = pair_cutoff(a, ctx->cs);
        ctx->lnslots = a.cstart[ctx->grid.ncell];  // binned particles (N undecomposed)
        ctx->ldisp = 0.f;
        ctx->lbuilds += 1;
        ctx->nactive = 0;  // the list step's tail reads every workgroup's partial row
    }
    int ntot = 0;
    unsigned long long* const dbg = a.dbg_build ? a.dbg_build + 8 * blockIdx.x : nullptr;
    if (dbg && threadIdx.x == 0) dbg[0] = wall_clock64();
    bool first = true;
    // the launch has force_grid(n) workgroups, the cell rows need ntiles (device-side): remap over the ones in use
    const int gused = min((int)gridDim.x, ntiles);
    for (int tile = (int)blockIdx.x < gused ? xcd_block<LE>(blockIdx.x, gused) : ntiles; tile < ntiles;
         tile += gridDim.x) {
        const int2 tr = a.tile_range[tile];
        const int s_begin = uniform(tr.x), s_end = uniform(tr.y);
        const int s = s_begin + lane;
        const bool valid = s < s_end;
        const int sl = valid ? s : s_end - 1;
        const float4 pi = a.spos[sl];
        const float bi = a.sb[sl];
        const int self = a.sidx[sl];
        float fx = 0.f, fy = 0.f, fz = 0.f, acc = 0.f;
        int cnt = 0;
        unsigned long long pend = 0ull;
        int4 lb = make_int4(0, 0, 0, 0);
        pair_forces_sub<kModeList, GCS_LBUILD_GROUPS, LE>(ctx, a, lane, s, s_begin, s_end, pi, bi, fx, fy, fz, acc, s_rowV[wave],
                                      s_rowJ[wave], s_cand[wave], nullptr, ntot, wave, kListWaves, self, valid, &cnt,
                                      &pend, &lb);
        if (ListFmt<LE>::rel && valid && wave == 0) a.lbase[s] = lb;
        {  // the last, partial word of the lane's segment (its r entries sit in the top r slots: shift them down)
            constexpr int E = 8 / (int)sizeof(LE);
            const int r = cnt % E;
            if (valid && cnt < a.list_cap && r != 0)
                reinterpret_cast<unsigned long long*>(a.list)[((size_t)wave * (a.list_cap / E) + cnt / E) * a.list_stride + s] =
                    pend >> (8 * (int)sizeof(LE) * (E - r));
        }
        if (dbg && first && lane == 0) dbg[2 + wave] = wall_clock64();
        s_ovf[wave][lane] = cnt > a.list_cap ? 1 : 0;
        __syncthreads();
        int ovf = 0;
#pragma unroll
        for (int w = 0; w < kListWaves; ++w) ovf |= s_ovf[w][lane];
        if (valid) a.lcount[(size_t)wave * a.list_stride + s] = min(cnt, a.list_cap) | (ovf ? kListOverflow : 0);
        __syncthreads();
        if (dbg && first && threadIdx.x == 0) {
            dbg[1] = wall_clock64();
            dbg[6] = (unsigned long long)ntot;
            dbg[7] = (unsigned long long)tile;
        }
        first = false;
    }
}

// the mixed soft-core pair force of one partner (the tile kernel's phase-2 arithmetic, in the global frame)
template <typename R>
__device__ __forceinline__ void list_pair(R xi, R yi, R zi, real4<R> q, real2<R> t, R ahi, R bhi, R kA, R kB, R k2a,
                                          R k2b, R rc2, bool real, R& fx, R& fy, R& fz, R& nbr)
{
    const R dx = xi - q.x, dy = yi - q.y, dz = zi - q.z;
    const R r2 = r_fma(dz, dz, r_fma(dy, dy, dx * dx));
    const R ga = r_fmax(r_fma(-k2a, r2, R(1)), R(0));
    const R tt = r2 * k2b;
    const R t2 = tt * tt;
    const R gb = r_fmax(r_fma(-t2, t2, R(1)), R(0));
    const R A = r_fma(kA, t.x, ahi), B = r_fma(kB, t.y, bhi);
    const bool in = real && r2 < rc2;
    const R coef = in ? r_fma(A, ga * ga, B * (gb * gb * t2 * tt)) : R(0);
    fx = r_fma(coef, dx, fx);
    fy = r_fma(coef, dy, fy);
    fz = r_fma(coef, dz, fz);
    nbr += in ? R(1) : R(0);
}


__device__ __forceinline__ int lgrid_cell(const Grid& g, int k, float v)
{
    const float q = (v - g.lo[k]) * g.inv[k];
    const int c = (q > 0.f) ? (int)fminf(q, 1.0e9f) : 0;
    return min(c, g.n[k] - 1);
}


#ifndef GCS_LIST_WAVES_PER_EU_CT
#define GCS_LIST_WAVES_PER_EU_CT 4  // the contact-step instantiation (CT, 1 launch in 20): 4 -> <= 128, no spills
#endif
#ifndef GCS_LIST_WAVES_PER_EU64
#define GCS_LIST_WAVES_PER_EU64 4  // the fp64 step: every position / force register is a pair -> <= 128 VGPRs
#endif
#ifndef GCS_LIST_UNROLL64
// fp64 step: list entries per batch of the pair loop.  Same-box A/B (tools/gpu_r04b.sh, profiles/r04_variants.txt):
// 4 entries 3.92e9 (single trajectory 1.95e9, k_lstep 29.0 us) vs 8 entries 3.84e9 (1.80e9, 31.2 us); at 5 waves
// per SIMD either spills (3.74e9 / 1.15e9)
#define GCS_LIST_UNROLL64 4
#endif
#ifndef GCS_LIST_PF_BATCH
#define GCS_LIST_PF_BATCH 8  // fp64 step, prefilter: list entries per fp32 batch
#endif
#ifndef GCS_LIST_PF_HITS
#define GCS_LIST_PF_HITS 2  // fp64 step, prefilter: hits whose fp64 records are gathered per round
#endif
constexpr int kPfRing = 16;  // per lane: queued prefilter hits (a power of two >= GCS_LIST_PF_BATCH + GCS_LIST_PF_HITS)
static_assert(kPfRing >= GCS_LIST_PF_BATCH + GCS_LIST_PF_HITS && (kPfRing & (kPfRing - 1)) == 0, "the hit ring");
// One list step.  A workgroup takes 64 consecutive slots (W waves).  Phases, with nothing but LDS carried from one to
// the next (every wave's registers are free for the next phase):
//   1. slot loads: current position (.w = particle | class << 24), build position, list count, the first kU
//      entries of the wave's segment; the local-terms wave (W - 1) also the slot's constants and bond row.
//   2. wave W - 1: the particle-local terms (bond CSR, droplet, bending, tethers, point sources, walls) -> LDS
//   3. every wave: its list segment, kU entries per batch (one gather per entry, the next batch's entries in flight),
//      the exact search for the lanes the lists may not cover; forces + neighbour counts -> LDS.  Wave 1: the
//      Philox noise -> LDS
//   4. (barrier) wave 0: sum the waves' forces, integrate, store; the launch statistics it owns (largest
//      displacement, fallbacks; bbox / neighbour count on flagged launches) into the group's accumulators.
//      Waves 1.. (in parallel): the wall reactions into the accumulators
//   5. (barrier) the two-level ticket; the final workgroup reads the accumulators and advances the context
// DOM (decomposed): a slot is integrated only when it belongs to this build (s < ctx->lnslots) and its
// particle lies in the domain's box at the step start; the final workgroup writes the local reduction to a.dom_red
// (the tail runs after the allreduce: k_ldom_tail)
// R: the arithmetic precision (GCS_PRECISION_F32 / F64).  Positions, forces, the integration, the pair test and the
// contact predicate are in R; the list bookkeeping (build positions, displacements, cell ranges, bbox) is fp32 with
// margins (a partner within the cutoff in R is always in the list or found by the exact search: the skin test keeps
// 0.1 % of the skin, ~1e-4, against fp32 roundings of ~1e-6 of the coordinates).
// RLX (the relaxation step's force launch, simulation_driver_relaxation.cpp:48-55): wave 0 stores the force (slot
// order, .w = mu) instead of integrating and folds max mu |F| into the accumulators; the final workgroup sets the
// adapted timestep ctx->dt_used (k_red64's arithmetic) and the reactions; k_lupdate then moves the particles.
// List words are read once per step, with the non-temporal hint (ForceArgs::list_nt) when the lists are far beyond the
// L2s, so they do not displace the partners (same-box A/B, profiles/r04_list_format_ab.txt: C5 fp64 +3-5 %, C2 fp64
// with 4 trajectories -16 % when applied to its 16-bit lists, which the L2 / Infinity Cache keep).
template <typename LE, int W, bool CT, bool DOM = false, typename R = float, bool RLX = false>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(CT ? GCS_LIST_WAVES_PER_EU_CT : (sizeof(R) == 8 ? GCS_LIST_WAVES_PER_EU64 : GCS_LIST_WAVES_PER_EU)))) void k_lstep(DevCtx* __restrict__ ctx, ForceArgs a, int flags)
{
    using R4 = real4<R>;
    using R2 = real2<R>;
    // fp64 (not the contact step): the fp32 prefilter (PF, below); its per-lane rings of hits in LDS
    constexpr bool PF = sizeof(R) == 8 && !CT && GCS_LIST_PREFILTER;
    using QT = typename std::conditional<sizeof(LE) == 2, unsigned short, int>::type;
    __shared__ QT s_hq[PF ? W : 1][PF ? kPfRing : 1][kTile];
    __shared__ R red[W][4][kTile];
    __shared__ R4 s_locf[kTile], s_noise[kTile];
    __shared__ R2 s_tab[kMaxTypes];
    __shared__ int s_last, s_final;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uniform(tid >> 6);
    // GCS_DEBUG_TIMES: per workgroup 8 wall-clock stamps (start, wave 0: pair loop start / end, reduced, integrated,
    // workgroup end, ticket taken, tail end)
    unsigned long long* const dbg = a.dbg_times ? a.dbg_times + 8 * blockIdx.x : nullptr;
    if (dbg && tid == 0) dbg[0] = wall_clock64();
    const int n = a.n;
    const FieldPrm<R>& P = St<R>::prm(a);
    const int tile = xcd_block<LE>(blockIdx.x, gridDim.x);
    const int s = tile * kTile + lane;
    const bool valid = s < n;
    const int sl = valid ? s : n - 1;
    const int par = a.par_hint >= 0 ? a.par_hint : ctx->parity;
    const R4* __restrict__ qc = St<R>::psort(a, par);  // slot order (pair partners)
    const int cap = a.list_cap;
    const size_t stride = (size_t)a.list_stride;
    constexpr int kU = sizeof(R) == 4 ? GCS_LIST_UNROLL : GCS_LIST_UNROLL64;
    constexpr int kE = 8 / (int)sizeof(LE);  // entries per 8-byte list word
    constexpr int kW = kU / kE;              // list words per batch
    static_assert(kU % kE == 0, "a batch is whole list words");
    constexpr int kIdx = (1 << kListIndexBits) - 1;
    const int klast = (cap / kU - 1) * kU;  // the segment's last batch (list_cap is a multiple of kU)
    const bool lnt = a.list_nt != 0;
    auto word = [&](const uint2* p) -> uint2 {
        if (lnt) {
            const unsigned long long v = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(p));
            return make_uint2((unsigned)v, (unsigned)(v >> 32));
        }
        return *p;
    };
    const uint2* __restrict__ segw = reinterpret_cast<const uint2*>(a.list) + (size_t)wave * (cap / kE) * stride + sl;

    // 1. slot loads (one round trip)
    const R2* __restrict__ tab = St<R>::type_ab(a);
    for (int t = tid; t < a.ntypes; t += blockDim.x) s_tab[t] = tab[t];
    const R4 pi = qc[sl];
    const float4 pb = a.spos[sl];
    const int cw = a.lcount[(size_t)wave * stride + sl];
    int4 lb = make_int4(0, 0, 0, 0);
    if constexpr (ListFmt<LE>::rel) lb = a.lbase[sl];
    uint2 e[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) e[j] = word(segw + (size_t)j * stride);  // list_cap >= kU: in bounds
    const R cs = (R)ctx->cs;
    const float D = ctx->ldisp;
    const float lrc_b = ctx->lrc_b;
    // the contact distance from the context (k_set_contact before the launch), so a captured graph serves any update
    R cd2 = R(0);
    if constexpr (CT) {
        if constexpr (sizeof(R) == 4) cd2 = ctx->contact_d2; else cd2 = ctx->contact_d2_64;
    }
    __syncthreads();  // s_tab, the LDS image
    const int ngroups = min((int)gridDim.x, 8);
    const int g = blockIdx.x % ngroups;
    unsigned* const acc = a.lticket + kListAccBase + 32 * kAccWords * g;

    const int pk = wbits(pi.w);
    // (clamped: a decomposed ghost slot that missed its band record -- a band over capacity -- may hold a stale
    // record of another build in this parity; such a lane integrates nothing, but its local terms index by i)
    const int i = min(pk & kIdx, n - 1);
    const bool act = DOM ? (valid && s < ctx->lnslots && box_has(a.dom, (float)pi.x, (float)pi.y, (float)pi.z)) : valid;
    const R scale = a.pair_scaled ? cs : R(1);
    const R sa = P.pa_sig * scale, sbb = P.pb_sig * scale;
    const R k2a = R(1) / (sa * sa), k2b = R(1) / (sbb * sbb);
    const R kA = R(0.5) * R(6) * P.pa_eps * k2a, kB = R(0.5) * R(24) * P.pb_eps * k2b;
    const R rc = pair_cutoff_r<R>(a, (double)cs), rc2 = rc * rc;
    const float rcf = (float)rc;
    // a particle whose own displacement exceeds this may miss a partner in its list (0.999: fp32 margin)
    const float slack = 0.999f * a.list_skin - D - fmaxf(rcf - lrc_b, 0.f);
    const float ex = (float)(pi.x - (R)pb.x), ey = (float)(pi.y - (R)pb.y), ez = (float)(pi.z - (R)pb.z);
    const float di = sqrtf(fmaf(ez, ez, fmaf(ey, ey, ex * ex)));
    const bool fb = act && (di > slack || (cw & kListOverflow) != 0);
    // contacts (CT): the lists must cover the contact distance; a particle whose list does not is searched for its
    // contacts only (its forces take exactly the path they take without contacts: identical bits)
    const float rcc = CT ? fmaxf(rcf, sqrtf((float)cd2)) : rcf;
    const bool fbc = CT && valid && (di > 0.999f * a.list_skin - D - fmaxf(rcc - lrc_b, 0.f) || (cw & kListOverflow) != 0);

    // 2. the particle-local terms (a dependent-gather chain: first, on the last wave), parked in LDS
    if (wave == W - 1) {
        const R4 km = St<R>::skmu(a)[sl];
        const int2 erow = a.sbrow[sl];
        R lfx = 0, lfy = 0, lfz = 0, en[kEnergyKinds];
        R rin[3] = {0, 0, 0}, rout[3] = {0, 0, 0};
        local_terms<kModeStep, sizeof(R) == 8 ? GCS_LIST_BOND_BATCH64 : GCS_LIST_BOND_BATCH, R>(ctx, a, i, pi.x, pi.y,
                                                                                             pi.z, km, lfx, lfy, lfz, en, rin, rout,
                                                       erow, a.bslot ? qc : nullptr);
        if constexpr (DOM) {
            // the fused pack's bond check (k_domain_pack's): a bond of an owned particle longer than the halo (its
            // partner may be a stale ghost); the cut-off droplet and shared particles excepted
            if (a.dom_bands && act && a.has_bonds && !(a.dom_shared && a.dom_shared[i])) {
                const R4* __restrict__ pc = St<R>::pos(a, par);
                const float h2 = a.dom_halo * a.dom_halo;
                bool far = false;
                for (int q = erow.x; q < erow.y; ++q) {
                    const int2 en2 = a.bent[q];
                    if ((en2.y & 15) == kSoftwell || (a.dom_shared && a.dom_shared[en2.x])) continue;
                    const R4 pj = pc[en2.x];
                    const float dx = (float)pi.x - (float)pj.x, dy = (float)pi.y - (float)pj.y,
                                dz = (float)pi.z - (float)pj.z;
                    far |= dx * dx + dy * dy + dz * dz >= h2;
                }
                if (far) atomicOr(a.dom_flags, 1);
            }
        }
        s_locf[lane] = mk4<R>(lfx, lfy, lfz, km.x);
        // the wall reactions straight into the launch accumulators (lane c: component c, inward then outward)
        R rv = 0;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const R x = wave_sum_r(act ? (c < 3 ? rin[c] : rout[c - 3]) : R(0));
            if (lane == c) rv = x;
        }
        if (lane < 6) acc_fold(acc, lane, (double)rv);
    }

    // 3. the wave's list segment
    R fx = 0, fy = 0, fz = 0, nbr = 0;
    const R2 own = s_tab[(unsigned)pk >> kListIndexBits];
    const R ahi = kA * own.x, bhi = kB * own.y;
    if (dbg && tid == 0) dbg[1] = wall_clock64();
    if (a.has_pair) {
        const int cnt = (act && !fb) ? min(cw & kListCountMask, cap) : 0;
        const int kmax = uniform(wave_max_int(cnt));
        if constexpr (PF) {
        // fp64: a software pipeline of two gathers per round, issued together (one round trip): the fp32 roundings
        // (fsort, 16 B) of the next kUF entries, and the fp64 records (32 B) of the kUD oldest hits of the lane's
        // prefilter queue; then the exact pairs of those hits in R (list_pair) and the fp32 test of the batch, whose
        // hits join the queue.  A pair within rc in R always passes the test (the margin: k_pstep's), and an entry
        // that fails it contributes exactly 0 in list_pair, so the forces, the neighbour counts and their order (list
        // order) are those of gathering every entry in R: bitwise the same.  At the 350 per-mille skin ~41 % of the
        // entries lie within the cutoff: the fp64 gathers and pair arithmetic of the rest are skipped, and the fp32
        // batches hold half the registers of fp64 ones per entry in flight
        constexpr int kUF = GCS_LIST_PF_BATCH, kUD = GCS_LIST_PF_HITS;
        constexpr int kWF = kUF / kE;
        static_assert(kUF % kE == 0 && kUF % kU == 0, "a prefilter batch is whole list words and list batches");
        const float4* __restrict__ fq = St<R>::fsort(a, par);
        const float pxf = (float)pi.x, pyf = (float)pi.y, pzf = (float)pi.z;
        const float mag = fmaxf(fabsf(pxf), fmaxf(fabsf(pyf), fabsf(pzf)));
        const float thr = (float)rc2 * 1.001f + 1.0e-4f * rcf + 1.0e-6f * rcf * (mag + rcf);
        const int klastF = (cap / kUF - 1) * kUF;  // the segment's last prefilter batch (list_cap: whole batches of 8)
        QT* const hq = &s_hq[wave][0][lane];
        uint2 ef[kWF];
#pragma unroll
        for (int j = 0; j < kWF; ++j) ef[j] = j < kW ? e[j] : word(segw + (size_t)j * stride);
        int qh = 0, qt = 0;  // this lane's hits consumed / queued
        for (int k0 = 0;;) {
            const int take = min(qt - qh, kUD);
            if (k0 >= kmax && !__any(qt > qh)) break;
            R4 d[kUD];
#pragma unroll
            for (int u = 0; u < kUD; ++u)
                d[u] = qc[u < take ? list_slot<LE>((int)hq[((qh + u) & (kPfRing - 1)) * kTile], lb) : sl];
            const bool pre = k0 < kmax && uniform(wave_max_int(qt - qh - take)) + kUF <= kPfRing;
            float4 f[kUF];
            uint2 ec[kWF];  // this batch's entry words (ef then takes the next batch's)
            if (pre) {
#pragma unroll
                for (int j = 0; j < kWF; ++j) ec[j] = ef[j];
#pragma unroll
                for (int u = 0; u < kUF; ++u)
                    f[u] = fq[(k0 + u < cnt) ? list_slot<LE>(list_entry<LE>(ec, u), lb) : sl];
                const int kn = min(k0 + kUF, klastF);
#pragma unroll
                for (int j = 0; j < kWF; ++j) ef[j] = word(segw + (size_t)(kn / kE + j) * stride);
            }
            __builtin_amdgcn_sched_barrier(0);  // every gather of the round in flight before the arithmetic
#pragma unroll
            for (int u = 0; u < kUD; ++u)
                list_pair<R>(pi.x, pi.y, pi.z, d[u], s_tab[(unsigned)wbits(d[u].w) >> kListIndexBits], ahi, bhi, kA,
                             kB, k2a, k2b, rc2, u < take, fx, fy, fz, nbr);
            qh += take;
            if (pre) {
#pragma unroll
                for (int u = 0; u < kUF; ++u) {
                    const float dx = f[u].x - pxf, dy = f[u].y - pyf, dz = f[u].z - pzf;
                    const float r2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                    if (k0 + u < cnt && r2 < thr) {
                        hq[(qt & (kPfRing - 1)) * kTile] = (QT)list_entry<LE>(ec, u);
                        ++qt;
                    }
                }
                k0 += kUF;
            }
        }
        } else {
        // batches of kU entries: the partners' gathers are issued first, then the next batch's entry words (they
        // return right behind the gathers, so each batch costs one round trip), then the pair forces (and contacts)
        for (int k0 = 0; k0 < kmax; k0 += kU) {
            R4 q[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) q[u] = qc[(k0 + u < cnt) ? list_slot<LE>(list_entry<LE>(e, u), lb) : sl];
            const int kn = min(k0 + kU, klast);
#pragma unroll
            for (int j = 0; j < kW; ++j) e[j] = word(segw + (size_t)(kn / kE + j) * stride);
            __builtin_amdgcn_sched_barrier(0);  // keep the entry loads here, ahead of the arithmetic
#pragma unroll
            for (int u = 0; u < kU; ++u)
                list_pair<R>(pi.x, pi.y, pi.z, q[u], s_tab[(unsigned)wbits(q[u].w) >> kListIndexBits], ahi, bhi, kA,
                             kB, k2a, k2b, rc2, k0 + u < cnt, fx, fy, fz, nbr);
            if constexpr (CT) {
#pragma unroll
                for (int u = 0; u < kU; ++u)
                    if (!fbc && k0 + u < cnt) list_contact<R>(a, cd2, pi, q[u], i, wbits(q[u].w) & kIdx);
            }
        }
        }
        // exact search of the build's cell list for the particles the lists may not cover: a partner within rc
        // now was within rc + D at the build.  Wave-cooperative: the wave takes its fallback lanes one at a time,
        // its 64 lanes sweep that particle's candidate slots (the waves of the tile alternate over cell rows), and
        // a wave sum hands the result to the particle's lane
        unsigned long long fbm = __ballot(fb);
        if (fbm) {
            const Grid lg = ctx->lgrid;
            const float Rr = rcf + D + 1.0e-5f * (rcf + D);
            while (fbm) {
                const int L = __ffsll((long long)fbm) - 1;
                fbm &= fbm - 1ull;
                const R px = __shfl(pi.x, L), py = __shfl(pi.y, L), pz = __shfl(pi.z, L);
                const R pah = __shfl(ahi, L), pbh = __shfl(bhi, L);
                const int sL = uniform(__shfl(s, L));
                const float fpx = (float)px, fpy = (float)py, fpz = (float)pz;
                const int x0 = uniform(lgrid_cell(lg, 0, fpx - Rr)), x1 = uniform(lgrid_cell(lg, 0, fpx + Rr));
                const int y0 = uniform(lgrid_cell(lg, 1, fpy - Rr)), y1 = uniform(lgrid_cell(lg, 1, fpy + Rr));
                const int z0 = uniform(lgrid_cell(lg, 2, fpz - Rr)), z1 = uniform(lgrid_cell(lg, 2, fpz + Rr));
                R gx = 0, gy = 0, gz = 0, gn = 0;
                int row = 0;
                for (int z = z0; z <= z1; ++z)
                    for (int y = y0; y <= y1; ++y, ++row) {
                        if ((row % W) != wave) continue;
                        const int base = (z * lg.n[1] + y) * lg.n[0];
                        const int t0 = a.cstart[base + x0], t1 = a.cstart[base + x1 + 1];
                        for (int t = t0 + lane; t < t1; t += kTile) {
                            const R4 q = qc[t];
                            list_pair<R>(px, py, pz, q, s_tab[(unsigned)wbits(q.w) >> kListIndexBits], pah, pbh, kA, kB,
                                         k2a, k2b, rc2, t != sL, gx, gy, gz, gn);
                        }
                    }
                gx = wave_sum_r(gx);
                gy = wave_sum_r(gy);
                gz = wave_sum_r(gz);
                gn = wave_sum_r(gn);
                if (lane == L) {
                    fx += gx;
                    fy += gy;
                    fz += gz;
                    nbr += gn;
                }
            }
        }
    }
    if constexpr (CT) {
        // contacts of the particles whose lists do not cover the contact distance: the build's cell list around
        // the current position with radius d + D, swept by the whole wave per particle as above
        unsigned long long fcm = __ballot(fbc);
        if (fcm) {
            const Grid lg = ctx->lgrid;
            const float Rr = rcc + D + 1.0e-5f * (rcc + D);
            while (fcm) {
                const int L = __ffsll((long long)fcm) - 1;
                fcm &= fcm - 1ull;
                const R4 pL = mk4<R>(__shfl(pi.x, L), __shfl(pi.y, L), __shfl(pi.z, L), R(0));
                const int iL = __shfl(i, L), sL = uniform(__shfl(s, L));
                const float fpx = (float)pL.x, fpy = (float)pL.y, fpz = (float)pL.z;
                const int x0 = uniform(lgrid_cell(lg, 0, fpx - Rr)), x1 = uniform(lgrid_cell(lg, 0, fpx + Rr));
                const int y0 = uniform(lgrid_cell(lg, 1, fpy - Rr)), y1 = uniform(lgrid_cell(lg, 1, fpy + Rr));
                const int z0 = uniform(lgrid_cell(lg, 2, fpz - Rr)), z1 = uniform(lgrid_cell(lg, 2, fpz + Rr));
                int row = 0;
                for (int z = z0; z <= z1; ++z)
                    for (int y = y0; y <= y1; ++y, ++row) {
                        if ((row % W) != wave) continue;
                        const int base = (z * lg.n[1] + y) * lg.n[0];
                        const int t0 = a.cstart[base + x0], t1 = a.cstart[base + x1 + 1];
                        for (int t = t0 + lane; t < t1; t += kTile) {
                            const R4 q = qc[t];
                            if (t != sL) list_contact<R>(a, cd2, pL, q, iL, wbits(q.w) & kIdx);
                        }
                    }
            }
        }
    }
    if (dbg && tid == 0) dbg[2] = wall_clock64();
    if (!RLX && wave == (W > 1 ? 1 : 0)) {  // the noise (depends on the particle and the step only) off wave 0's path
        R n0, n1, n2;
        noise3<R>(a, ctx, i, n0, n1, n2);
        s_noise[lane] = mk4<R>(n0, n1, n2, R(0));
    }
    red[wave][0][lane] = fx;
    red[wave][1][lane] = fy;
    red[wave][2][lane] = fz;
    red[wave][3][lane] = nbr;
    __syncthreads();
    if (dbg && tid == 0) dbg[3] = wall_clock64();

    // 4. integrate (wave 0) / the reactions (waves 1..)
    if (wave == 0) {
        R fsx = red[0][0][lane], fsy = red[0][1][lane], fsz = red[0][2][lane], ns = red[0][3][lane];
#pragma unroll
        for (int w = 1; w < W; ++w) {
            fsx += red[w][0][lane];
            fsy += red[w][1][lane];
            fsz += red[w][2][lane];
            ns += red[w][3][lane];
        }
        const R4 lf = s_locf[lane];
        fsx += lf.x;
        fsy += lf.y;
        fsz += lf.z;
        const R mu = lf.w;
        if constexpr (RLX) {
            // the force for k_lupdate, the drift for the adapted timestep (k_eval64's expression)
            if (act) St<R>::force(a)[s] = mk4<R>(fsx, fsy, fsz, mu);
            const double drift =
                wave_total_max_d(act ? (double)(mu * r_sqrt(fsx * fsx + fsy * fsy + fsz * fsz)) : 0.0);
            const float nfb = (float)__popcll(__ballot(fb));
            double v = 0.0;
            if (flags & kLFlagStats) {
                const R nt = wave_sum_r(act ? ns : R(0));
                if (lane == 6) v = (double)nt;
            }
            if (lane == 8) v = nfb;
            if (lane == kAccDrift) v = drift;
            if (lane == 8 || lane == kAccDrift || ((flags & kLFlagStats) && lane == 6)) acc_fold(acc, lane, v);
        } else {
        // Euler-Maruyama: x += mu dt F + sqrt(2 T mu dt) xi
        const R4 xi = s_noise[lane];
        const R dt = P.timestep;
        const R amp = r_sqrt(R(2) * P.temperature * mu * dt);
        const R mdt = mu * dt;
        const R nxp = pi.x + mdt * fsx + amp * xi.x;
        const R nyp = pi.y + mdt * fsy + amp * xi.y;
        const R nzp = pi.z + mdt * fsz + amp * xi.z;
        if (act) {
            R4* __restrict__ pn = St<R>::pos(a, par ^ 1);  // particle order (see kLFlagPos)
            R4* __restrict__ qn = St<R>::psort(a, par ^ 1);
            if (!a.bslot || (flags & kLFlagPos)) pn[i] = mk4<R>(nxp, nyp, nzp, R(0));
            qn[s] = mk4<R>(nxp, nyp, nzp, pi.w);
            if constexpr (sizeof(R) == 8) {  // the prefilter copy (put_slot's)
                float4* const fn = St<R>::fsort(a, par ^ 1);
                if (fn) fn[s] = make_float4((float)nxp, (float)nyp, (float)nzp, 0.f);
            }
        }
        if constexpr (DOM) {
            if (a.dom_bands) {
                // the fused band pack (k_domain_pack's rule: owned at the step start, old or new position in the
                // peer's region) and the owned shared particles' new positions (k_domain_shared_out's)
                const float ox = (float)pi.x, oy = (float)pi.y, oz = (float)pi.z;
                const float nx = (float)nxp, ny = (float)nyp, nz = (float)nzp;
                if (act && a.dom_shared) {
                    const int k = a.dom_shared[i];
                    if (k > 0) {
                        double* r = a.dom_red + kDomainRed + 3 * (k - 1);
                        r[0] = (double)nxp;
                        r[1] = (double)nyp;
                        r[2] = (double)nzp;
                    }
                }
                R4* const bands = reinterpret_cast<R4*>(a.dom_bands);
                int* const counts = reinterpret_cast<int*>(a.dom_bands);
                const size_t cstride = (size_t)a.dom_bstride * (sizeof(R4) / sizeof(int));  // (ints per band)
                // every peer's ballot first, then one counter atomic per peer, all in flight together (lane p)
                int mine = 0;
                for (int p = 0; p < a.dom_npeer; ++p) {
                    const DomBox r = a.dom_regions[p];
                    const bool send = act && (box_has(r, ox, oy, oz) || box_has(r, nx, ny, nz));
                    const int c = __popcll(__ballot(send));
                    if (lane == p) mine = c;
                }
                int base = 0;
                if (lane < a.dom_npeer && mine > 0) base = atomicAdd(&counts[(size_t)lane * cstride], mine);
                for (int p = 0; p < a.dom_npeer; ++p) {
                    const DomBox r = a.dom_regions[p];
                    const bool send = act && (box_has(r, ox, oy, oz) || box_has(r, nx, ny, nz));
                    const unsigned long long m = __ballot(send);
                    const int at = __shfl(base, p);
                    if (send) {
                        const int o = at + __popcll(m & ((1ull << lane) - 1ull));
                        if (o < a.dom_cap)
                            bands[(size_t)p * a.dom_bstride + 1 + o] = mk4<R>(nxp, nyp, nzp, wpack<R>(i));
                        else
                            atomicOr(a.dom_flags, 2);
                    }
                }
            }
        }
        if (dbg && tid == 0) dbg[4] = wall_clock64();
        // the list bookkeeping in fp32: the displacement from the build and the bbox of the roundings
        const float fnx = (float)nxp, fny = (float)nyp, fnz = (float)nzp;
        const float gx = (float)(nxp - (R)pb.x), gy = (float)(nyp - (R)pb.y), gz = (float)(nzp - (R)pb.z);
        const float dmax = wave_max(act ? sqrtf(fmaf(gz, gz, fmaf(gy, gy, gx * gx))) : 0.f);
        const float nfb = (float)__popcll(__ballot(fb));
        const float nact = DOM ? (float)__popcll(__ballot(act)) : 0.f;  // (ballots outside the lane branches)
        double v = 0.0;  // lane k: the value of accumulator slot k this wave owns
        if (flags & kLFlagStats) {
            const R nt = wave_sum_r(act ? ns : R(0));
            if (lane == 6) v = (double)nt;
        }
        if (flags & kLFlagBBox) {
            const float big = 3.0e38f;
            const float l0 = wave_min(act ? fnx : big), l1 = wave_min(act ? fny : big), l2 = wave_min(act ? fnz : big);
            const float h0 = wave_max(act ? fnx : -big), h1 = wave_max(act ? fny : -big),
                        h2 = wave_max(act ? fnz : -big);
            v = lane == 9 ? l0 : lane == 10 ? l1 : lane == 11 ? l2 : lane == 12 ? h0 : lane == 13 ? h1 : lane == 14 ? h2 : v;
        }
        if (lane == 7) v = dmax;
        if (lane == 8) v = nfb;
        if (DOM && lane == 15) v = nact;
        const bool mine = lane == 7 || lane == 8 || ((flags & kLFlagStats) && lane == 6) ||
                          ((flags & kLFlagBBox) && lane >= 9 && lane < 15) || (DOM && lane == 15);
        if (mine) acc_fold(acc, lane, v);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's accumulator atomics are performed
    __syncthreads();
    if (dbg && tid == 0) dbg[5] = wall_clock64();
    // 5. the two-level ticket (one counter per group of workgroups b % 8, then one over the groups; a single
    // counter serialises ~1000 returning atomics); the final workgroup reads the totals and advances the context
    const int gsize = ((int)gridDim.x - g + ngroups - 1) / ngroups;
    if (tid == 0) {
        const unsigned old = atomicAdd(&a.lticket[32 * g], 1u);
        s_last = (old == (unsigned)gsize - 1) ? 1 : 0;
        if (dbg) {
            dbg[6] = wall_clock64();
            dbg[7] = 0ull;
        }
    }
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) {
        a.lticket[32 * g] = 0u;  // ready for the next launch
        const unsigned old = atomicAdd(&a.lticket[32 * 8], 1u);
        s_final = (old == (unsigned)ngroups - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!s_final) return;
    unsigned long long* const dbt = a.dbg_times ? a.dbg_times + 8 * gridDim.x : nullptr;
    if (dbt && tid == 0) dbt[0] = wall_clock64();
    ListTailIn tin;
    if (!DOM && !RLX && tid == 0) tin = list_tail_load(ctx, a);  // in flight during the accumulator reads
    ListTotals tot;
    list_totals(a.lticket + kListAccBase, ngroups, tot);
    if (tid != 0) return;
    if (dbt) dbt[1] = wall_clock64();
    a.lticket[32 * 8] = 0u;
    if constexpr (RLX) {
        // the force launch's part of the tail: reactions, neighbours, fallbacks, the drift -> the adapted timestep
        for (int k = 0; k < 3; ++k) {
            ctx->react_in[k] = tot.react[k];
            ctx->react_out[k] = tot.react[3 + k];
        }
        if (flags & kLFlagStats) ctx->neighbors = tot.nbr / (double)a.n;
        ctx->lfallback += tot.nfb;
        ctx->max_drift = tot.drift;
        double dt = a.relax_timestep;
        if (a.relax_spacestep > 0.0 && tot.drift * dt > a.relax_spacestep) dt = a.relax_spacestep / tot.drift;
        ctx->dt_used = dt;
        return;
    }
    if constexpr (DOM) {
        // the local reduction (layout kDomainRed); this domain's largest displacement in its own slot
        double* r = a.dom_red;
        for (int k = 0; k < 6; ++k) r[k] = tot.react[k];
        r[6] = tot.nbr;
        r[7] = (double)tot.nown;
        r[8] = (double)tot.nfb;
        r[9] = 0.0;
        for (int q = 0; q < a.dom_ndom; ++q) r[a.dom_dbase + q] = q == a.dom_index ? (double)tot.ld : 0.0;
        if ((flags & kLFlagBBox) && tot.nown > 0)  // the local box of the next build (k_ldom_tail pads it)
            for (int k = 0; k < 3; ++k) {
                ctx->bbox_lo[k] = tot.bb[k];
                ctx->bbox_hi[k] = tot.bb[3 + k];
            }
        return;
    }
    list_tail_apply(ctx, a, tin, tot, flags);
    if (dbg) dbg[7] = wall_clock64();
}

// The relaxation step's update (after k_lstep<..., RLX>): one thread per slot moves its particle with the adapted
// timestep ctx->dt_used, x += mu dt F + sqrt(2 T mu dt) xi (k_update's arithmetic, from the slot-ordered force), into
// both position buffers of the next parity; the largest displacement from the build and, before a rebuild, the
// bounding box go to the launch accumulators, and the final workgroup advances the context (list_tail_apply, with
// the reactions of the force launch).
constexpr int kLUpdateBlock = 256;
template <typename R>
__global__ __launch_bounds__(kLUpdateBlock) void k_lupdate(DevCtx* __restrict__ ctx, ForceArgs a, int flags)
{
    using R4 = real4<R>;
    __shared__ int s_last, s_final;
    const int tid = threadIdx.x, lane = tid & 63;
    const int n = a.n;
    const int s = blockIdx.x * kLUpdateBlock + tid;
    const bool valid = s < n;
    const int sl = valid ? s : n - 1;
    const int par = a.par_hint >= 0 ? a.par_hint : ctx->parity;
    constexpr int kIdx = (1 << kListIndexBits) - 1;
    const R4 pi = St<R>::psort(a, par)[sl];
    const R4 f = St<R>::force(a)[sl];
    const float4 pb = a.spos[sl];
    const int i = wbits(pi.w) & kIdx;
    const R dt = (R)ctx->dt_used;
    R n0, n1, n2;
    noise3<R>(a, ctx, i, n0, n1, n2);
    const R mu = f.w;
    const R amp = r_sqrt(R(2) * St<R>::prm(a).temperature * mu * dt);
    const R mdt = mu * dt;
    const R nxp = pi.x + mdt * f.x + amp * n0;
    const R nyp = pi.y + mdt * f.y + amp * n1;
    const R nzp = pi.z + mdt * f.z + amp * n2;
    if (valid) {
        St<R>::pos(a, par ^ 1)[i] = mk4<R>(nxp, nyp, nzp, R(0));
        put_slot<R>(a, par ^ 1, s, mk4<R>(nxp, nyp, nzp, pi.w));
    }
    // the list bookkeeping in fp32 (as k_lstep's): displacement from the build, bbox of the roundings
    const float fnx = (float)nxp, fny = (float)nyp, fnz = (float)nzp;
    const float gx = (float)(nxp - (R)pb.x), gy = (float)(nyp - (R)pb.y), gz = (float)(nzp - (R)pb.z);
    const float dmax = wave_max(valid ? sqrtf(fmaf(gz, gz, fmaf(gy, gy, gx * gx))) : 0.f);
    const int ngroups = min((int)gridDim.x, 8);
    const int g = blockIdx.x % ngroups;
    unsigned* const acc = a.lticket + kListAccBase + 32 * kAccWords * g;
    double v = lane == 7 ? (double)dmax : 0.0;
    if (flags & kLFlagBBox) {
        const float big = 3.0e38f;
        const float l0 = wave_min(valid ? fnx : big), l1 = wave_min(valid ? fny : big), l2 = wave_min(valid ? fnz : big);
        const float h0 = wave_max(valid ? fnx : -big), h1 = wave_max(valid ? fny : -big), h2 = wave_max(valid ? fnz : -big);
        v = lane == 9 ? l0 : lane == 10 ? l1 : lane == 11 ? l2 : lane == 12 ? h0 : lane == 13 ? h1 : lane == 14 ? h2 : v;
    }
    if (lane == 7 || ((flags & kLFlagBBox) && lane >= 9 && lane < 15)) acc_fold(acc, lane, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's accumulator atomics are performed
    __syncthreads();
    // the two-level ticket (as k_lstep)
    const int gsize = ((int)gridDim.x - g + ngroups - 1) / ngroups;
    if (tid == 0) {
        const unsigned old = atomicAdd(&a.lticket[32 * g], 1u);
        s_last = (old == (unsigned)gsize - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) {
        a.lticket[32 * g] = 0u;
        const unsigned old = atomicAdd(&a.lticket[32 * 8], 1u);
        s_final = (old == (unsigned)ngroups - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!s_final) return;
    ListTailIn tin;
    double react[6];
    if (tid == 0) {
        tin = list_tail_load(ctx, a);
        for (int k = 0; k < 3; ++k) {
            react[k] = ctx->react_in[k];
            react[3 + k] = ctx->react_out[k];
        }
    }
    ListTotals tot;
    list_totals(a.lticket + kListAccBase, ngroups, tot);
    if (tid != 0) return;
    a.lticket[32 * 8] = 0u;
    for (int k = 0; k < 6; ++k) tot.react[k] = react[k];  // (the force launch's; list_tail_apply rewrites them)
    tot.nfb = 0;  // (counted by the force launch)
    list_tail_apply(ctx, a, tin, tot, flags & (kLFlagSched | kLFlagBBox));
}

// ----------------------------------------------------------------------------------------------------
// The persistent small-system step (the mitotic stages: 586 / 1,172 particles; any system of <= kPMax particles).
// At these sizes a step of the list step is ~10-19 workgroups and its cost is latency: a launch, a chain of dependent
// round trips, a cross-workgroup tail (~16 us per step).  Here ONE cooperative launch runs a chunk
// of steps with one workgroup per kPP = 16 particles (4 waves; a wave's 64 lanes are 16 particles x 4 candidate
// segments; all workgroups resident, one per CU by their LDS), and every workgroup holds the WHOLE system's
// positions in LDS:
//   * pairs: all N candidates per particle, a fp32 prefilter on the LDS image (r^2 against rc^2 with a margin that
//     grows with the coordinates' magnitude: every pair within the cutoff in R passes), the hits listed per lane in
//     LDS, then the exact pair in R over the list (list_pair, the list step's arithmetic: the same pair set).  No
//     cell list, no neighbour lists, no rebuilds, no skin: exact at every step by construction;
//   * particle-local terms on the LDS image (local_terms with the image as its positions), on the last wave;
//   * the hand-off, no grid barrier: wave 0 stores each particle's new position as tagged 8-byte granules {data
//     word, tag = step + 1} (16-B sc1 stores, two halves by step parity) together with the workgroup's partial totals
//     (6 wall reactions, the neighbour count); every workgroup loads every granule with sc1 loads and re-polls those
//     whose tag is not yet the step's (MI355X_MICROARCH.md, the tagged-granule hand-off: no fence, no counter).  A
//     half is rewritten two steps later, only after every workgroup has read it;
//   * the tail (reactions -> wall ODE, schedule, step / parity / noise cursor) computed REDUNDANTLY by every
//     workgroup from the totals summed in a fixed workgroup order (every copy the same bits) on its own LDS copy of
//     the context; workgroup 0 writes the context back at the end.
//   * a poll that gives up (pget_image) stops every workgroup and fails the run (ForceArgs::pstall, run_small).
// The force on a particle sums its partners in index order, its lane groups' and waves' sums in a fixed order:
// bitwise reproducible, and independent of how a run is chunked.  The sum order differs from the list step's, so
// the two agree to rounding (tests: both within the oracle's bound).
#ifndef GCS_PSTEP_SPIN
#define GCS_PSTEP_SPIN (1 << 22)  // hand-off polls before a workgroup gives up (ForceArgs::pstall; the host fails the run)
#endif
#ifndef GCS_PSTEP_STALL_TICKS
// ... or wall-clock ticks (100 MHz: 0.25 s) without the granules arriving, whichever comes first.  A step takes ~6 us
// and every workgroup of the cooperative launch is resident, so only a lost hand-off waits that long
#define GCS_PSTEP_STALL_TICKS 25000000ull
#endif
constexpr int kPWaves = 4;
#ifndef GCS_PSTEP_PP
#define GCS_PSTEP_PP 16
#endif
constexpr int kPP = GCS_PSTEP_PP;  // particles per workgroup; a wave's lanes are kPP particles x (64 / kPP) segments
constexpr int kHitCap = 64;      // prefilter hits listed per lane before a flush
// the hand-off (a.psync, zeroed before every launch): two halves, step k writes half k & 1 with tag k + 1.  A half:
// every particle's record (fp64: 3 chunks, fp32: 2), then every workgroup's 8 chunks of partial totals (6 reactions,
// the neighbour count).  A chunk is 16 B = two 8-B granules {data word, tag}: written by one sc1 store, read by sc1
// loads, each granule checked by its own tag (MI355X_MICROARCH.md, the tagged-granule hand-off: no fence, no
// counter, no ordering between granules).  Step k + 2 overwrites half k & 1 only after every workgroup has read it:
// a workgroup writes step k + 2's records after it read all of step k + 1's, which every workgroup wrote after it
// had read step k's.  (Measured and not kept: 16-B chunks of three data words and a check word mixing the tag with
// them -- 2 / 1 chunks a record instead of 3 / 2 -- took 8.0 against 6.9 us per fp64 anatelophase step, same box.)
template <typename R> constexpr int kPRecBytes = sizeof(R) == 8 ? 48 : 32;
// a workgroup's totals: records kPMax + TR g .. (TR = 3 fp64 / 4 fp32 records: 9 / 8 chunks, 7 used, one double each)
template <typename R> constexpr int kPTotRecs = sizeof(R) == 8 ? 3 : 4;
template <typename R> constexpr int kPTotChunks = kPTotRecs<R> * kPRecBytes<R> / 16;
template <typename R> constexpr int kPTotOff = kPMax * kPRecBytes<R>;
template <typename R> constexpr int kPTotBytes = kPTotRecs<R> * kPRecBytes<R>;
constexpr int kPGroups = (kPMax + kPP - 1) / kPP;
static_assert(kPTotOff<double> + kPTotBytes<double> * kPGroups <= kPHalfBytes, "psync half");
static_assert(kPTotOff<float> + kPTotBytes<float> * kPGroups <= kPHalfBytes, "psync half");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t phalf_rsrc(char* half, int bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc((void*)half, 0, bytes, 0x00020000);
}
__device__ __forceinline__ void pput_chunk(char* half, int off, unsigned d0, unsigned d1, unsigned tag)
{
    st_sc1_f4(phalf_rsrc(half, kPHalfBytes), off,
              make_float4(__uint_as_float(d0), __uint_as_float(tag), __uint_as_float(d1), __uint_as_float(tag)));
}
__device__ __forceinline__ void pput_double(char* half, int off, double v, unsigned tag)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    pput_chunk(half, off, (unsigned)b, (unsigned)(b >> 32), tag);
}
template <typename R>
__device__ __forceinline__ void pput_record(char* half, int i, const real4<R>& p, unsigned tag)
{
    const int o = i * kPRecBytes<R>;
    if constexpr (sizeof(R) == 8) {
        pput_double(half, o, p.x, tag);
        pput_double(half, o + 16, p.y, tag);
        pput_double(half, o + 32, p.z, tag);
    } else {
        pput_chunk(half, o, __float_as_uint(p.x), __float_as_uint(p.y), tag);
        pput_chunk(half, o + 16, __float_as_uint(p.z), 0u, tag);
    }
}
__device__ __forceinline__ bool pchunk_ok(const int4& v, unsigned tag)
{
    return (unsigned)v.y == tag && (unsigned)v.w == tag;
}
__device__ __forceinline__ double pchunk_double(const int4& v)
{
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)v.z << 32) | (unsigned)v.x));
}

// the image of step tag and the G workgroups' partial totals: units u < n are the records, u in [n, n + G TR) the
// totals records (record kPMax + u - n); thread t of T walks u = ub + t, ub + t + T, ... < ue, a batch's loads issued
// together, polls until every granule carries the tag; records into s_pos and the fp32 coordinate arrays s_pfx /
// s_pfy / s_pfz, totals chunks (one double each) into s_tot.  A stall -- GCS_PSTEP_SPIN polls or
// GCS_PSTEP_STALL_TICKS of wall clock without the granules, or the global stall word set by another workgroup (read
// every 64 polls) -- sets the workgroup's stall flag (its step loop then stops) and adds 1 to the global word (the
// other workgroups stop at their next poll; engine.hip run_small fails the run and restores the context)
template <typename R, typename Mid>
__device__ __forceinline__ void pget_image(char* half, int n, int G, int ub, int ue, int t, int T, unsigned tag, real4<R>* s_pos,
                                           float* s_pfx, float* s_pfy, float* s_pfz, double* s_tot,
                                           volatile int* stall, int* gstall, Mid&& mid, unsigned long long* dbg = nullptr)
{
    // mid(): work of the caller's that runs while the first batch's loads are in flight
    constexpr int C = sizeof(R) == 8 ? 3 : 2, RB = sizeof(R) == 8 ? 4 : 6, RBY = kPRecBytes<R>;
    const auto rp = phalf_rsrc(half, kPHalfBytes);
    auto rec = [&](int u) { return u < n ? u : kPMax + (u - n); };
    for (int u0 = ub; u0 < ue; u0 += RB * T) {
        int4 v[RB][C];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int u = u0 + t + r * T;
#pragma unroll
            for (int c = 0; c < C; ++c) v[r][c] = u < ue ? ld_sc1_i4(rp, rec(u) * RBY + 16 * c) : int4{};
        }
        if (u0 == ub) mid();
        unsigned long long t0 = 0ull;
        for (int spin = 0;; ++spin) {
            bool ok = true;
#pragma unroll
            for (int r = 0; r < RB; ++r)
#pragma unroll
                for (int c = 0; c < C; ++c) ok = ok && (u0 + t + r * T >= ue || pchunk_ok(v[r][c], tag));
            if (dbg && u0 == ub) {
                if (spin == 0) dbg[0] = wall_clock64();
                dbg[1] = spin;
            }
            if (ok) break;
            if (*stall) break;
            if ((spin & 63) == 0) {
                const unsigned long long now = wall_clock64();
                if (spin == 0) t0 = now;
                if (__hip_atomic_load(gstall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    *stall = 1;
                    break;
                }
                if (spin >= GCS_PSTEP_SPIN || now - t0 > GCS_PSTEP_STALL_TICKS) {
                    *stall = 1;
                    atomicAdd(gstall, 1);
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(1);  // (longer backoffs measured slower: 2 / 4 / 8 x 64 clocks)
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int u = u0 + t + r * T;
#pragma unroll
                for (int c = 0; c < C; ++c)
                    if (u < ue && !pchunk_ok(v[r][c], tag)) v[r][c] = ld_sc1_i4(rp, rec(u) * RBY + 16 * c);
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const int u = u0 + t + r * T;
            if (u < n) {
                real4<R> p;
                if constexpr (sizeof(R) == 8) {
                    p = mk4<R>(pchunk_double(v[r][0]), pchunk_double(v[r][1]), pchunk_double(v[r][2]), R(0));
                } else {
                    p = mk4<R>(__int_as_float(v[r][0].x), __int_as_float(v[r][0].z), __int_as_float(v[r][1].x), R(0));
                }
                s_pos[u] = p;
                s_pfx[u] = (float)p.x;
                s_pfy[u] = (float)p.y;
                s_pfz[u] = (float)p.z;
            } else if (u < ue) {
#pragma unroll
                for (int c = 0; c < C; ++c) s_tot[(u - n) * C + c] = pchunk_double(v[r][c]);
            }
        }
    }
}

constexpr int kPDbgSteps = 32;  // GCS_DEBUG_PSTEP: the steps stamped (the first of the launch)
template <typename R>
__global__ __launch_bounds__(64 * kPWaves) void k_pstep(DevCtx* __restrict__ ctx, ForceArgs a, int steps, int flags)
{
    using R4 = real4<R>;
    using R2 = real2<R>;
    constexpr int W = kPWaves;
    __shared__ R4 s_pos[kPMax];      // every particle's position at the step start (particle order)
    // its fp32 rounding (the prefilter), by coordinate (a b128 read: 4 candidates; padded for the last chunk's reads)
    __shared__ __attribute__((aligned(16))) float s_pfx[kPMax + 32], s_pfy[kPMax + 32], s_pfz[kPMax + 32];
    __shared__ R2 s_ab[kPMax];       // its pair factors (a, b)
    constexpr int Q = kTile / kPP;   // candidate segments per wave (lane group q = lane / kPP)
    __shared__ R red[W][4][kTile];
    __shared__ R4 s_locf[kPP], s_noise[2][kPP];  // (the noise by step parity: the next step's is made early)
    __shared__ int s_stall;
    __shared__ unsigned long long s_dbg[kPDbgSteps][16], s_dbw[kPDbgSteps];  // GCS_DEBUG_PSTEP stamps
    __shared__ double s_react[6];  // the workgroup's wall reactions of the step (wave W - 1 -> wave 0)
    __shared__ double s_tot[kPGroups * kPTotChunks<R>];  // the step's partial totals, by workgroup
    __shared__ DevCtx s_ctx;
    __shared__ unsigned short s_hit[kPWaves][kHitCap][kTile];  // per wave: each lane's prefilter hits (column)
    // (fp32: pad the workgroup beyond half a CU's LDS -- one workgroup per CU, the hand-off's validated form)
    __shared__ char s_pad[sizeof(R) == 4 ? 32 * 1024 : 16];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uniform(tid >> 6);
    const int n = a.n;
    const int G = gridDim.x;
    const int pl = lane & (kPP - 1), lq = lane / kPP;
    const int i = blockIdx.x * kPP + pl;
    const bool valid = i < n;
    const bool lead = valid && lq == 0;  // the lane that stores / folds particle i (the others hold copies)
    const int il = valid ? i : n - 1;
    unsigned* const sync = a.psync;  // the hand-off halves
    if (tid == 0) {
        s_pad[0] = 0;
        // an earlier launch of the run stalled: do nothing (the host restores the context of that launch's start)
        s_stall = __hip_atomic_load(a.pstall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ? 1 : 0;
    }
    const FieldPrm<R>& P = St<R>::prm(a);
    const R4* __restrict__ kmu = St<R>::kmu(a);

    // launch start: the context, the pair factors and the run's positions (earlier launches wrote them: the launch
    // boundary orders them), the particle's constants for every step
    if (tid == 0) s_ctx = *ctx;
    for (int j = tid; j < n; j += blockDim.x) {
        const R4 k = kmu[j];
        R2 t;
        t.x = a.pair_mix ? k.y : R(1);
        t.y = a.pair_mix ? k.z : R(0);
        s_ab[j] = t;
    }
    __syncthreads();
    int par = s_ctx.parity;
    for (int j = tid; j < n; j += blockDim.x) {
        const R4 p = St<R>::pos(a, par)[j];
        s_pos[j] = p;
        s_pfx[j] = (float)p.x;
        s_pfy[j] = (float)p.y;
        s_pfz[j] = (float)p.z;
    }
    R4 km = mk4<R>(R(0), R(0), R(0), R(0));
    int2 erow = make_int2(0, 0);
    LocalPre<R> pre{};
    if (wave == W - 1) {
        km = kmu[il];
        erow = a.has_bonds ? make_int2(a.boff[il], a.boff[il + 1]) : make_int2(0, 0);
        // this lane's constants of the particle-local terms for the whole launch (local_terms, LocalPre)
        const int qb = erow.x + lq;
        pre.enb = qb < erow.y ? a.bent[qb] : make_int2(il, 0);
        pre.bv = qb < erow.y ? St<R>::bval(a)[qb] : mk4<R>(R(0), R(0), R(0), R(0));
        pre.beps = (a.has_bend && lq < 3 && il - lq >= 0 && il - lq + 2 < n) ? St<R>::bend(a)[il - lq] : R(0);
        pre.tb = a.has_tether ? a.toff[il] : 0;
        pre.te = a.has_tether ? a.toff[il + 1] : 0;
        if (pre.tb + lq < pre.te) pre.tt = St<R>::tent(a)[pre.tb + lq];
    }
    const R2 own = s_ab[il];  // (s_ab was filled before the barrier above)
    // this lane's candidates [cj0, cj1): the wave's share of the candidates in 1/64, split evenly over its Q lane
    // groups.  The local-terms wave (W - 1) takes a share that grows with n from none at ~600 particles (its terms
    // then take about as long as the others' pairs: 2.6 us against ~3.1 us at 586) to 4/64 at ~1,100 (3.8 us
    // against ~5.7 at 1,172), waves 0..2 split the rest.  Static: the sum order is the same at every step and chunk.
    int cj0, cj1;
    {
        static_assert(kPWaves == 4, "four waves");
        const int s3 = min(8, max(0, (n - 600) / 128));
        const int rest = 64 - s3;
        int sh[4] = {rest / 3 + (rest % 3 > 0), rest / 3 + (rest % 3 > 1), rest / 3, s3};
        int b = 0;
        for (int w = 0; w < wave; ++w) b += sh[w];
        cj0 = (int)((long long)n * (b * Q + lq * sh[wave]) / (64 * Q));
        cj1 = (int)((long long)n * (b * Q + (lq + 1) * sh[wave]) / (64 * Q));
    }

    for (int k = 0; k < steps; ++k) {
        __syncthreads();  // s_pos / s_pf* of this step, s_ctx
        if (s_stall) break;  // a hand-off stalled (this workgroup or another): stop integrating
        const unsigned tag = (unsigned)k + 1u;  // step k's hand-off: half k & 1, tag k + 1
        char* const half = reinterpret_cast<char*>(sync) + (k & 1) * kPHalfBytes;
        // debug stamps (GCS_DEBUG_PSTEP): workgroup 0's phases of the first 64 steps ([16 k ...]), every workgroup's
        // hand-off time ([1024 + 128 k + workgroup])
        // (kept in LDS and written out at the end: a global store would hold the storing wave's next vmcnt wait)
        unsigned long long* const dbs = (a.dbg_times && blockIdx.x == 0 && k < kPDbgSteps) ? s_dbg[k] : nullptr;
        unsigned long long* const dbw = (a.dbg_times && k < kPDbgSteps) ? &s_dbw[k] : nullptr;
        if (dbs && tid == 0) dbs[0] = wall_clock64();
        const long long c_step = s_ctx.step, c_cursor = s_ctx.noise_cursor;  // (the tail advances s_ctx mid-step)
        const R4 pi = s_pos[il];
        const R cs = (R)s_ctx.cs;
        const R scale = a.pair_scaled ? cs : R(1);
        const R sa = P.pa_sig * scale, sbb = P.pb_sig * scale;
        const R k2a = R(1) / (sa * sa), k2b = R(1) / (sbb * sbb);
        const R kA = R(0.5) * R(6) * P.pa_eps * k2a, kB = R(0.5) * R(24) * P.pb_eps * k2b;
        const R rc = pair_cutoff_r<R>(a, (double)cs), rc2 = rc * rc;
        const R ahi = kA * own.x, bhi = kB * own.y;

        if (k == 0 && wave == 1) {  // the first step's noise (the later steps': while the previous hand-off lands)
            R n0, n1, n2;
            noise3<R>(a, &s_ctx, il, n0, n1, n2);
            if (lq == 0) s_noise[0][pl] = mk4<R>(n0, n1, n2, R(0));
        }
        // the particle-local terms first on the last wave (image positions); the workgroup's reaction partials out
        if (wave == W - 1) {
            R lfx = 0, lfy = 0, lfz = 0, en[kEnergyKinds];
            R rin[3] = {0, 0, 0}, rout[3] = {0, 0, 0};
            local_terms<kModeStep, 1, R, true>(&s_ctx, a, il, pi.x, pi.y, pi.z, km, lfx, lfy, lfz, en, rin, rout, erow,
                                               s_pos, lq, Q, &pre);
#pragma unroll
            for (int o = kPP; o < kTile; o <<= 1) {  // the lane groups' shares, in a fixed order
                lfx += __shfl_down(lfx, o);
                lfy += __shfl_down(lfy, o);
                lfz += __shfl_down(lfz, o);
            }
            if (lq == 0) s_locf[pl] = mk4<R>(lfx, lfy, lfz, km.x);
            R rv = 0;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                const R x = wave_sum_r(lead ? (c < 3 ? rin[c] : rout[c - 3]) : R(0));
                if (lane == c) rv = x;
            }
            // (published by wave 0 with its hand-off: a store here would hold this wave's next vmcnt wait -- loads
            // and stores share the counter -- until the write-through store is acknowledged, ~1 us)
            if (lane < 6) s_react[lane] = (double)rv;
            if (dbs && lane == 0) dbs[1] = wall_clock64();
        }

        // pairs: this wave's share of the candidates (the local-terms wave a smaller one), 32 at a time through the
        // fp32 prefilter; each lane appends its hits (ascending index) to its column of the wave's hit list, and the
        // exact pairs in R run over the list -- wave-max(hits) iterations instead of one per hit of the chunk's
        // densest lane, chunk after chunk (the candidates of a chunk are a chain segment: its hits bunch on a few
        // lanes).  A list that could overflow is flushed first.
        R fx = 0, fy = 0, fz = 0, nbr = 0;
        if (a.has_pair) {
            const float pxf = (float)pi.x, pyf = (float)pi.y, pzf = (float)pi.z;
            // margin against the fp32 roundings: a coordinate's rounding is <= 2^-24 |x|, so for a pair within rc
            // (|x_j| <= |x_i| + rc) r^2 moves by <= ~4.2e-7 rc (mag + rc), mag = the particle's largest |coordinate|;
            // the margin keeps 2x that on top of 0.1 % of rc^2 (the fixed margin held to |x| ~ 400 only)
            const float mag = fmaxf(fabsf(pxf), fmaxf(fabsf(pyf), fabsf(pzf)));
            const float thr = (float)rc2 * 1.001f + 1.0e-4f * (float)rc + 1.0e-6f * (float)rc * (mag + (float)rc);
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 PX = {pxf, pxf}, PY = {pyf, pyf}, PZ = {pzf, pzf};
            unsigned short* const hl = &s_hit[wave][0][0];
            int cnt = 0;
            auto flush = [&]() {
                const int kmax = uniform(wave_max_int(cnt));
                for (int q = 0; q < kmax; ++q) {
                    const bool real = q < cnt;
                    const int j = real ? hl[q * kTile + lane] : il;
                    list_pair<R>(pi.x, pi.y, pi.z, s_pos[j], s_ab[j], ahi, bhi, kA, kB, k2a, k2b, rc2, real, fx, fy,
                                 fz, nbr);
                }
                cnt = 0;
            };
            const float4* const X4 = reinterpret_cast<const float4*>(s_pfx);
            const float4* const Y4 = reinterpret_cast<const float4*>(s_pfy);
            const float4* const Z4 = reinterpret_cast<const float4*>(s_pfz);
            // chunks from cj0 rounded down to 4 (b128 reads of 4 candidates a coordinate; the 16 candidates of a half
            // chunk loaded together), the candidates outside [cj0, cj1) masked
            for (int c0 = cj0 < cj1 ? (cj0 & ~3) : cj1; c0 < cj1; c0 += 32) {  // (an empty share: no chunk)
                unsigned m = 0u;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    float4 X[4], Y[4], Z[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int q = (c0 >> 2) + 4 * hh + g;
                        X[g] = X4[q];
                        Y[g] = Y4[q];
                        Z[g] = Z4[q];
                    }
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const f2 dx0 = f2{X[g].x, X[g].y} - PX, dx1 = f2{X[g].z, X[g].w} - PX;
                        const f2 dy0 = f2{Y[g].x, Y[g].y} - PY, dy1 = f2{Y[g].z, Y[g].w} - PY;
                        const f2 dz0 = f2{Z[g].x, Z[g].y} - PZ, dz1 = f2{Z[g].z, Z[g].w} - PZ;
                        const f2 r0 = __builtin_elementwise_fma(dz0, dz0, __builtin_elementwise_fma(dy0, dy0, dx0 * dx0));
                        const f2 r1 = __builtin_elementwise_fma(dz1, dz1, __builtin_elementwise_fma(dy1, dy1, dx1 * dx1));
                        const int b = 16 * hh + 4 * g;
                        m |= (r0.x < thr ? 1u : 0u) << b;
                        m |= (r0.y < thr ? 1u : 0u) << (b + 1);
                        m |= (r1.x < thr ? 1u : 0u) << (b + 2);
                        m |= (r1.y < thr ? 1u : 0u) << (b + 3);
                    }
                }
                if (c0 < cj0) m &= ~((1u << (cj0 - c0)) - 1u);
                const int rem = cj1 - c0;
                if (rem < 32) m &= (1u << rem) - 1u;
                if ((unsigned)(i - c0) < 32u) m &= ~(1u << (i - c0));  // not itself
                if (!valid) m = 0u;
                if (__ballot(cnt + __popc(m) > kHitCap)) flush();
                while (m) {
                    hl[cnt * kTile + lane] = (unsigned short)(c0 + __ffs(m) - 1);
                    ++cnt;
                    m &= m - 1u;
                }
            }
            if (dbs && lane == 0 && wave == 0) dbs[8] = wall_clock64();
            flush();
        }
        if (dbs && lane == 0) dbs[wave == 0 ? 2 : 8 + wave] = wall_clock64();
        // the lane groups' sums in a fixed order ((q0 + q1) + (q2 + q3)), lanes of group 0 keep them
#pragma unroll
        for (int o = kPP; o < kTile; o <<= 1) {
            fx += __shfl_down(fx, o);
            fy += __shfl_down(fy, o);
            fz += __shfl_down(fz, o);
            nbr += __shfl_down(nbr, o);
        }
        if (lq == 0) {
            red[wave][0][pl] = fx;
            red[wave][1][pl] = fy;
            red[wave][2][pl] = fz;
            red[wave][3][pl] = nbr;
        }
        __syncthreads();

        if (wave == 0) {
            // integrate: the new position (the waves' sums in wave order), handed off as tagged granules
            R fsx = red[0][0][pl], fsy = red[0][1][pl], fsz = red[0][2][pl], ns = red[0][3][pl];
#pragma unroll
            for (int w = 1; w < W; ++w) {
                fsx += red[w][0][pl];
                fsy += red[w][1][pl];
                fsz += red[w][2][pl];
                ns += red[w][3][pl];
            }
            if (dbs && lane == 0) dbs[13] = wall_clock64();
            // the workgroup's totals out first (wave 0 of every workgroup waits on them before its tail), then the
            // records
            const R nt = wave_sum_r(lead ? ns : R(0));
            const bool pub = a.pstep_skip < 0 || a.pstep_skip != (int)((blockIdx.x << 16) | (unsigned)k);  // (tests)
            if (pub && lane < kPTotChunks<R>)  // reactions, neighbours (the unused chunks tagged too: all are polled)
                pput_double(half, kPTotOff<R> + blockIdx.x * kPTotBytes<R> + 16 * lane,
                            lane < 6 ? s_react[min(lane, 5)] : lane == 6 ? (double)nt : 0.0, tag);
            const R4 lf = s_locf[pl];
            fsx += lf.x;
            fsy += lf.y;
            fsz += lf.z;
            const R mu = lf.w;
            const R4 xi = s_noise[k & 1][pl];
            const R dt = P.timestep;
            const R amp = r_sqrt(R(2) * P.temperature * mu * dt);
            const R mdt = mu * dt;
            const R4 np = mk4<R>(pi.x + mdt * fsx + amp * xi.x, pi.y + mdt * fsy + amp * xi.y,
                                 pi.z + mdt * fsz + amp * xi.z, R(0));
            if (lead && pub) {
                pput_record<R>(half, i, np, tag);
                if (k == steps - 1) St<R>::pos(a, par ^ 1)[i] = np;  // the launch's result (the launch end orders it)
            }
            if (dbs && lane == 0) dbs[14] = wall_clock64();
            if (dbs && lane == 0) dbs[3] = wall_clock64();
            if (dbw && lane == 0) *dbw = wall_clock64();
        }
        // the next step's image (waves 1..) and every workgroup's partial totals (wave 0), from the granules: wave 0
        // sums the totals and runs the tail while the image lands; wave 1 makes the next step's noise (the particle
        // and the step only: the step and cursor as of the step start, the tail may advance the context meanwhile)
        // while its first loads are in flight
        if (wave > 0) {
            pget_image<R>(half, n, G, 0, n, tid - 64, 64 * (W - 1), tag, s_pos, s_pfx, s_pfy, s_pfz, s_tot, &s_stall,
                          a.pstall, [&]() {
                if (wave == 1 && k + 1 < steps) {
                    R n0, n1, n2;
                    noise3_at<R>(a, c_step + 1, c_cursor + 1, il, n0, n1, n2);
                    if (lq == 0) s_noise[(k + 1) & 1][pl] = mk4<R>(n0, n1, n2, R(0));
                }
            });
            if (dbs && tid == 64) dbs[12] = wall_clock64();
        } else {
            ListTailIn tin;
            TailSched tsc;
            if (tid == 0) {  // the tail's inputs and the schedule's closed forms: they need no totals
                tin = list_tail_load(&s_ctx, a);
                tsc = list_tail_sched(tin);
            }
            pget_image<R>(half, n, G, n, n + G * kPTotRecs<R>, lane, 64, tag, s_pos, s_pfx, s_pfy, s_pfz, s_tot,
                          &s_stall, a.pstall, [] {}, dbs && tid == 0 ? dbs + 4 : nullptr);
            // the step's totals, in a fixed order (the same totals in every workgroup, bitwise): lane 8 c + p sums
            // quantity c over workgroups p, p + 8, ..., then the 8 lanes of c pairwise (this wave's own LDS writes)
            const int tc = lane >> 3, tp = lane & 7;
            double s = 0.0;
            if (tc < 7)
                for (int g = tp; g < G; g += 8) s += s_tot[g * kPTotChunks<R> + tc];
            s += __shfl_xor(s, 1);
            s += __shfl_xor(s, 2);
            s += __shfl_xor(s, 4);
            double tot[7];
#pragma unroll
            for (int c = 0; c < 7; ++c) tot[c] = __shfl(s, 8 * c);
            if (dbs && lane == 0) dbs[7] = wall_clock64();
            ListTotals t;
            for (int c = 0; c < 6; ++c) t.react[c] = tot[c];
            t.nbr = tot[6];
            t.ld = 0.f;
            t.nfb = 0;
            t.nown = 0;
            for (int c = 0; c < 6; ++c) t.bb[c] = 0.f;
            t.drift = 0.0;
            if (tid == 0) {
                list_tail_apply(&s_ctx, a, tin, t, flags | (k == steps - 1 ? kLFlagStats : 0), &tsc);
                if (dbs) dbs[6] = wall_clock64();
            }
        }
        par ^= 1;
    }
    __syncthreads();
    if (a.dbg_times && tid < kPDbgSteps) {  // the stamps: workgroup 0's phases, every workgroup's hand-off
        if (blockIdx.x == 0)
            for (int c = 0; c < 16; ++c) a.dbg_times[16 * tid + c] = tid < steps ? s_dbg[tid][c] : 0ull;
        if (blockIdx.x < 128) a.dbg_times[1024 + 128 * tid + blockIdx.x] = tid < steps ? s_dbw[tid] : 0ull;
    }
    __syncthreads();
    // the context of a stalled launch is not written back (the host fails the run either way)
    if (blockIdx.x == 0 && tid == 0 && !s_stall) *ctx = s_ctx;
}

// run_small's guard around each k_pstep launch: before it (save) the context is kept unless a launch of the run has
// stalled already; after the run (restore) a stalled run gets back the context of its failing launch's start (whose
// position buffer that launch never writes: it writes the other parity)
__global__ void k_pstep_guard(DevCtx* __restrict__ ctx, DevCtx* __restrict__ keep, const int* __restrict__ stall,
                              int restore)
{
    constexpr int kWords = (int)(sizeof(DevCtx) / sizeof(int));
    static_assert(sizeof(DevCtx) % sizeof(int) == 0, "DevCtx in words");
    const bool stalled = *stall != 0;
    int* const dst = reinterpret_cast<int*>(restore ? ctx : keep);
    const int* const src = reinterpret_cast<const int*>(restore ? keep : ctx);
    if (restore ? stalled : !stalled)
        for (int w = threadIdx.x; w < kWords; w += blockDim.x) dst[w] = src[w];
}

// The decomposed list step's tail (one workgroup, after the allreduce of every domain's k_lstep<..., DOM> reduction):
// the same context update as the undecomposed step's final workgroup from the global sums (reactions, neighbours,
// fallbacks) and the largest of the domains' displacement slots; the next build's grid is this domain's owned bbox
// padded by the halo (ghosts beyond it are clamped into the edge cells, which is still exact).  Checks: every
// particle owned by some domain's lists (kDomFlagLost), cutoff + largest displacement within the halo
// (kDomFlagMotion).  Then the shared particles' allreduced positions into both buffers, by index and by slot, and the
// send bands' header rows zeroed for the pack.
// the grid k_ldom_tail computes before a rebuild (ctx->bbox: this domain's owned box at its last bounding-box step,
// padded by the binning halo; any box is exact, particles outside it are clamped into the border cells), for a
// skin that changed since
__global__ void k_dom_grid(DevCtx* __restrict__ ctx, ForceArgs a)
{
    float bb[6];
    for (int k = 0; k < 3; ++k) {
        bb[k] = ctx->bbox_lo[k] - a.dom_bin_halo;
        bb[3 + k] = ctx->bbox_hi[k] + a.dom_bin_halo;
    }
    ctx->grid = make_grid(bb, bb + 3, pair_cutoff(a, ctx->cs) + a.list_skin, a.ncell_max, kPairFx);
}

// the tail of a decomposed list step from the allreduced buffer glob (thread tid of nt >= 1 in one workgroup; the
// context by thread 0): the undecomposed tail arithmetic on the global sums, the checks, the shared particles in
// (by index and slot), the send bands' headers zeroed (bands != nullptr), the shared block of the reduction buffer
// zeroed for the next step's owners
template <typename R>
__device__ __forceinline__ void ldom_tail_body(DevCtx* __restrict__ ctx, const ForceArgs& a, const double* __restrict__ glob,
                                               int flags, const int* __restrict__ shared, int nshared,
                                               real4<R>* __restrict__ bands, int npeer, int bstride, int tid, int nt)
{
    if (tid == 0) {
        const ListTailIn tin = list_tail_load(ctx, a);
        ListTotals t;
        for (int k = 0; k < 6; ++k) t.react[k] = glob[k];
        t.nbr = glob[6];
        const long long nown = (long long)glob[7];
        t.nfb = (long long)glob[8];
        t.nown = nown;
        float ld = 0.f;
        for (int q = 0; q < a.dom_ndom; ++q) ld = fmaxf(ld, (float)glob[a.dom_dbase + q]);
        t.ld = ld;
        for (int k = 0; k < 3; ++k) {
            t.bb[k] = ctx->bbox_lo[k] - a.dom_bin_halo;
            t.bb[3 + k] = ctx->bbox_hi[k] + a.dom_bin_halo;
        }
        list_tail_apply(ctx, a, tin, t, flags);
        int fl = nown != (long long)a.n ? kDomFlagLost : 0;
        if (pair_cutoff(a, ctx->cs) + ld > a.dom_bin_halo) fl |= kDomFlagMotion;
        if (fl) atomicOr(a.dom_flags, fl);
    }
    constexpr int kIdx = (1 << kListIndexBits) - 1;
    for (int k = tid; k < nshared; k += nt) {
        const int i = shared[k];
        const R x = (R)glob[kDomainRed + 3 * k], y = (R)glob[kDomainRed + 3 * k + 1], z = (R)glob[kDomainRed + 3 * k + 2];
        St<R>::pos(a, 0)[i] = mk4<R>(x, y, z, R(0));
        St<R>::pos(a, 1)[i] = mk4<R>(x, y, z, R(0));
        const int sl = a.islot[i];
        if (sl >= 0) {
            const real4<R> q = mk4<R>(x, y, z, wpack<R>((i & kIdx) | (a.ptype[i] << kListIndexBits)));
            put_slot<R>(a, 0, sl, q);
            put_slot<R>(a, 1, sl, q);
        }
    }
    if (bands)
        for (int p = tid; p < npeer; p += nt) bands[(size_t)p * bstride] = mk4<R>(R(0), R(0), R(0), R(0));
    // the shared block of this domain's reduction buffer for the next step's owners (the fused pack writes only
    // the owned particles' rows; the allreduce of this step has consumed it)
    if (a.dom_red)
        for (int k = tid; k < 3 * nshared; k += nt) a.dom_red[kDomainRed + k] = 0.0;
}

template <typename R>
__global__ __launch_bounds__(64) void k_ldom_tail(DevCtx* __restrict__ ctx, ForceArgs a, const double* __restrict__ glob,
                                                  int flags, const int* __restrict__ shared, int nshared,
                                                  real4<R>* __restrict__ bands, int npeer, int bstride)
{
    ldom_tail_body<R>(ctx, a, glob, flags, shared, nshared, bands, npeer, bstride, threadIdx.x, blockDim.x);
}

// The engine-issued RCCL list step's finish after BOTH collectives (the band exchange does not depend on the tail,
// only the next step does): workgroup 0's first wave runs the tail, every thread of every workgroup unpacks the
// received bands (k_domain_unpack's scatter, slots on) -- one launch per step instead of two.  The tail's shared
// particles and a band record of the same particle carry the same new position, so their order does not matter.
template <typename R>
__global__ __launch_bounds__(256) void k_ldom_finish(DevCtx* __restrict__ ctx, ForceArgs a, const double* __restrict__ glob,
                                                     int flags, const int* __restrict__ shared, int nshared,
                                                     const real4<R>* __restrict__ in, const int* __restrict__ counts,
                                                     int nbuf, int cap, int istride, int cstride,
                                                     real4<R>* __restrict__ send, int nsend, int sstride)
{
    if (blockIdx.x == 0 && threadIdx.x < 64)
        ldom_tail_body<R>(ctx, a, glob, flags, shared, nshared, send, nsend, sstride, threadIdx.x, 64);
    dom_unpack_records<R>(a, in, counts, nbuf, cap, istride, cstride, 1, blockIdx.x * blockDim.x + threadIdx.x,
                          gridDim.x * blockDim.x);
}

// ----------------------------------------------------------------------------------------------------
// neighbor search (contact map / md::neighbor_searcher): strict fp32 predicate, pairs i < j

__device__ inline bool strict_pair(float4 p, float4 q, float rc2)
{
    const float dx = __fsub_rn(p.x, q.x), dy = __fsub_rn(p.y, q.y), dz = __fsub_rn(p.z, q.z);
    const float r2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
    return r2 < rc2;
}

// F64: the predicate in fp64 on pos64 (the fp64 engine's positions, or fp64 query points) with d2 = d64 * d64; the
// cells (fp32 roundings, edge >= distance * (1 + 1e-4)) still hold every candidate
template <bool EMIT, bool F64>
__global__ __launch_bounds__(256) void k_search(const DevCtx* __restrict__ ctx, int n, const float4* __restrict__ spos,
                                                const int* __restrict__ sidx, const int* __restrict__ scell,
                                                const int* __restrict__ cstart, int* __restrict__ counts,
                                                const int* __restrict__ offsets, unsigned long long* __restrict__ keys,
                                                const double4* __restrict__ pos64, double d64)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const Grid g = ctx->grid;
    const float rc2 = __fmul_rn(g.rc, g.rc);
    const double d2 = __dmul_rn(d64, d64);
    const int i = sidx[s];
    const float4 p = spos[s];
    double4 p64 = make_double4(0.0, 0.0, 0.0, 0.0);
    if constexpr (F64) p64 = pos64[i];
    const int c = scell[s];
    const int nx = g.n[0], ny = g.n[1], nz = g.n[2];
    const int cx = c % nx, cy = (c / nx) % ny, cz = c / (nx * ny);
    int cnt = 0;
    long long o = EMIT ? offsets[s] : 0;
    for (int z = max(cz - 1, 0); z <= min(cz + 1, nz - 1); ++z)
        for (int y = max(cy - 1, 0); y <= min(cy + 1, ny - 1); ++y) {
            const int base = (z * ny + y) * nx;
            const int jb = cstart[base + max(cx - g.fx, 0)], je = cstart[base + min(cx + g.fx, nx - 1) + 1];
            for (int t = jb; t < je; ++t) {
                const int j = sidx[t];
                if (j <= i) continue;
                if constexpr (F64) {
                    const double4 q = pos64[j];
                    if (!strict_lt(p64.x, p64.y, p64.z, q.x, q.y, q.z, d2)) continue;
                } else {
                    if (!strict_pair(p, spos[t], rc2)) continue;
                }
                if (EMIT) keys[o++] = ((unsigned long long)(unsigned)i << 32) | (unsigned)j;
                cnt++;
            }
        }
    if (!EMIT) counts[s] = cnt;
}

__global__ __launch_bounds__(1024) void k_scan_small(const int* __restrict__ in, int* __restrict__ out, int n,
                                                     int* __restrict__ total)
{
    __shared__ int wtot[16];
    const int T = blockDim.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + T - 1) / T;
    const int b = min(n, tid * per), e = min(n, b + per);
    int sum = 0;
    for (int k = b; k < e; ++k) sum += in[k];
    int incl = wave_incl_scan(sum, lane);
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    if (wave == 0) {
        int v = (lane < T / 64) ? wtot[lane] : 0;
        int vi = wave_incl_scan(v, lane);
        if (lane < T / 64) wtot[lane] = vi - v;
        if (lane == T / 64 - 1) *total = vi;
    }
    __syncthreads();
    int run = wtot[wave] + incl - sum;
    for (int k = b; k < e; ++k) {
        int c = in[k];
        out[k] = run;
        run += c;
    }
}


// ----------------------------------------------------------------------------------------------------
// fp64 force / energy evaluation (GCS_PRECISION_F64: md::system::compute_energy / the force pass of a spacestep
// relaxation step, simulation_driver_relaxation.cpp:48-55, and gcs_engine_compute_forces).  Not on the fixed-timestep
// step path (that is k_lstep<..., double>), so it is written for clarity: one thread per cell-sorted slot, a gather
// of every candidate of the 3 x 3 neighbouring cell rows (x within +-fx cells) by particle index, the pair potential
// in fp64 with the pair's mean (a, b) factors, then the fp64 particle-local terms.  Partial rows per block are
// reduced in a fixed order (k_red64 / the host): bitwise reproducible.
constexpr int kEval64Block = 256;

template <int MODE>
__global__ __launch_bounds__(kEval64Block) void k_eval64(const DevCtx* __restrict__ ctx, ForceArgs a)
{
    __shared__ double s_red[kEnergyKinds][kEval64Block / 64];
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const Grid g = ctx->grid;
    const bool valid = s < a.n && s < a.cstart[g.ncell];
    const int sl = valid ? s : 0;
    const int i = a.sidx[sl];
    const double4* __restrict__ pos = St<double>::pos(a, ctx->parity);
    const double4 p = pos[i];
    const double4 km = a.dkmu[i];
    const FieldPrm<double>& P = a.pd;
    double fx = 0, fy = 0, fz = 0, ep = 0, nbr = 0;
    if (valid && a.has_pair) {
        const double cs = ctx->cs;
        const double scale = a.pair_scaled ? cs : 1.0;
        const double sa = P.pa_sig * scale, sbb = P.pb_sig * scale;
        const double k2a = 1.0 / (sa * sa), k2b = 1.0 / (sbb * sbb);
        const double rc = pair_cutoff_r<double>(a, cs), rc2 = rc * rc;
        const double ai = a.pair_mix ? km.y : 1.0, bi = a.pair_mix ? km.z : 0.0;
        const int c = a.scell[s];
        const int nx = g.n[0], ny = g.n[1], nz = g.n[2];
        const int cx = c % nx, cy = (c / nx) % ny, cz = c / (nx * ny);
        for (int z = max(cz - 1, 0); z <= min(cz + 1, nz - 1); ++z)
            for (int y = max(cy - 1, 0); y <= min(cy + 1, ny - 1); ++y) {
                const int base = (z * ny + y) * nx;
                const int jb = a.cstart[base + max(cx - g.fx, 0)], je = a.cstart[base + min(cx + g.fx, nx - 1) + 1];
                for (int t = jb; t < je; ++t) {
                    if (t == s) continue;
                    const int j = a.sidx[t];
                    const double4 q = pos[j];
                    const double dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
                    const double r2 = fma(dz, dz, fma(dy, dy, dx * dx));
                    if (!(r2 < rc2)) continue;
                    const double4 kj = a.dkmu[j];
                    const double A = a.pair_mix ? 0.5 * (ai + kj.y) : 1.0, B = a.pair_mix ? 0.5 * (bi + kj.z) : 0.0;
                    const double ga = fmax(1.0 - k2a * r2, 0.0);
                    const double tt = r2 * k2b, t2 = tt * tt;
                    const double gb = fmax(1.0 - t2 * t2, 0.0);
                    if (MODE == kModeEnergy) {
                        // each pair from both ends: half its energy here
                        ep += 0.5 * (A * P.pa_eps * ga * ga * ga + B * P.pb_eps * gb * gb * gb);
                    } else {
                        const double coef = A * 6.0 * P.pa_eps * k2a * ga * ga + B * 24.0 * P.pb_eps * k2b * gb * gb * t2 * tt;
                        fx = fma(coef, dx, fx);
                        fy = fma(coef, dy, fy);
                        fz = fma(coef, dz, fz);
                        nbr += 1.0;
                    }
                }
            }
    }
    double en[kEnergyKinds] = {0, 0, 0, 0, 0, 0, 0, 0};
    double rin[3] = {0, 0, 0}, rout[3] = {0, 0, 0};
    // every lane calls it (the droplet term is wave-cooperative); invalid lanes' results are dropped below
    local_terms<MODE, 1, double>(ctx, a, i, p.x, p.y, p.z, km, fx, fy, fz, en, rin, rout);
    double v[kEnergyKinds];
    if (MODE == kModeEnergy) {
        en[0] = ep;
        for (int k = 0; k < kEnergyKinds; ++k) v[k] = valid ? en[k] : 0.0;
    } else {
        if (valid) St<double>::force(a)[i] = make_double4(fx, fy, fz, 0.0);
        for (int k = 0; k < 3; ++k) {
            v[k] = valid ? rin[k] : 0.0;
            v[3 + k] = valid ? rout[k] : 0.0;
        }
        v[6] = valid ? km.x * sqrt(fx * fx + fy * fy + fz * fz) : 0.0;  // mu |F| (spacestep)
        v[7] = valid ? nbr : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kEnergyKinds; ++k) {
        const double w = (MODE != kModeEnergy && k == 6) ? wave_total_max_d(v[k]) : wave_total_sum_d(v[k]);
        if (lane == 0) s_red[k][wave] = w;
    }
    __syncthreads();
    if (threadIdx.x < kEnergyKinds) {
        const int k = threadIdx.x;
        double r = s_red[k][0];
        for (int w = 1; w < kEval64Block / 64; ++w) r = (MODE != kModeEnergy && k == 6) ? fmax(r, s_red[k][w]) : r + s_red[k][w];
        if (MODE == kModeEnergy)
            a.part_energy[blockIdx.x * kEnergyKinds + k] = r;
        else
            a.dpart[blockIdx.x * 8 + k] = r;
    }
}

// the fp64 evaluation's rows in a fixed order -> the context (reactions, max drift, neighbours), react_out[6] for
// the tail's ext_react, and (spacestep >= 0) the step's adapted timestep; oracle/gcs_oracle.c gcso_run's spacestep
__global__ __launch_bounds__(256) void k_red64(DevCtx* ctx, ForceArgs a, int rows, double spacestep, double timestep,
                                               double* react_out)
{
    __shared__ double s_red[8][4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = tid; b < rows; b += blockDim.x)
        for (int k = 0; k < 8; ++k) acc[k] = (k == 6) ? fmax(acc[k], a.dpart[b * 8 + k]) : acc[k] + a.dpart[b * 8 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const double w = (k == 6) ? wave_total_max_d(acc[k]) : wave_total_sum_d(acc[k]);
        if (lane == 0) s_red[k][wave] = w;
    }
    __syncthreads();
    if (tid != 0) return;
    double tot[8];
    for (int k = 0; k < 8; ++k) {
        tot[k] = s_red[k][0];
        for (int w = 1; w < (int)(blockDim.x / 64); ++w) tot[k] = (k == 6) ? fmax(tot[k], s_red[k][w]) : tot[k] + s_red[k][w];
    }
    for (int k = 0; k < 3; ++k) {
        ctx->react_in[k] = tot[k];
        ctx->react_out[k] = tot[3 + k];
    }
    if (react_out)
        for (int k = 0; k < 6; ++k) react_out[k] = tot[k];
    ctx->max_drift = tot[6];
    ctx->neighbors = tot[7] / (double)a.n;
    if (spacestep >= 0.0) {
        double dt = timestep;
        if (spacestep > 0.0 && tot[6] * dt > spacestep) dt = spacestep / tot[6];
        ctx->dt_used = dt;
    }
}

}  // namespace

// ----------------------------------------------------------------------------------------------------
// launch wrappers

void launch_prime(hipStream_t s, DevCtx* ctx, const ForceArgs& a, float rc_fixed, int ncell_max, const double* sched)
{
    if (a.prec == 64)
        hipLaunchKernelGGL(k_prime<double>, dim3(1), dim3(1024), 0, s, ctx, a, rc_fixed, ncell_max, sched);
    else
        hipLaunchKernelGGL(k_prime<float>, dim3(1), dim3(1024), 0, s, ctx, a, rc_fixed, ncell_max, sched);
}

void launch_cell_count(hipStream_t s, const DevCtx* ctx, const float4* pos0, const float4* pos1, int n, int* cell_of,
                       int* slot, int* count, const DomBox* reg, int* islot)
{
    const DomBox r = reg ? *reg : DomBox{};
    hipLaunchKernelGGL(k_cell_count<float4>, dim3((n + 255) / 256), dim3(256), 0, s, ctx, pos0, pos1, n, cell_of, slot,
                       count, reg ? 1 : 0, r, islot);
}

void launch_cell_count(hipStream_t s, const DevCtx* ctx, const double4* pos0, const double4* pos1, int n, int* cell_of,
                       int* slot, int* count, const DomBox* reg, int* islot)
{
    const DomBox r = reg ? *reg : DomBox{};
    hipLaunchKernelGGL(k_cell_count<double4>, dim3((n + 255) / 256), dim3(256), 0, s, ctx, pos0, pos1, n, cell_of, slot,
                       count, reg ? 1 : 0, r, islot);
}

void launch_tail_reduce(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int fblocks, double* out)
{
    hipLaunchKernelGGL(k_tail_reduce, dim3(1), dim3(256), 0, s, ctx, a, fblocks, out);
}

int rebuild_blocks(int ncell_max) { return 1 + ncell_max / (kRbCells / 2) + 2; }

int rebuild_sync_words(int ncell_max) { return 2 + 2 * (ncell_max / (kRbCells / 2) + 2); }

void launch_rebuild(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int* tmp, unsigned long long* scan_sync,
                    int fblocks, int apply_sched)
{
    // block 0: the tail; then enough rebuild blocks for any grid of <= ncell_max cells
    const int blocks = rebuild_blocks(a.ncell_max);
    hipLaunchKernelGGL(k_rebuild, dim3(blocks), dim3(kRbThreads), 0, s, ctx, a, tmp, scan_sync, fblocks,
                       apply_sched);
}

int scan_sync_words(int ncell_max) { return 2 + 2 * (ncell_max / (kMbCells / 2) + 2); }

void launch_cell_scan(hipStream_t s, DevCtx* ctx, int n, int* count, int* cstart, int* tile_start, int2* tile_range,
                      bool use_next, int4* units, int resident, unsigned long long* scan_sync, int ncell_max)
{
    if (scan_sync && !(units && resident > 0)) {
        // blocks for any grid of <= ncell_max cells: R*nx > kMbCells/2 cells per block (or one row of nx >= kMbCells)
        const int blocks = ncell_max / (kMbCells / 2) + 2;
        hipLaunchKernelGGL(k_cell_scan_mb, dim3(blocks), dim3(kMbThreads), 0, s, ctx, n, count, cstart, tile_start,
                           tile_range, use_next ? 1 : 0, scan_sync);
        return;
    }
    hipLaunchKernelGGL(k_cell_scan, dim3(1), dim3(1024), 0, s, ctx, n, count, cstart, tile_start, tile_range,
                       use_next ? 1 : 0, units, resident);
}

int force_step_resident(int waves)
{
    // workgroups of the fused step kernel resident at once on the whole device
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    hipError_t e = hipErrorInvalidValue;
    switch (waves) {
    case 1: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_force<kModeStep, 1, true, 1>, 64, 0); break;
    case 2: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_force<kModeStep, 2, true, 1>, 128, 0); break;
    case 8: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_force<kModeStep, 8, true, 1>, 512, 0); break;
    default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_force<kModeStep, 4, true, 4>, 256, 0); break;
    }
    return e == hipSuccess ? per * cus : 0;
}

void launch_cell_scatter(hipStream_t s, int n, const int* cell_of, const int* slot, const int* cstart, int* tmp,
                         int* count)
{
    hipLaunchKernelGGL(k_cell_scatter, dim3((n + 255) / 256), dim3(256), 0, s, n, cell_of, slot, cstart, tmp, count);
}

void launch_cell_sort(hipStream_t s, const DevCtx* ctx, const float4* pos0, const float4* pos1, const float4* kmu, int n,
                      const int* tmp, const int* cell_of, const int* cstart, int* sidx, int* scell, float4* spos,
                      float* sb, int pair_mix, const int* ptype, float4* psort0, float4* psort1, float4* skmu,
                      int2* sbrow, const int* boff, int* islot, const int* brev, int* bslot, const int* swt,
                      int* swslot)
{
    hipLaunchKernelGGL(k_cell_sort<float>, dim3((n + 255) / 256), dim3(256), 0, s, ctx, pos0, pos1, kmu, n, tmp,
                       cell_of, cstart, sidx, scell, spos, sb, pair_mix, ptype, psort0, psort1, skmu, sbrow, boff, islot,
                       (float4*)nullptr, (float4*)nullptr, brev, bslot, swt, swslot);
}

void launch_cell_sort(hipStream_t s, const DevCtx* ctx, const double4* pos0, const double4* pos1, const double4* kmu,
                      int n, const int* tmp, const int* cell_of, const int* cstart, int* sidx, int* scell, float4* spos,
                      float* sb, int pair_mix, const int* ptype, double4* psort0, double4* psort1, double4* skmu,
                      int2* sbrow, const int* boff, int* islot, float4* fsort0, float4* fsort1, const int* brev,
                      int* bslot, const int* swt, int* swslot)
{
    hipLaunchKernelGGL(k_cell_sort<double>, dim3((n + 255) / 256), dim3(256), 0, s, ctx, pos0, pos1, kmu, n, tmp,
                       cell_of, cstart, sidx, scell, spos, sb, pair_mix, ptype, psort0, psort1, skmu, sbrow, boff, islot,
                       fsort0, fsort1, brev, bslot, swt, swslot);
}

template <int MODE, bool FUSED>
static void launch_force_mode(hipStream_t s, int waves, DevCtx* ctx, const ForceArgs& a)
{
    const dim3 grid((MODE == kModeStep && a.split) ? force_grid_split(a.n) : force_grid(a.n));  // >= units
    switch (waves) {
    case 1: hipLaunchKernelGGL((k_force<MODE, 1, FUSED, 1>), grid, dim3(64), 0, s, ctx, a); break;
    case 2: hipLaunchKernelGGL((k_force<MODE, 2, FUSED, 1>), grid, dim3(128), 0, s, ctx, a); break;
    case 8: hipLaunchKernelGGL((k_force<MODE, 8, FUSED, 1>), grid, dim3(512), 0, s, ctx, a); break;
    default:
        if (a.subtiles == 4)
            hipLaunchKernelGGL((k_force<MODE, 4, FUSED, 4>), grid, dim3(256), 0, s, ctx, a);
        else if (a.subtiles == 2)
            hipLaunchKernelGGL((k_force<MODE, 4, FUSED, 2>), grid, dim3(256), 0, s, ctx, a);
        else
            hipLaunchKernelGGL((k_force<MODE, 4, FUSED, 1>), grid, dim3(256), 0, s, ctx, a);
        break;
    }
}

void launch_force(hipStream_t s, int mode, int waves, DevCtx* ctx, const ForceArgs& a, bool fused)
{
    if (mode == kModeStep) {
        if (fused)
            launch_force_mode<kModeStep, true>(s, waves, ctx, a);
        else
            launch_force_mode<kModeStep, false>(s, waves, ctx, a);
    } else if (mode == kModeForce) {
        launch_force_mode<kModeForce, false>(s, waves, ctx, a);
    } else {
        launch_force_mode<kModeEnergy, false>(s, waves, ctx, a);
    }
}

// the list step's launch: one workgroup per 64 consecutive slots
int list_step_grid(const ForceArgs& a) { return force_blocks(a.n); }

// the entry type of the launch's list format (ForceArgs::list_fmt), handed to fn as a value of that type
template <typename Fn>
static void with_list_entry(const ForceArgs& a, Fn&& fn)
{
    if (a.list_fmt == kListFmtAbs16)
        fn((unsigned short)0);
    else if (a.list_fmt == kListFmtRel16)
        fn(ListRel16{});
    else
        fn((int)0);
}

void launch_list_build(hipStream_t s, DevCtx* ctx, const ForceArgs& a)
{
    const dim3 g(force_grid(a.n));
    with_list_entry(a, [&](auto tag) {
        using LE = decltype(tag);
        if (a.list_waves == 2)
            hipLaunchKernelGGL((k_lbuild<LE, 2>), g, dim3(128), 0, s, ctx, a);
        else
            hipLaunchKernelGGL((k_lbuild<LE, 4>), g, dim3(256), 0, s, ctx, a);
    });
}

template <bool CT, typename R>
static void launch_list_step_ct(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int flags)
{
    const dim3 g(list_step_grid(a));
    with_list_entry(a, [&](auto tag) {
        using LE = decltype(tag);
        if (a.list_waves == 2)
            hipLaunchKernelGGL((k_lstep<LE, 2, CT, false, R>), g, dim3(128), 0, s, ctx, a, flags);
        else
            hipLaunchKernelGGL((k_lstep<LE, 4, CT, false, R>), g, dim3(256), 0, s, ctx, a, flags);
    });
}

__global__ void k_set_contact(DevCtx* ctx, float d2, double d2_64)
{
    ctx->contact_d2 = d2;
    ctx->contact_d2_64 = d2_64;
}
void launch_set_contact(hipStream_t s, DevCtx* ctx, float d2, double d2_64)
{
    hipLaunchKernelGGL(k_set_contact, dim3(1), dim3(1), 0, s, ctx, d2, d2_64);
}

template <typename R>
static void launch_list_relax_r(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int force_flags, int update_flags)
{
    const dim3 g(list_step_grid(a));
    with_list_entry(a, [&](auto tag) {
        using LE = decltype(tag);
        if (a.list_waves == 2)
            hipLaunchKernelGGL((k_lstep<LE, 2, false, false, R, true>), g, dim3(128), 0, s, ctx, a, force_flags);
        else
            hipLaunchKernelGGL((k_lstep<LE, 4, false, false, R, true>), g, dim3(256), 0, s, ctx, a, force_flags);
    });
    hipLaunchKernelGGL(k_lupdate<R>, dim3((a.n + kLUpdateBlock - 1) / kLUpdateBlock), dim3(kLUpdateBlock), 0, s, ctx, a,
                       update_flags);
}
void launch_dom_grid(hipStream_t s, DevCtx* ctx, const ForceArgs& a)
{
    hipLaunchKernelGGL(k_dom_grid, dim3(1), dim3(1), 0, s, ctx, a);
}

__global__ void k_poison(unsigned* p, size_t words)
{
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < words; k += (size_t)gridDim.x * blockDim.x)
        p[k] = (unsigned)((k + 1) * 2654435761ull) ^ 0x5bd1e995u;
}
void launch_poison(hipStream_t s, void* p, size_t bytes)
{
    const size_t words = bytes / sizeof(unsigned);
    hipLaunchKernelGGL(k_poison, dim3((unsigned)std::min<size_t>(1024, (words + 255) / 256 + 1)), dim3(256), 0, s,
                       (unsigned*)p, words);
}

void launch_pstep_guard(hipStream_t s, DevCtx* ctx, DevCtx* keep, const int* stall, int restore)
{
    hipLaunchKernelGGL(k_pstep_guard, dim3(1), dim3(64), 0, s, ctx, keep, stall, restore);
}

int launch_pstep(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int steps, int flags)
{
    const dim3 g((a.n + kPP - 1) / kPP), b(64 * kPWaves);
    ForceArgs args = a;
    void* kargs[] = {(void*)&ctx, (void*)&args, (void*)&steps, (void*)&flags};
    // cooperative: the runtime launches the grid only if every workgroup can be resident at once (the grid barrier)
    const void* fn = a.prec == 64 ? (const void*)k_pstep<double> : (const void*)k_pstep<float>;
    return hipLaunchCooperativeKernel(fn, g, b, kargs, 0, s) == hipSuccess ? 0 : -1;
}

void launch_list_relax(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int force_flags, int update_flags)
{
    if (a.prec == 64)
        launch_list_relax_r<double>(s, ctx, a, force_flags, update_flags);
    else
        launch_list_relax_r<float>(s, ctx, a, force_flags, update_flags);
}

template <typename R>
static void launch_list_step_dom(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int flags)
{
    const dim3 g(list_step_grid(a));
    with_list_entry(a, [&](auto tag) {
        using LE = decltype(tag);
        if (a.list_waves == 2)
            hipLaunchKernelGGL((k_lstep<LE, 2, false, true, R>), g, dim3(128), 0, s, ctx, a, flags);
        else
            hipLaunchKernelGGL((k_lstep<LE, 4, false, true, R>), g, dim3(256), 0, s, ctx, a, flags);
    });
}

void launch_list_step(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int flags)
{
    if (flags & kLFlagDomain) {  // decomposed (no fused contacts: the engine flushes them before a decomposed step)
        if (a.prec == 64)
            launch_list_step_dom<double>(s, ctx, a, flags);
        else
            launch_list_step_dom<float>(s, ctx, a, flags);
        return;
    }
    if (a.prec == 64) {
        if (a.contact_on)
            launch_list_step_ct<true, double>(s, ctx, a, flags);
        else
            launch_list_step_ct<false, double>(s, ctx, a, flags);
    } else {
        if (a.contact_on)
            launch_list_step_ct<true, float>(s, ctx, a, flags);
        else
            launch_list_step_ct<false, float>(s, ctx, a, flags);
    }
}

void launch_list_domain_tail(hipStream_t s, DevCtx* ctx, const ForceArgs& a, const double* glob, int flags,
                             const int* shared, int nshared, void* bands, int npeer, int band_stride)
{
    if (a.prec == 64)
        hipLaunchKernelGGL(k_ldom_tail<double>, dim3(1), dim3(64), 0, s, ctx, a, glob, flags, shared, nshared,
                           (double4*)bands, npeer, band_stride);
    else
        hipLaunchKernelGGL(k_ldom_tail<float>, dim3(1), dim3(64), 0, s, ctx, a, glob, flags, shared, nshared,
                           (float4*)bands, npeer, band_stride);
}

void launch_list_domain_finish(hipStream_t s, DevCtx* ctx, const ForceArgs& a, const double* glob, int flags,
                               const int* shared, int nshared, const void* in, const int* counts, int nbuf, int cap,
                               int istride, int cstride, void* send, int nsend, int sstride)
{
    const int blocks = nbuf > 0 ? std::max(1, std::min(1024, (cap + 255) / 256)) : 1;
    if (a.prec == 64)
        hipLaunchKernelGGL(k_ldom_finish<double>, dim3(blocks), dim3(256), 0, s, ctx, a, glob, flags, shared, nshared,
                           (const double4*)in, counts, nbuf, cap, istride, cstride, (double4*)send, nsend, sstride);
    else
        hipLaunchKernelGGL(k_ldom_finish<float>, dim3(blocks), dim3(256), 0, s, ctx, a, glob, flags, shared, nshared,
                           (const float4*)in, counts, nbuf, cap, istride, cstride, (float4*)send, nsend, sstride);
}

void launch_update(hipStream_t s, const DevCtx* ctx, const ForceArgs& a)
{
    if (a.prec == 64)
        hipLaunchKernelGGL(k_update<double>, dim3(update_blocks(a.n)), dim3(kUpdateBlock), 0, s, ctx, a);
    else
        hipLaunchKernelGGL(k_update<float>, dim3(update_blocks(a.n)), dim3(kUpdateBlock), 0, s, ctx, a);
}

int eval64_blocks(int n) { return (n + kEval64Block - 1) / kEval64Block; }

void launch_eval64(hipStream_t s, int mode, const DevCtx* ctx, const ForceArgs& a)
{
    const dim3 g(eval64_blocks(a.n));
    if (mode == kModeEnergy)
        hipLaunchKernelGGL(k_eval64<kModeEnergy>, g, dim3(kEval64Block), 0, s, ctx, a);
    else
        hipLaunchKernelGGL(k_eval64<kModeForce>, g, dim3(kEval64Block), 0, s, ctx, a);
}

void launch_red64(hipStream_t s, DevCtx* ctx, const ForceArgs& a, double spacestep, double timestep, double* react_out)
{
    hipLaunchKernelGGL(k_red64, dim3(1), dim3(256), 0, s, ctx, a, eval64_blocks(a.n), spacestep, timestep, react_out);
}

void launch_adapt(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int fblocks, float spacestep, float timestep)
{
    hipLaunchKernelGGL(k_adapt, dim3(1), dim3(256), 0, s, ctx, a, fblocks, spacestep, timestep);
}

void launch_tail(hipStream_t s, DevCtx* ctx, const ForceArgs& a, int fblocks, int bblocks, int advance, int apply_sched,
                 int ncell_max, const double* sched)
{
    hipLaunchKernelGGL(k_tail, dim3(1), dim3(256), 0, s, ctx, a, fblocks, bblocks, advance, apply_sched, ncell_max,
                       sched);
}

void launch_search_count(hipStream_t s, const DevCtx* ctx, int n, const float4* spos, const int* sidx, const int* scell,
                         const int* cstart, int* counts, const double4* pos64, double d64)
{
    if (pos64)
        hipLaunchKernelGGL((k_search<false, true>), dim3((n + 255) / 256), dim3(256), 0, s, ctx, n, spos, sidx, scell,
                           cstart, counts, (const int*)nullptr, (unsigned long long*)nullptr, pos64, d64);
    else
        hipLaunchKernelGGL((k_search<false, false>), dim3((n + 255) / 256), dim3(256), 0, s, ctx, n, spos, sidx, scell,
                           cstart, counts, (const int*)nullptr, (unsigned long long*)nullptr, pos64, d64);
}

void launch_search_emit(hipStream_t s, const DevCtx* ctx, int n, const float4* spos, const int* sidx, const int* scell,
                        const int* cstart, const int* offsets, unsigned long long* keys, const double4* pos64,
                        double d64)
{
    if (pos64)
        hipLaunchKernelGGL((k_search<true, true>), dim3((n + 255) / 256), dim3(256), 0, s, ctx, n, spos, sidx, scell,
                           cstart, (int*)nullptr, offsets, keys, pos64, d64);
    else
        hipLaunchKernelGGL((k_search<true, false>), dim3((n + 255) / 256), dim3(256), 0, s, ctx, n, spos, sidx, scell,
                           cstart, (int*)nullptr, offsets, keys, pos64, d64);
}

void launch_exclusive_scan_small(hipStream_t s, const int* in, int* out, int n, int* total)
{
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, s, in, out, n, total);
}

size_t sort_u64_temp_bytes(int n)
{
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr, n);
    return bytes;
}

void sort_u64_keys(hipStream_t s, unsigned long long* keys, unsigned long long* tmp, int n, void* temp, size_t temp_bytes)
{
    (void)hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, keys, tmp, n, 0, 64, s);
}

}  // namespace gcs
