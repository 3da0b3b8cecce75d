// domain.hip -- the band exchange of the spatial domain decomposition (C5; DESIGN.md "Multi-GPU").
//
// Every engine of a decomposed run holds all N particles by global index.  Domain d OWNS the particles that lie in
// its box [lo_d, hi_d) (per axis; the boxes tile space) at the start of a step and integrates only those; its
// pair/bond terms read the particles within `halo` of the box (its region E_d = [lo_d - halo, hi_d + halo)), which
// must therefore be fresh.  After every step each domain sends to every peer p the (index, new position) of each particle it owned
// whose old OR new position lies in E_p; the receiver writes both position buffers.  So every copy inside E_p is
// refreshed each step, and a copy that goes stale was last sent from outside E_p (the "old or new" rule sends the
// exit position), i.e. it is never mistaken for a particle within the cutoff of p's slab.  Bonded partners need
// the same guarantee: every bond of an owned particle must be shorter than `halo` (checked here each step,
// flags[0]; LAMMPS's "bond atom missing" condition).  Ownership hand-over needs no message: a particle that
// crosses from box d to box p lands in E_p, is sent, and both sides then compute the same owner from the same
// bits.  The decomposed list step packs from its list slots (every owned particle has one: kDomFlagLost otherwise)
// and the receiver refreshes the records' slots too (islot), so the pair gathers by slot see fresh ghosts.
#include <hip/hip_runtime.h>

#include "engine_internal.hpp"

namespace gcs {
namespace {

// Records are real4<R> {x, y, z, index bits} (16 B at fp32, 32 B at fp64; the engine's precision), appended per peer
// with one atomic per wave (order is irrelevant: the unpack is a scatter by index).  flags[0] |= 1: a bond (not the
// cut-off softwell) of an owned particle reaches beyond the halo; flags[0] |= 2: a peer's band exceeded `cap`.
// Band b's records are out[b * ostride + k], its count counts[b * cstride] (the engine-owned bands keep the count in
// the band's header row: one message per peer carries both).
// One lane per particle (slots == 0: every particle by index) or per list slot (slots != 0: the ctx->lnslots slots
// of the decomposed list step's lists, the particle index in the record's .w), grid-stride with wave-uniform trips.
template <typename R>
__global__ __launch_bounds__(256) void k_domain_pack(const DevCtx* __restrict__ ctx, ForceArgs a,
                                                     const DomBox* __restrict__ regions, int npeer,
                                                     real4<R>* __restrict__ out, int* __restrict__ counts, int cap,
                                                     int* __restrict__ flags, const int* __restrict__ shared,
                                                     int ostride, int cstride, int slots)
{
    using R4 = real4<R>;
    const int lane = threadIdx.x & 63;
    // after the step's tail: pos[parity] holds the new positions, pos[parity ^ 1] the step's start
    const R4* pnew = St<R>::pos(a, ctx->parity);
    const R4* pold = St<R>::pos(a, ctx->parity ^ 1);
    const R4* qnew = St<R>::psort(a, ctx->parity);
    const R4* qold = St<R>::psort(a, ctx->parity ^ 1);
    const int total = slots ? ctx->lnslots : a.n;
    const int stride = gridDim.x * blockDim.x;
    for (int base = blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < total; base += stride) {
        const int k = base + lane;
        const bool in = k < total;
        R4 po = mk4<R>(R(0), R(0), R(0), R(0));
        int i = 0;
        if (in) {
            po = slots ? qold[k] : pold[k];
            i = slots ? (wbits(po.w) & ((1 << kListIndexBits) - 1)) : k;
        }
        const float ox = (float)po.x, oy = (float)po.y, oz = (float)po.z;
        const bool own = in && box_has(a.dom, ox, oy, oz);
        const R4 pn = own ? (slots ? qnew[k] : pnew[k]) : po;
        const float nx = (float)pn.x, ny = (float)pn.y, nz = (float)pn.z;
        if (own && a.has_bonds && !(shared && shared[i])) {
            const float h2 = a.dom_halo * a.dom_halo;
            bool far = false;
            for (int q = a.boff[i]; q < a.boff[i + 1]; ++q) {
                const int2 en = a.bent[q];
                if ((en.y & 15) == kSoftwell) continue;  // cut off below the halo (droplet): a pair term
                if (shared && shared[en.x]) continue;    // shared particles are fresh everywhere
                const R4 pj = pold[en.x];
                const float dx = ox - (float)pj.x, dy = oy - (float)pj.y, dz = oz - (float)pj.z;
                far |= dx * dx + dy * dy + dz * dz >= h2;
            }
            if (far) atomicOr(&flags[0], 1);
        }
        for (int p = 0; p < npeer; ++p) {
            const DomBox r = regions[p];
            const bool send = own && (box_has(r, ox, oy, oz) || box_has(r, nx, ny, nz));
            const unsigned long long m = __ballot(send);
            if (m == 0ull) continue;
            int at = 0;
            if (lane == 0) at = atomicAdd(&counts[(size_t)p * cstride], __popcll(m));
            at = __shfl(at, 0);
            if (send) {
                const int o = at + __popcll(m & ((1ull << lane) - 1ull));
                if (o < cap)
                    out[(size_t)p * ostride + o] = mk4<R>(pn.x, pn.y, pn.z, wpack<R>(i));
                else
                    atomicOr(&flags[0], 2);
            }
        }
    }
}

// received bands: nbuf buffers of `cap` records, counts[b] valid in buffer b; both position buffers are written
// (slots != 0: also the record's list slot in both slot-order buffers, when the current lists have one)
template <typename R>
__global__ __launch_bounds__(256) void k_domain_unpack(ForceArgs a, const real4<R>* __restrict__ in,
                                                       const int* __restrict__ counts, int nbuf, int cap, int istride,
                                                       int cstride, int slots, real4<R>* __restrict__ send, int nsend,
                                                       int sstride)
{
    using R4 = real4<R>;
    // the send bands' header rows for the next step's fused pack (this step's sends are done: stream order)
    if (blockIdx.x == 0)
        for (int p = threadIdx.x; p < nsend; p += blockDim.x) send[(size_t)p * sstride] = mk4<R>(R(0), R(0), R(0), R(0));
    dom_unpack_records<R>(a, in, counts, nbuf, cap, istride, cstride, slots, blockIdx.x * blockDim.x + threadIdx.x,
                          gridDim.x * blockDim.x);
}

// Shared particles (the nucleolar beads and their NOR beads: their bonds are far softer than the chain's, so no
// practical halo covers them): every domain holds them fresh each step.  Before the step's tail the owner writes
// its shared particles' new positions into the allreduce buffer (the others write 0; one owner per particle, so
// the sum is exact), after it every domain copies the sums into both position buffers.
template <typename R>
__global__ __launch_bounds__(64) void k_domain_shared_out(const DevCtx* __restrict__ ctx, ForceArgs a,
                                                          const int* __restrict__ idx, int nshared,
                                                          double* __restrict__ buf)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nshared) return;
    const real4<R>* cur = St<R>::pos(a, ctx->parity);      // before the tail: the step's start
    const real4<R>* nxt = St<R>::pos(a, ctx->parity ^ 1);  // the owners' new positions
    const int i = idx[k];
    const real4<R> c = cur[i];
    const bool own = box_has(a.dom, (float)c.x, (float)c.y, (float)c.z);
    const real4<R> p = nxt[i];
    buf[kDomainRed + 3 * k] = own ? (double)p.x : 0.0;
    buf[kDomainRed + 3 * k + 1] = own ? (double)p.y : 0.0;
    buf[kDomainRed + 3 * k + 2] = own ? (double)p.z : 0.0;
}

template <typename R>
__global__ __launch_bounds__(64) void k_domain_shared_in(ForceArgs a, const int* __restrict__ idx, int nshared,
                                                         const double* __restrict__ buf)
{
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nshared) return;
    const int i = idx[k];
    const real4<R> p = mk4<R>((R)buf[kDomainRed + 3 * k], (R)buf[kDomainRed + 3 * k + 1], (R)buf[kDomainRed + 3 * k + 2],
                              R(0));
    St<R>::pos(a, 0)[i] = p;
    St<R>::pos(a, 1)[i] = p;
}

// zero the header rows (counts) of npeer bands of `stride` records
template <typename R>
__global__ void k_band_headers_zero(real4<R>* bands, int npeer, int stride)
{
    const int p = threadIdx.x;
    if (p < npeer) bands[(size_t)p * stride] = mk4<R>(R(0), R(0), R(0), R(0));
}

}  // namespace

// band buffers are untyped at these entry points: records of the engine's precision (band_record_bytes)
void launch_domain_pack(hipStream_t s, const DevCtx* ctx, const ForceArgs& a, const DomBox* regions, int npeer,
                        void* out, int* counts, int cap, int* flags, const int* shared, int ostride, int cstride,
                        int slots)
{
    const int blocks = std::max(1, std::min(2048, (a.n + 255) / 256));
    if (a.prec == 64)
        hipLaunchKernelGGL(k_domain_pack<double>, dim3(blocks), dim3(256), 0, s, ctx, a, regions, npeer,
                           (double4*)out, counts, cap, flags, shared, ostride > 0 ? ostride : cap, cstride, slots);
    else
        hipLaunchKernelGGL(k_domain_pack<float>, dim3(blocks), dim3(256), 0, s, ctx, a, regions, npeer, (float4*)out,
                           counts, cap, flags, shared, ostride > 0 ? ostride : cap, cstride, slots);
}

void launch_domain_shared_out(hipStream_t s, const DevCtx* ctx, const ForceArgs& a, const int* idx, int nshared,
                              double* buf)
{
    if (nshared <= 0) return;
    if (a.prec == 64)
        hipLaunchKernelGGL(k_domain_shared_out<double>, dim3((nshared + 63) / 64), dim3(64), 0, s, ctx, a, idx, nshared, buf);
    else
        hipLaunchKernelGGL(k_domain_shared_out<float>, dim3((nshared + 63) / 64), dim3(64), 0, s, ctx, a, idx, nshared, buf);
}

void launch_domain_shared_in(hipStream_t s, const ForceArgs& a, const int* idx, int nshared, const double* buf)
{
    if (nshared <= 0) return;
    if (a.prec == 64)
        hipLaunchKernelGGL(k_domain_shared_in<double>, dim3((nshared + 63) / 64), dim3(64), 0, s, a, idx, nshared, buf);
    else
        hipLaunchKernelGGL(k_domain_shared_in<float>, dim3((nshared + 63) / 64), dim3(64), 0, s, a, idx, nshared, buf);
}

void launch_domain_unpack(hipStream_t s, const ForceArgs& a, const void* in, const int* counts, int nbuf, int cap,
                          int istride, int cstride, int slots, void* send, int nsend, int sstride)
{
    const int blocks = std::max(1, std::min(1024, (cap + 255) / 256));
    if (a.prec == 64)
        hipLaunchKernelGGL(k_domain_unpack<double>, dim3(blocks), dim3(256), 0, s, a, (const double4*)in, counts, nbuf,
                           cap, istride > 0 ? istride : cap, cstride, slots, (double4*)send, send ? nsend : 0, sstride);
    else
        hipLaunchKernelGGL(k_domain_unpack<float>, dim3(blocks), dim3(256), 0, s, a, (const float4*)in, counts, nbuf,
                           cap, istride > 0 ? istride : cap, cstride, slots, (float4*)send, send ? nsend : 0, sstride);
}

void launch_band_headers_zero(hipStream_t s, void* bands, int npeer, int stride, int prec)
{
    if (npeer <= 0) return;
    if (prec == 64)
        hipLaunchKernelGGL(k_band_headers_zero<double>, dim3(1), dim3(64), 0, s, (double4*)bands, npeer, stride);
    else
        hipLaunchKernelGGL(k_band_headers_zero<float>, dim3(1), dim3(64), 0, s, (float4*)bands, npeer, stride);
}

}  // namespace gcs
