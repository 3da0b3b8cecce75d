// contacts.hip -- off-step-loop device work of the interphase driver surface (gfx950):
//   * the contact map (stage_interphase/contact_map.cpp:33-85): every contactmap_update_interval steps every pair
//     i < j closer than the contact distance is counted into an open-addressing hash table in HBM (64-bit key
//     i << 32 | j, 32-bit count); at the output window the occupied slots are compacted and radix-sorted by (i, j)
//     on the device (contact_map.cpp:66-85 sorts the same keys on the host)
//   * the sampled-position quantisation of simulation_store.cpp:22-33 / 192-216 (16 fraction bits, stored as f32)
// The pair predicate is the strict one of the neighbour search (kernels.hip k_search), fp32 or (the fp64 engine)
// fp64: bit-exact against the oracle's gcso_search_neighbors / gcso_search_neighbors64.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "engine_internal.hpp"

namespace gcs {
namespace {

__device__ __forceinline__ bool contact_pair(float4 p, float4 q, float d2)
{
    const float dx = __fsub_rn(p.x, q.x), dy = __fsub_rn(p.y, q.y), dz = __fsub_rn(p.z, q.z);
    const float r2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
    return r2 < d2;
}
// the fp64 engine's predicate (the same strict form in fp64, kernels.hip strict_lt)
__device__ __forceinline__ bool contact_pair(double4 p, double4 q, double d2)
{
    const double dx = __dsub_rn(p.x, q.x), dy = __dsub_rn(p.y, q.y), dz = __dsub_rn(p.z, q.z);
    const double r2 = __dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz));
    return r2 < d2;
}


// One thread per cell-sorted particle of any cell list (the engine's own, or a search list built for the
// distance): the stencil reach per axis is ceil(distance / cell edge) cells (for the engine's list, whose cells
// are >= the force cutoff >= the contact distance, that is the usual 3 x 3 rows x 5 x-cells; clamped outliers
// only get closer in cell units).  Every pair i < j inside the distance is counted into the table.  A failed insert (probe sequence
// exhausted: table too full) raises overflow; counts stay exact for the inserted keys.
// F64: the pair test in fp64 on pos64[particle] (the fp64 engine's positions) with d2 = dist64 * dist64
template <bool F64>
__global__ __launch_bounds__(256) void k_contact_insert(const DevCtx* __restrict__ ctx, int n, float dist,
                                                        const float4* __restrict__ spos, const int* __restrict__ sidx,
                                                        const int* __restrict__ scell, const int* __restrict__ cstart,
                                                        unsigned long long* __restrict__ keys,
                                                        unsigned* __restrict__ counts, int bits,
                                                        int* __restrict__ overflow, const double4* __restrict__ pos64,
                                                        double dist64)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const Grid g = ctx->grid;
    if (s >= n || s >= cstart[g.ncell]) return;
    const float d2 = __fmul_rn(dist, dist);
    const double d2_64 = __dmul_rn(dist64, dist64);
    const float widen = 1.0f + 1.0e-6f;  // never round a reach down
    const int rx = (int)ceilf(dist * g.inv[0] * widen), ry = (int)ceilf(dist * g.inv[1] * widen),
              rz = (int)ceilf(dist * g.inv[2] * widen);
    const int i = sidx[s];
    const float4 p = spos[s];
    double4 p64 = make_double4(0.0, 0.0, 0.0, 0.0);
    if constexpr (F64) p64 = pos64[i];
    const int c = scell[s];
    const int nx = g.n[0], ny = g.n[1], nz = g.n[2];
    const int cx = c % nx, cy = (c / nx) % ny, cz = c / (nx * ny);
    for (int z = max(cz - rz, 0); z <= min(cz + rz, nz - 1); ++z)
        for (int y = max(cy - ry, 0); y <= min(cy + ry, ny - 1); ++y) {
            const int base = (z * ny + y) * nx;
            const int jb = cstart[base + max(cx - rx, 0)], je = cstart[base + min(cx + rx, nx - 1) + 1];
            for (int t = jb; t < je; ++t) {
                const int j = sidx[t];
                if (j <= i) continue;
                if constexpr (F64) {
                    if (!contact_pair(p64, pos64[j], d2_64)) continue;
                } else {
                    if (!contact_pair(p, spos[t], d2)) continue;
                }
                const unsigned long long key = ((unsigned long long)(unsigned)i << 32) | (unsigned)j;
                if (!contact_count(keys, counts, bits, key)) atomicOr(overflow, 1);
            }
        }
}

// Both table scans below add to ONE global counter, so they aggregate per workgroup: one atomic per 4,096 slots.
// (Per-wave atomics -- 2^24 / 64 = 262k adds to one address at C2's table -- serialised in L2 and took 5.8 ms per
// output window at C2, 46 ms at C5; profiles/r04s_c5_kernel_stats.csv, profiles/r06_contact_bits.txt.)
constexpr int kCompactPer = 16;                          // slots per thread per chunk
constexpr long long kCompactChunk = 256LL * kCompactPer;  // slots per workgroup per chunk

// block-wide sum of v (256 threads), valid in thread 0
__device__ __forceinline__ int block_sum_256(int v, int* s_wave)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = v;
    __syncthreads();
    const int t = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    __syncthreads();
    return t;
}

// occupied slots of the table: sizes the compaction's scratch before the compaction
__global__ __launch_bounds__(256) void k_contact_occupied(const unsigned long long* __restrict__ keys, long long slots,
                                                          int* __restrict__ total)
{
    __shared__ int s_wave[4];
    int c = 0;
    for (long long h = (long long)blockIdx.x * blockDim.x + threadIdx.x; h < slots;
         h += (long long)gridDim.x * blockDim.x)
        c += keys[h] != kContactEmpty ? 1 : 0;
    const int t = block_sum_256(c, s_wave);
    if (threadIdx.x == 0 && t) atomicAdd(total, t);
}

// occupied slots -> (key, count) lists; output order is arbitrary (the sort that follows fixes it).  A workgroup
// takes 4,096 consecutive slots (16 per thread, coalesced loads kept in registers), scans the per-thread occupancy
// across the workgroup, reserves its run of the output with one atomic and writes each thread's keys in its run.
__global__ __launch_bounds__(256) void k_contact_compact(const unsigned long long* __restrict__ keys,
                                                         const unsigned* __restrict__ counts, long long slots,
                                                         unsigned long long* __restrict__ out_k,
                                                         unsigned* __restrict__ out_c, int* __restrict__ total)
{
    __shared__ int s_wave[4];
    __shared__ int s_base;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (long long c0 = (long long)blockIdx.x * kCompactChunk; c0 < slots;
         c0 += (long long)gridDim.x * kCompactChunk) {
        unsigned long long k[kCompactPer];
        int m = 0;
#pragma unroll
        for (int u = 0; u < kCompactPer; ++u) {
            const long long h = c0 + (long long)u * 256 + t;
            k[u] = h < slots ? keys[h] : kContactEmpty;
            m += k[u] != kContactEmpty ? 1 : 0;
        }
        int x = m;  // inclusive scan over the wave
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wave[w] = x;
        __syncthreads();
        if (t == 0) {
            const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
            s_base = tot ? atomicAdd(total, tot) : 0;
        }
        __syncthreads();
        int o = s_base + x - m;
        for (int v = 0; v < w; ++v) o += s_wave[v];
#pragma unroll
        for (int u = 0; u < kCompactPer; ++u)
            if (k[u] != kContactEmpty) {
                out_k[o] = k[u];
                out_c[o] = counts[c0 + (long long)u * 256 + t];
                ++o;
            }
        __syncthreads();  // s_wave / s_base are rewritten by the next chunk
    }
}

// simulation_store.cpp:22-33: frexp, round the mantissa to `bits` fraction bits (nearbyint, round-half-even), ldexp
// back.  On an fp32 value every step is exact in fp32, so the result equals the fp64 reference applied to the same
// (fp32) coordinate; on an fp64 value it is the reference's arithmetic itself, and the result (<= 24 significant
// bits for bits <= 23) converts to the stored f32 exactly.
__device__ __forceinline__ float quantize_v(float v, int bits)
{
    int ex = 0;
    const float m = frexpf(v, &ex);
    const float sm = rintf(ldexpf(m, bits));
    return ldexpf(sm, ex - bits);
}
__device__ __forceinline__ float quantize_v(double v, int bits)
{
    int ex = 0;
    const double m = frexp(v, &ex);
    const double sm = rint(ldexp(m, bits));
    return (float)ldexp(sm, ex - bits);
}

template <typename P>
__global__ __launch_bounds__(256) void k_quantize(const P* __restrict__ pos, float* __restrict__ out, int n, int bits)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const P p = pos[i];
    out[3 * i] = quantize_v(p.x, bits);
    out[3 * i + 1] = quantize_v(p.y, bits);
    out[3 * i + 2] = quantize_v(p.z, bits);
}

}  // namespace

void launch_contact_insert(hipStream_t s, const DevCtx* ctx, int n, double dist, const float4* spos, const int* sidx,
                           const int* scell, const int* cstart, unsigned long long* keys, unsigned* counts, int bits,
                           int* overflow, const double4* pos64)
{
    if (pos64)
        hipLaunchKernelGGL(k_contact_insert<true>, dim3((n + 255) / 256), dim3(256), 0, s, ctx, n, (float)dist, spos,
                           sidx, scell, cstart, keys, counts, bits, overflow, pos64, dist);
    else
        hipLaunchKernelGGL(k_contact_insert<false>, dim3((n + 255) / 256), dim3(256), 0, s, ctx, n, (float)dist, spos,
                           sidx, scell, cstart, keys, counts, bits, overflow, pos64, dist);
}

void launch_contact_occupied(hipStream_t s, const unsigned long long* keys, long long slots, int* total)
{
    const long long blocks = std::min<long long>((slots + 255) / 256, 4096);
    hipLaunchKernelGGL(k_contact_occupied, dim3((unsigned)blocks), dim3(256), 0, s, keys, slots, total);
}

void launch_contact_compact(hipStream_t s, const unsigned long long* keys, const unsigned* counts, long long slots,
                            unsigned long long* out_k, unsigned* out_c, int* total)
{
    const long long chunks = (slots + kCompactChunk - 1) / kCompactChunk;
    const long long blocks = std::max<long long>(1, std::min<long long>(chunks, 8192));
    hipLaunchKernelGGL(k_contact_compact, dim3((unsigned)blocks), dim3(256), 0, s, keys, counts, slots, out_k, out_c,
                       total);
}

// sorted (key, count) -> the (i, j, count) rows the caller reads (one copy to the host, no host-side reformatting)
__global__ __launch_bounds__(256) void k_contact_emit(const unsigned long long* __restrict__ k,
                                                      const unsigned* __restrict__ c, int n, unsigned* __restrict__ out)
{
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const unsigned long long key = k[t];
        out[3 * (size_t)t] = (unsigned)(key >> 32);
        out[3 * (size_t)t + 1] = (unsigned)key;
        out[3 * (size_t)t + 2] = c[t];
    }
}

void launch_contact_emit(hipStream_t s, const unsigned long long* k, const unsigned* c, int n, unsigned* out)
{
    const int blocks = std::max(1, std::min((n + 255) / 256, 4096));
    hipLaunchKernelGGL(k_contact_emit, dim3(blocks), dim3(256), 0, s, k, c, n, out);
}

size_t sort_pairs_u64_u32_temp_bytes(int n)
{
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (unsigned long long*)nullptr,
                                             (unsigned long long*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr, n);
    return bytes;
}

void sort_pairs_u64_u32(hipStream_t s, const unsigned long long* k_in, unsigned long long* k_out, const unsigned* v_in,
                        unsigned* v_out, int n, void* temp, size_t temp_bytes, int end_bit)
{
    (void)hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k_in, k_out, v_in, v_out, n, 0, end_bit, s);
}

void launch_quantize(hipStream_t s, const float4* pos, float* out, int n, int bits)
{
    hipLaunchKernelGGL(k_quantize<float4>, dim3((n + 255) / 256), dim3(256), 0, s, pos, out, n, bits);
}

void launch_quantize(hipStream_t s, const double4* pos, float* out, int n, int bits)
{
    hipLaunchKernelGGL(k_quantize<double4>, dim3((n + 255) / 256), dim3(256), 0, s, pos, out, n, bits);
}

}  // namespace gcs
