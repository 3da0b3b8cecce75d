// FETCH_SIZE / WRITE_SIZE calibration: kernels with known request bytes, run one after another;
// tools/calib/run.sh collects the counters in separate rocprofv3 passes and tools/calib/summarize.py divides.
//   stream16 / stream8 / stream2: every byte of a 1 GiB buffer read once, 16 / 8 / 2 B per lane, coalesced
//   gather32 / gather16 / gather2: 32 Mi random records of 32 / 16 / 2 B from a 2 GiB buffer (far beyond the L2 and the
//   256 MB Infinity Cache: every record is its own line), the indices from a hash (no index traffic)
//   write16: 1 GiB written, 16 B per lane
// Every kernel folds what it reads into a value stored only when it equals a constant the data never produces (but
// the compiler cannot rule out: a 16-bit pattern, since 2-B reads fold to 16 bits), so no load is dropped.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

template <typename T>
__global__ __launch_bounds__(256) void k_stream(const T* __restrict__ p, size_t n, unsigned* __restrict__ out)
{
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = p[i];
        const unsigned* w = reinterpret_cast<const unsigned*>(&v);
        if constexpr (sizeof(T) >= 4) {
            for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc ^= w[k];
        } else {
            acc ^= (unsigned)v;
        }
    }
    if (acc == 0x1234u) out[threadIdx.x] = acc;  // (a value XOR-folded 16-bit reads can reach: the loads stay)
}

template <typename T>
__global__ __launch_bounds__(256) void k_gather(const T* __restrict__ p, size_t nrec, size_t count, unsigned* __restrict__ out)
{
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        const T v = p[mix(i) % nrec];
        const unsigned* w = reinterpret_cast<const unsigned*>(&v);
        if constexpr (sizeof(T) >= 4) {
            for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc ^= w[k];
        } else {
            acc ^= (unsigned)v;
        }
    }
    if (acc == 0x1234u) out[threadIdx.x] = acc;  // (a value XOR-folded 16-bit reads can reach: the loads stay)
}

__global__ __launch_bounds__(256) void k_write16(uint4* __restrict__ p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

struct Rec32 {
    uint4 a, b;
};

int main()
{
    const size_t stream_bytes = 1ull << 30, gather_bytes = 2ull << 30, count = 32ull << 20;
    void *s = nullptr, *g = nullptr;
    unsigned* out = nullptr;
    CK(hipMalloc(&s, stream_bytes));
    CK(hipMalloc(&g, gather_bytes));
    CK(hipMalloc(&out, 4096));
    CK(hipMemset(s, 1, stream_bytes));
    CK(hipMemset(g, 2, gather_bytes));
    CK(hipDeviceSynchronize());
    const dim3 grid(8192), block(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_stream<uint4>, grid, block, 0, 0, (const uint4*)s, stream_bytes / 16, out);
        hipLaunchKernelGGL(k_stream<uint2>, grid, block, 0, 0, (const uint2*)s, stream_bytes / 8, out);
        hipLaunchKernelGGL(k_stream<unsigned short>, grid, block, 0, 0, (const unsigned short*)s, stream_bytes / 2, out);
        hipLaunchKernelGGL(k_gather<Rec32>, grid, block, 0, 0, (const Rec32*)g, gather_bytes / 32, count, out);
        hipLaunchKernelGGL(k_gather<uint4>, grid, block, 0, 0, (const uint4*)g, gather_bytes / 16, count, out);
        hipLaunchKernelGGL(k_gather<unsigned short>, grid, block, 0, 0, (const unsigned short*)g, gather_bytes / 2, count, out);
        hipLaunchKernelGGL(k_write16, grid, block, 0, 0, (uint4*)s, stream_bytes / 16);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::printf("fetch_calib: stream %zu B, gathers %zu records from %zu B, write %zu B\n", stream_bytes, count,
                gather_bytes, stream_bytes);
    CK(hipFree(s));
    CK(hipFree(g));
    CK(hipFree(out));
    return 0;
}
