// LDS-DMA lane layout probe: where does global_load_lds of width 4 / 12 / 16 put lane l's bytes in LDS?
// usage: hipcc --offload-arch=gfx950 -O2 glds_width.hip -o glds_width && ./glds_width
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void* lds_t;
template <int WIDTH>
__global__ void k(const unsigned* src, unsigned* out)
{
    __shared__ unsigned s[64 * 4 + 64];
    for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) s[i] = 0xdeadbeefu;
    __syncthreads();
    // lane l reads WIDTH bytes starting at dword 100 * l of src (dwords 100 l, 100 l + 1, ...)
    const void* g = (const void*)(src + 100 * threadIdx.x);
    if constexpr (WIDTH == 4) __builtin_amdgcn_global_load_lds(g, (lds_t)s, 4, 0, 0);
    if constexpr (WIDTH == 12) __builtin_amdgcn_global_load_lds(g, (lds_t)s, 12, 0, 0);
    if constexpr (WIDTH == 16) __builtin_amdgcn_global_load_lds(g, (lds_t)s, 16, 0, 0);
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) out[i] = s[i];
}
int main()
{
    unsigned h[6400], *d, *o, r[320];
    for (int i = 0; i < 6400; ++i) h[i] = i;
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, sizeof(r));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    auto run = [&](auto kern, int w) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, d, o);
        hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
        printf("width %2d: dwords 0..11 =", w);
        for (int i = 0; i < 12; ++i) printf(" %u", r[i]);
        printf(" | dword of lane 63's first value at index:");
        for (int i = 0; i < 320; ++i)
            if (r[i] == 6300u) printf(" %d", i);
        printf("\n");
    };
    run(k<4>, 4);
    run(k<12>, 12);
    run(k<16>, 16);
    return 0;
}
