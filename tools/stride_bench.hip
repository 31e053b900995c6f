// stride_bench.hip — developer micro-benchmark: rate of 16-byte row gathers as a function of the
// row pitch and of the ORDER in which the rows are issued (lane i of the grid reads row
// perm(i) = (i % G) * (R / G) + i / G, i.e. G interleaved streams).
// Build: hipcc -O3 --offload-arch=gfx950 tools/stride_bench.hip -o tools/bin/stride_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do                                                                                       \
    {                                                                                        \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess)                                                                 \
        {                                                                                    \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                  \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

using v4 = unsigned __attribute__((ext_vector_type(4)));

template<int U>
__global__ __launch_bounds__(256) void gather(const char* __restrict__ src, char* __restrict__ dst,
                                              long pitch, long rows, long G, long off)
{
    const long gs = long(gridDim.x) * 256;
    const long per = rows / G;
    for (long base = long(blockIdx.x) * 256 * U + threadIdx.x; base < rows; base += gs * U)
    {
        v4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const long i = base + long(u) * 256;
            const long r = (i % G) * per + i / G;
            if (i < rows) v[u] = *(const v4*)(src + r * pitch + off);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const long i = base + long(u) * 256;
            if (i < rows) *(v4*)(dst + i * 16) = v[u];
        }
    }
}

int main()
{
    const long rows = 262144;
    const long span = rows * 8320 + 4096;
    char *src, *dst;
    CK(hipMalloc(&src, span));
    CK(hipMalloc(&dst, 64l << 20));
    CK(hipMemset(src, 1, span));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct cfg
    {
        long pitch, G, off;
    };
    const cfg cs[] = {{4096, 1, 0},  {4128, 1, 0},  {4128, 1, 16}, {4160, 1, 0},  {4224, 1, 0},
                      {4352, 1, 0},  {4128, 2, 16}, {4128, 4, 16}, {4128, 8, 16}, {4128, 16, 16},
                      {4128, 64, 16}, {4128, 512, 16}, {4128, 4096, 16}, {8256, 1, 16},
                      {2064, 1, 16}, {1032, 1, 16}};
    for (const auto& c : cs)
    {
        float sum = 0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r)
        {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL((gather<4>), dim3(2048), dim3(256), 0, 0, src, dst, c.pitch, rows,
                               c.G, c.off);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) sum += ms;
        }
        const float us = sum / reps * 1000.f;
        printf("{\"pitch\":%ld,\"G\":%ld,\"off\":%ld,\"us\":%.2f}\n", c.pitch, c.G, c.off, us);
    }
    return 0;
}
