// perm2_bench.hip — developer micro-benchmark: x-face gather (16 B rows, 4128 B pitch, 512 x 512
// rows) with the rows of each 4096-row workgroup tile visited in the order r = (j * S) mod 4096
// (S odd), values staged through LDS so the buffer is still written lane-linearly.
// Does any visiting order spread the row requests better over the memory channels?
// Build: hipcc -O3 --offload-arch=gfx950 tools/perm2_bench.hip -o tools/bin/perm2_bench
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
constexpr int T = 4096;  // rows per tile

template<bool PACK>
__global__ __launch_bounds__(256) void k(char* __restrict__ field, char* __restrict__ buf,
                                         long pitch, long off, unsigned S)
{
    __shared__ v4 st[T];
    const long base = long(blockIdx.x) * T;
    const int t = threadIdx.x;
    if (PACK)
    {
        for (int it = 0; it < T / 1024; ++it)
        {
            v4 v[4];
            int r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                const unsigned j = unsigned(it * 1024 + u * 256 + t);
                r[u] = int((j * S) & (T - 1));
                v[u] = *(const v4*)(field + (base + r[u]) * pitch + off);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) st[r[u]] = v[u];
        }
        __syncthreads();
        for (int j = t; j < T; j += 256) *(v4*)(buf + (base + j) * 16) = st[j];
    }
    else
    {
        for (int j = t; j < T; j += 256) st[j] = *(const v4*)(buf + (base + j) * 16);
        __syncthreads();
        for (int it = 0; it < T / 1024; ++it)
        {
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                const unsigned j = unsigned(it * 1024 + u * 256 + t);
                const int r = int((j * S) & (T - 1));
                *(v4*)(field + (base + r) * pitch + off) = st[r];
            }
        }
    }
}

int main()
{
    const long rows = 262144, pitch = 4128;
    char *src, *dst;
    CK(hipMalloc(&src, rows * pitch + 8192));
    CK(hipMalloc(&dst, 64l << 20));
    CK(hipMemset(src, 1, rows * pitch + 8192));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int dir = 0; dir < 2; ++dir)
        for (unsigned S : {1u, 3u, 5u, 7u, 9u, 17u, 31u, 33u, 63u, 65u, 127u, 129u, 255u, 257u, 511u,
                           513u, 1023u, 1025u, 2047u, 2049u})
        {
            float sum = 0;
            const int reps = 20;
            for (int rp = 0; rp < reps + 3; ++rp)
            {
                CK(hipEventRecord(e0));
                if (dir == 0)
                    hipLaunchKernelGGL((k<true>), dim3(rows / T), dim3(256), 0, 0, src, dst, pitch, 16l, S);
                else
                    hipLaunchKernelGGL((k<false>), dim3(rows / T), dim3(256), 0, 0, src, dst, pitch, 0l, S);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rp >= 3) sum += ms;
            }
            printf("{\"dir\":\"%s\",\"S\":%u,\"us\":%.2f}\n", dir ? "unpack" : "pack", S,
                   sum / reps * 1000.f);
        }
    return 0;
}
