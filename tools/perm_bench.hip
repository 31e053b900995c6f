// perm_bench.hip — developer micro-benchmark: 16-byte row gather/scatter at the field's row
// pitch (4128 B = 516 fp64) with a permuted lane->row mapping inside each 1024-row block, so that
// the 64 lanes of a wave touch rows S apart (their 16 B pieces then sit at distinct 128 B line
// positions), with the buffer side written/read directly (scattered 16 B) or through LDS
// (transposed back to contiguous 16 B per lane).
// Build: hipcc -O3 --offload-arch=gfx950 tools/perm_bench.hip -o tools/bin/perm_bench
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

__device__ __forceinline__ int perm(int j, int S)
{
    if (S == 1) return j;
    const int g = 64 * S;
    return (j % 64) * S + (j / 64) % S + (j / g) * g;
}

// pack: rows -> buffer. LDS: 0 direct scattered buffer writes, 1 via LDS transpose
template<bool PACK, int LDS>
__global__ __launch_bounds__(256) void k(char* __restrict__ field, char* __restrict__ buf,
                                         long pitch, long off, int rows, int S)
{
    __shared__ v4 st[1024];
    const int blk0 = blockIdx.x * 1024;
    if (blk0 >= rows) return;
    const int t = threadIdx.x;
    v4 v[4];
    int r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = perm(u * 256 + t, S);
    if (PACK)
    {
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *(const v4*)(field + long(blk0 + r[u]) * pitch + off);
        if (LDS)
        {
#pragma unroll
            for (int u = 0; u < 4; ++u) st[r[u]] = v[u];
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 4; ++u)
                *(v4*)(buf + long(blk0 + u * 256 + t) * 16) = st[u * 256 + t];
        }
        else
        {
#pragma unroll
            for (int u = 0; u < 4; ++u) *(v4*)(buf + long(blk0 + r[u]) * 16) = v[u];
        }
    }
    else
    {
        if (LDS)
        {
#pragma unroll
            for (int u = 0; u < 4; ++u) st[u * 256 + t] = *(const v4*)(buf + long(blk0 + u * 256 + t) * 16);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = st[r[u]];
        }
        else
        {
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *(const v4*)(buf + long(blk0 + r[u]) * 16);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) *(v4*)(field + long(blk0 + r[u]) * pitch + off) = v[u];
    }
}

int main()
{
    const int rows = 262144;
    const long pitch = 4128;
    char *src, *dst;
    CK(hipMalloc(&src, rows * pitch + 4096));
    CK(hipMalloc(&dst, 64l << 20));
    CK(hipMemset(src, 1, rows * pitch + 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int dir = 0; dir < 2; ++dir)
        for (int lds = 0; lds < 2; ++lds)
            for (int S : {1, 2, 4, 8, 16})
            {
                float sum = 0;
                const int reps = 20;
                for (int rp = 0; rp < reps + 3; ++rp)
                {
                    CK(hipEventRecord(e0));
                    if (dir == 0 && lds == 0) hipLaunchKernelGGL((k<true, 0>), dim3(rows / 1024), dim3(256), 0, 0, src, dst, pitch, 16l, rows, S);
                    if (dir == 0 && lds == 1) hipLaunchKernelGGL((k<true, 1>), dim3(rows / 1024), dim3(256), 0, 0, src, dst, pitch, 16l, rows, S);
                    if (dir == 1 && lds == 0) hipLaunchKernelGGL((k<false, 0>), dim3(rows / 1024), dim3(256), 0, 0, src, dst, pitch, 0l, rows, S);
                    if (dir == 1 && lds == 1) hipLaunchKernelGGL((k<false, 1>), dim3(rows / 1024), dim3(256), 0, 0, src, dst, pitch, 0l, rows, S);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (rp >= 3) sum += ms;
                }
                printf("{\"dir\":\"%s\",\"lds\":%d,\"S\":%d,\"us\":%.2f}\n", dir ? "unpack" : "pack",
                       lds, S, sum / reps * 1000.f);
            }
    return 0;
}
