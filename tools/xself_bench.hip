// xself_bench.hip — developer micro-benchmark: the two x-normal faces of a periodic SELF exchange
// of a 516^3 fp64 field at halo 2 (512 x 512 rows of 16 B per face, row pitch 4128 B).
// Box A (left halo): pack reads row bytes [4096,4112), unpack writes [0,16).
// Box B (right halo): pack reads [16,32), unpack writes [4112,4128).
// So the 32 B chunk [0,32) of a row is read by B's pack and written by A's unpack (and likewise
// [4096,4128)). Question: does co-scheduling A and B on the same rows in one workgroup (the read
// and the partial write of a chunk meet in L2) beat processing the boxes in separate tiles?
//   sep : tiles of A, then tiles of B; each tile packs its rows, barrier, unpacks them
//   co  : each tile packs A and B for its rows, barrier, unpacks A and B
//   pk/up: pack-only / unpack-only launches of both faces (the two-launch form)
// Build: hipcc -O3 --offload-arch=gfx950 tools/xself_bench.hip -o tools/bin/xself_bench
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
constexpr int N = 512, H = 2, E = N + 2 * H;
constexpr long SY = long(E) * 8, SZ = long(E) * E * 8;
constexpr long ROWS = long(N) * N;
constexpr long RD_A = long(N) * 8, WR_A = 0, RD_B = H * 8, WR_B = long(N + H) * 8;

__device__ __forceinline__ long row_off(long i)
{
    const long y = i % N, z = i / N;
    return (z + H) * SZ + (y + H) * SY;
}

template<int U>
__device__ __forceinline__ void copy_rows(char* __restrict__ f, char* __restrict__ buf, long r0,
                                          long r1, long foff, bool pack)
{
    for (long b = r0 + threadIdx.x; b < r1; b += 256 * U)
    {
        v4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const long i = b + u * 256;
            if (i < r1)
                v[u] = pack ? *(const v4*)(f + row_off(i) + foff) : *(const v4*)(buf + i * 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const long i = b + u * 256;
            if (i < r1)
            {
                if (pack) *(v4*)(buf + i * 16) = v[u];
                else *(v4*)(f + row_off(i) + foff) = v[u];
            }
        }
    }
}

// mode 0 = sep, 1 = co, 2 = pack only, 3 = unpack only
template<int MODE>
__global__ __launch_bounds__(256) void k(char* f, char* bufA, char* bufB, long T)
{
    const long tiles = (ROWS + T - 1) / T;
    long t = blockIdx.x;
    if (MODE == 1)
    {
        const long r0 = t * T, r1 = r0 + T < ROWS ? r0 + T : ROWS;
        copy_rows<4>(f, bufA, r0, r1, RD_A, true);
        copy_rows<4>(f, bufB, r0, r1, RD_B, true);
        __syncthreads();
        copy_rows<4>(f, bufA, r0, r1, WR_A, false);
        copy_rows<4>(f, bufB, r0, r1, WR_B, false);
        return;
    }
    const bool isB = t >= tiles;
    if (isB) t -= tiles;
    char* buf = isB ? bufB : bufA;
    const long r0 = t * T, r1 = r0 + T < ROWS ? r0 + T : ROWS;
    if (MODE == 0 || MODE == 2) copy_rows<4>(f, buf, r0, r1, isB ? RD_B : RD_A, true);
    if (MODE == 0) __syncthreads();
    if (MODE == 0 || MODE == 3) copy_rows<4>(f, buf, r0, r1, isB ? WR_B : WR_A, false);
}

__global__ void touch(char* p, long n)
{
    for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 16; i < n; i += long(gridDim.x) * 256 * 16)
        *(v4*)(p + i) = v4{1, 2, 3, 4};
}

int main()
{
    const long fbytes = SZ * E;
    char *f, *bufA, *bufB, *flush;
    CK(hipMalloc(&f, fbytes));
    CK(hipMalloc(&bufA, ROWS * 16));
    CK(hipMalloc(&bufB, ROWS * 16));
    const long flush_bytes = 1l << 30;
    CK(hipMalloc(&flush, flush_bytes));
    CK(hipMemset(f, 0, fbytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double useful = 4.0 * ROWS * 16;  // both faces, pack + unpack (read + write each)
    for (int cold = 0; cold < 2; ++cold)
        for (long T : {256l, 1024l, 4096l})
        {
            const long tiles = (ROWS + T - 1) / T;
            float us[5] = {0, 0, 0, 0, 0};
            const int reps = 20;
            for (int m = 0; m < 5; ++m)
                for (int r = 0; r < reps + 2; ++r)
                {
                    if (cold) hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, flush, flush_bytes);
                    CK(hipEventRecord(e0));
                    switch (m)
                    {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(2 * tiles), dim3(256), 0, 0, f, bufA, bufB, T); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(tiles), dim3(256), 0, 0, f, bufA, bufB, T); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(2 * tiles), dim3(256), 0, 0, f, bufA, bufB, T); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(2 * tiles), dim3(256), 0, 0, f, bufA, bufB, T); break;
                    case 4:
                        hipLaunchKernelGGL(k<2>, dim3(2 * tiles), dim3(256), 0, 0, f, bufA, bufB, T);
                        hipLaunchKernelGGL(k<3>, dim3(2 * tiles), dim3(256), 0, 0, f, bufA, bufB, T);
                        break;
                    }
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 2) us[m] += ms * 1000.f / reps;
                }
            printf("{\"cold\":%d,\"tile_rows\":%ld,\"sep_us\":%.2f,\"co_us\":%.2f,\"pack_us\":%.2f,"
                   "\"unpack_us\":%.2f,\"pack_then_unpack_us\":%.2f,\"co_useful_GBps\":%.1f,"
                   "\"sep_useful_GBps\":%.1f}\n",
                   cold, T, us[0], us[1], us[2], us[3], us[4], useful / us[1] / 1e3,
                   useful / us[0] / 1e3);
        }
    return 0;
}
