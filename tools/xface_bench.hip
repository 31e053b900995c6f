// xface_bench.hip — developer micro-benchmark of the unit-stride-face access pattern:
// gather L bytes from each of R rows strided S bytes apart into a contiguous buffer (pack) or
// scatter back (unpack), as the x-normal faces of a 516^3 fp64 field at halo 2 do
// (L = 16 B, S = 4128 B, 512 x 512 rows per face). Variants: row order (y- or z-fastest),
// bytes per lane, loads in flight per lane, grid size, warm (Infinity-Cache resident) or cold.
// Build: hipcc -O3 --offload-arch=gfx950 tools/xface_bench.hip -o gpurun_out/xface_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

struct args
{
    char* field;
    char* buf;
    long sy, sz;        // row strides (y, z) in bytes
    int ny, nz;         // rows per dim
    int zfast;          // 1: consecutive lanes walk z
    long off;           // byte offset of the row start
    int lanes_per_row;  // 1 (16 B per row) or 4 (64 B per row)
};

template<int U, bool PACK>
__global__ __launch_bounds__(256) void k(args a, long nvec)
{
    const long stride = long(gridDim.x) * 256;
    for (long base = long(blockIdx.x) * 256 * U + threadIdx.x; base < nvec; base += stride * U)
    {
        v4 v[U];
        long fo[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            long i = base + long(u) * 256;
            long row = i / a.lanes_per_row;
            long col = i % a.lanes_per_row;
            long y, z;
            if (a.zfast)
            {
                z = row % a.nz;
                y = row / a.nz;
            }
            else
            {
                y = row % a.ny;
                z = row / a.ny;
            }
            fo[u] = a.off + z * a.sz + y * a.sy + col * 16;
            if (i < nvec) v[u] = PACK ? *(const v4*)(a.field + fo[u]) : *(const v4*)(a.buf + i * 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            long i = base + long(u) * 256;
            if (i < nvec)
            {
                if (PACK) *(v4*)(a.buf + i * 16) = v[u];
                else *(v4*)(a.field + fo[u]) = v[u];
            }
        }
    }
}

__global__ void touch(char* p, long n)
{
    for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 16; i < n; i += long(gridDim.x) * 256 * 16)
        *(v4*)(p + i) = v4{1, 2, 3, 4};
}

template<int U, bool PACK>
float run(args a, long nvec, int grid, bool cold, char* flush, long flush_bytes, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps + 2; ++r)
    {
        if (cold) hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, flush, flush_bytes);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((k<U, PACK>), dim3(grid), dim3(256), 0, 0, a, nvec);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2)
        {
            sum += ms;
            if (ms < best) best = ms;
        }
    }
    return sum / reps * 1000.f;
}

int main()
{
    const int N = 512, H = 2, E = N + 2 * H;
    const long sy = long(E) * 8, sz = long(E) * E * 8;
    const long fbytes = sz * E;
    char *field, *buf, *flush;
    CK(hipMalloc(&field, fbytes));
    CK(hipMalloc(&buf, 64l << 20));
    const long flush_bytes = 1l << 30;
    CK(hipMalloc(&flush, flush_bytes));
    CK(hipMemset(field, 0, fbytes));
    printf("{\"rows\":%d,\"row_stride\":%ld}\n", N * N, sy);
    for (int cold = 0; cold < 2; ++cold)
        for (int zfast = 0; zfast < 2; ++zfast)
            for (int lpr : {1, 4})
                for (int grid : {512, 2048, 8192})
                {
                    args a{field, buf, sy, sz, N, N, zfast, 16, lpr};
                    const long nvec = long(N) * N * lpr;
                    const double alg = 2.0 * N * N * 16;  // useful bytes read+written
                    float t4p = run<4, true>(a, nvec, grid, cold, flush, flush_bytes, 10);
                    float t8p = run<8, true>(a, nvec, grid, cold, flush, flush_bytes, 10);
                    float t4u = run<4, false>(a, nvec, grid, cold, flush, flush_bytes, 10);
                    printf("{\"cold\":%d,\"zfast\":%d,\"bytes_per_row\":%d,\"grid\":%d,"
                           "\"pack_u4_us\":%.2f,\"pack_u8_us\":%.2f,\"unpack_u4_us\":%.2f,"
                           "\"pack_u4_useful_GBps\":%.1f,\"unpack_u4_useful_GBps\":%.1f}\n",
                           cold, zfast, 16 * lpr, grid, t4p, t8p, t4u, alg / t4p / 1e3,
                           alg / t4u / 1e3);
                }
    // streaming reference: contiguous 8 MiB pack-like copy
    {
        args a{field, buf, 16, 1l << 40, 1 << 19, 1, 0, 0, 1};
        const long nvec = 1l << 19;
        for (int cold = 0; cold < 2; ++cold)
        {
            float t = run<4, true>(a, nvec, 2048, cold, flush, flush_bytes, 10);
            printf("{\"contiguous_8MiB\":1,\"cold\":%d,\"us\":%.2f,\"GBps\":%.1f}\n", cold, t,
                   2.0 * nvec * 16 / t / 1e3);
        }
    }
    return 0;
}
