// sector_bench.hip — developer micro-benchmark: are the x-face halo writes slow because they are
// HALF 32-B sectors? 516^3 fp64 field, halo 2, 2 x 512 x 512 rows (pitch 4128 B, every row start
// 32-B aligned). Left halo = row bytes [0,16) (sector [0,32) also holds interior x=2,3),
// right halo = [4112,4128) (sector [4096,4128) also holds interior x=512,513).
//   w16  : one lane per (row, side) writes the 16-B halo                  (what unpack does)
//   w32p : two lanes per (row, side) write the whole 32-B sector in one store instruction
//   w32s : one lane writes the whole sector as two 16-B stores
//   self16: self exchange of the x-faces, both sides of a row in one lane: 2 loads, 2 halo stores
//   self32: the same, storing full sectors {halo, interior} (the interior value rewritten as read)
//   wpair : lanes 2j / 2j+1 write row r's right halo and row r+1's left halo — 32 contiguous
//           bytes in one store instruction (rows are adjacent in memory: 4128-B pitch)
//   selfpair: self exchange with the same lane pairing of the halo writes
// Build: hipcc -O3 --offload-arch=gfx950 tools/sector_bench.hip -o tools/bin/sector_bench
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
#define G __attribute__((address_space(1)))
constexpr int N = 512, H = 2, E = N + 2 * H;
constexpr long SY = long(E) * 8, SZ = long(E) * E * 8;
constexpr long ROWS = long(N) * N;

__device__ __forceinline__ long row_off(long r)
{
    return (r / N + H) * SZ + (r % N + H) * SY;
}

template<int MODE>
__global__ __launch_bounds__(256) void k(char* f, const char* buf)
{
    const long gid = long(blockIdx.x) * 256 + threadIdx.x;
    if (MODE == 0)  // w16: gid over 2*ROWS (row, side)
    {
        const long r = gid >> 1, side = gid & 1;
        if (r >= ROWS) return;
        const v4 v = *(const G v4*)(buf + gid * 16);
        *(G v4*)(f + row_off(r) + (side ? 4112 : 0)) = v;
    }
    else if (MODE == 1)  // w32p: gid over 4*ROWS (row, side, half)
    {
        const long r = gid >> 2, side = (gid >> 1) & 1, half = gid & 1;
        if (r >= ROWS) return;
        const v4 v = *(const G v4*)(buf + gid * 16);
        *(G v4*)(f + row_off(r) + (side ? 4096 : 0) + half * 16) = v;
    }
    else if (MODE == 2)  // w32s
    {
        const long r = gid >> 1, side = gid & 1;
        if (r >= ROWS) return;
        const v4 v = *(const G v4*)(buf + gid * 32);
        const v4 w = *(const G v4*)(buf + gid * 32 + 16);
        char* p = f + row_off(r) + (side ? 4096 : 0);
        *(G v4*)(p) = v;
        *(G v4*)(p + 16) = w;
    }
    else if (MODE == 5 || MODE == 6)  // wpair / selfpair: gid over 2*ROWS (boundary r|r+1, side)
    {
        const long r = gid >> 1, second = gid & 1;
        if (r >= ROWS) return;
        const long row = r + second;  // second lane: row r+1's left halo
        if (row >= ROWS) return;
        char* p = f + row_off(row);
        v4 v;
        if (MODE == 5) v = *(const G v4*)(buf + gid * 16);
        else v = *(const G v4*)(p + (second ? 4096 : 16));
        *(G v4*)(p + (second ? 0 : 4112)) = v;
    }
    else if (MODE == 3 || MODE == 4)  // self16 / self32: gid over ROWS
    {
        const long r = gid;
        if (r >= ROWS) return;
        char* p = f + row_off(r);
        const v4 in_l = *(const G v4*)(p + 16);    // interior x = 2,3
        const v4 in_r = *(const G v4*)(p + 4096);  // interior x = 512,513
        if (MODE == 3)
        {
            *(G v4*)(p) = in_r;           // left halo  <- right interior
            *(G v4*)(p + 4112) = in_l;    // right halo <- left interior
        }
        else
        {
            *(G v4*)(p) = in_r;
            *(G v4*)(p + 16) = in_l;      // unchanged interior, completes sector [0,32)
            *(G v4*)(p + 4096) = in_r;    // unchanged interior, completes sector [4096,4128)
            *(G v4*)(p + 4112) = in_l;
        }
    }
}

__global__ void touch(char* p, long n)
{
    for (long i = (long(blockIdx.x) * 256 + threadIdx.x) * 16; i < n; i += long(gridDim.x) * 256 * 16)
        *(v4*)(p + i) = v4{1, 2, 3, 4};
}

int main()
{
    const long fbytes = SZ * E;
    char *f, *buf, *flush;
    CK(hipMalloc(&f, fbytes));
    CK(hipMalloc(&buf, ROWS * 64));
    const long flush_bytes = 1l << 30;
    CK(hipMalloc(&flush, flush_bytes));
    CK(hipMemset(f, 0, fbytes));
    CK(hipMemset(buf, 0, ROWS * 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[7] = {"w16", "w32p", "w32s", "self16", "self32", "wpair", "selfpair"};
    const long threads[7] = {2 * ROWS, 4 * ROWS, 2 * ROWS, ROWS, ROWS, 2 * ROWS, 2 * ROWS};
    for (int cold = 0; cold < 2; ++cold)
        for (int m = 0; m < 7; ++m)
        {
            float us = 0;
            const int reps = 20;
            const unsigned grid = unsigned((threads[m] + 255) / 256);
            for (int r = 0; r < reps + 2; ++r)
            {
                if (cold) hipLaunchKernelGGL(touch, dim3(4096), dim3(256), 0, 0, flush, flush_bytes);
                CK(hipEventRecord(e0));
                switch (m)
                {
                case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(grid), dim3(256), 0, 0, f, buf); break;
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) us += ms * 1000.f / reps;
            }
            printf("{\"cold\":%d,\"mode\":\"%s\",\"us\":%.2f}\n", cold, names[m], us);
        }
    return 0;
}
