// line_bench.hip — developer micro-benchmark: are the x-face halo writes slow because they are
// PARTIAL lines (masked writes the memory side has to merge) rather than because of their count?
// 516^3 fp64 field, halo 2, 512 x 512 interior rows (pitch 4128 B). The x-face halo bytes of row
// r's right side and row r+1's left side are adjacent: boundary r|r+1 has the 32-B halo pair
// [row_off(r) + 4112, row_off(r) + 4144) between interior x=512,513 of row r and x=2,3 of r+1.
//   w16    : one lane per (row, side) writes the 16-B halo from a linear buffer (= unpack today)
//   wspan32: one lane per boundary writes the 32-B halo pair (two 16-B stores)
//   wblk64 : the 64-B aligned blocks covering the halo pair are read and written back in full
//            (4 lanes per block, interior bytes rewritten unchanged)
//   wline  : the same with whole 128-B lines (8 lanes per line)
//   rspan  : read-only: the 64-B span around the halo pair (4 lanes per boundary)
//   rline  : read-only: the 128-B lines covering the halo pair (8 lanes per line)
//   self16 : x-face self exchange, halo bytes only (2 loads, 2 stores of 16 B per row)
//   rs8 / rs64 / rg8 : random scatter of 500k 8-B values into a 10M-cell fp64 array (plain 8-B
//            stores / read + full rewrite of the 64-B block holding the value) and random gather
// Build: hipcc -O3 --offload-arch=gfx950 tools/line_bench.hip -o tools/bin/line_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
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
using v2 = unsigned __attribute__((ext_vector_type(2)));
#define G __attribute__((address_space(1)))
constexpr int N = 512, H = 2, E = N + 2 * H;
constexpr long SY = long(E) * 8, SZ = long(E) * E * 8;
constexpr long ROWS = long(N) * N;
constexpr long NB = long(N) * (N - 1);  // boundaries (z, y) with y in [0, N-1)
constexpr long UC = 10000000, UH = 500000;  // unstructured cells, halo values

__device__ __forceinline__ long row_off(long r)
{
    return (r / N + H) * SZ + (r % N + H) * SY;
}

__device__ __forceinline__ long bnd_row(long b)
{
    return (b / (N - 1)) * N + (b % (N - 1));
}

template<int MODE>
__global__ __launch_bounds__(256) void k(char* f, char* buf, const int* idx, char* u)
{
    const long gid = long(blockIdx.x) * 256 + threadIdx.x;
    if (MODE == 0)  // w16
    {
        const long r = gid >> 1, side = gid & 1;
        if (r >= ROWS) return;
        const v4 v = *(const G v4*)(buf + gid * 16);
        *(G v4*)(f + row_off(r) + (side ? 4112 : 0)) = v;
    }
    else if (MODE == 1)  // wspan32
    {
        if (gid >= NB) return;
        char* p = f + row_off(bnd_row(gid)) + 4112;
        const v4 v = *(const G v4*)(buf + gid * 32);
        const v4 w = *(const G v4*)(buf + gid * 32 + 16);
        *(G v4*)(p) = v;
        *(G v4*)(p + 16) = w;
    }
    else if (MODE == 2 || MODE == 4)  // wblk64 / rspan: 4 lanes per boundary
    {
        const long b = gid >> 2, q = gid & 3;
        if (b >= NB) return;
        const long h = row_off(bnd_row(b)) + 4112;  // halo pair [h, h+32)
        if (MODE == 4)
        {
            const v4 v = *(const G v4*)(f + h - 16 + q * 16);
            *(G v4*)(buf + gid * 16) = v;
            return;
        }
        const long b0 = h & ~63l, b1 = (h + 31) & ~63l;
        {
            char* p = f + b0 + q * 16;
            v4 v = *(const G v4*)(p);
            v.x ^= 1u;
            *(G v4*)(p) = v;
        }
        if (b1 != b0)
        {
            char* p = f + b1 + q * 16;
            v4 v = *(const G v4*)(p);
            v.x ^= 1u;
            *(G v4*)(p) = v;
        }
    }
    else if (MODE == 3 || MODE == 5)  // wline / rline: 8 lanes per boundary
    {
        const long b = gid >> 3, q = gid & 7;
        if (b >= NB) return;
        const long h = row_off(bnd_row(b)) + 4112;
        const long l0 = h & ~127l, l1 = (h + 31) & ~127l;
        if (MODE == 5)
        {
            v4 v = *(const G v4*)(f + l0 + q * 16);
            if (l1 != l0) v += *(const G v4*)(f + l1 + q * 16);
            *(G v4*)(buf + gid * 16) = v;
            return;
        }
        {
            char* p = f + l0 + q * 16;
            v4 v = *(const G v4*)(p);
            v.x ^= 1u;
            *(G v4*)(p) = v;
        }
        if (l1 != l0)
        {
            char* p = f + l1 + q * 16;
            v4 v = *(const G v4*)(p);
            v.x ^= 1u;
            *(G v4*)(p) = v;
        }
    }
    else if (MODE == 6)  // self16
    {
        const long r = gid;
        if (r >= ROWS) return;
        char* p = f + row_off(r);
        const v4 in_l = *(const G v4*)(p + 16);
        const v4 in_r = *(const G v4*)(p + 4096);
        *(G v4*)(p) = in_r;
        *(G v4*)(p + 4112) = in_l;
    }
    else if (MODE == 7)  // rs8: random 8-B scatter
    {
        if (gid >= UH) return;
        const v2 v = *(const G v2*)(buf + gid * 8);
        *(G v2*)(u + long(idx[gid]) * 8) = v;
    }
    else if (MODE == 8)  // rs64: read + full rewrite of the value's 64-B block (4 lanes)
    {
        const long i = gid >> 2, q = gid & 3;
        if (i >= UH) return;
        const long a = long(idx[i]) * 8;
        char* p = u + (a & ~63l) + q * 16;
        v4 v = *(const G v4*)(p);
        v.x ^= 1u;
        *(G v4*)(p) = v;
    }
    else if (MODE == 9)  // rg8: random 8-B gather
    {
        if (gid >= UH) return;
        const v2 v = *(const G v2*)(u + long(idx[gid]) * 8);
        *(G v2*)(buf + gid * 8) = v;
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
    char *f, *buf, *flush, *u;
    int* idx;
    CK(hipMalloc(&f, fbytes));
    CK(hipMalloc(&buf, ROWS * 128));
    CK(hipMalloc(&u, UC * 8));
    CK(hipMalloc(&idx, UH * 4));
    const long flush_bytes = 1l << 30;
    CK(hipMalloc(&flush, flush_bytes));
    CK(hipMemset(f, 0, fbytes));
    CK(hipMemset(buf, 0, ROWS * 128));
    CK(hipMemset(u, 0, UC * 8));
    {
        std::vector<int> perm(UC);
        std::iota(perm.begin(), perm.end(), 0);
        std::mt19937_64 rng(20260715);
        std::shuffle(perm.begin(), perm.end(), rng);
        CK(hipMemcpy(idx, perm.data(), UH * 4, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int NM = 10;
    const char* names[NM] = {"w16", "wspan32", "wblk64", "wline", "rspan", "rline", "self16",
                             "rs8", "rs64", "rg8"};
    const long threads[NM] = {2 * ROWS, NB, 4 * NB, 8 * NB, 4 * NB, 8 * NB, ROWS, UH, 4 * UH, UH};
    for (int cold = 0; cold < 2; ++cold)
        for (int m = 0; m < NM; ++m)
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
                case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 7: hipLaunchKernelGGL(k<7>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 8: hipLaunchKernelGGL(k<8>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
                case 9: hipLaunchKernelGGL(k<9>, dim3(grid), dim3(256), 0, 0, f, buf, idx, u); break;
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
