// order_bench.hip — developer micro-benchmark: is the x-face read rate a property of the ADDRESS
// SET (pitch 4,128 B rows of a 516^3 fp64 field) or of the ORDER the rows are visited in?
// 262,144 reads of one 64-B span each (4 lanes x 16 B), written linearly to a buffer:
//   natural : span k = boundary k (y fastest, then z) — what the x-face tiles do
//   zfast   : z fastest, then y
//   random  : a uniformly random permutation of the same spans
//   uniform : 262,144 64-B spans at uniformly random 64-B-aligned offsets of the same 1.1 GB field
//   pitch4224 / pitch4160 : the natural order over a field whose rows are 4,224 / 4,160 B apart
// Build: hipcc -O3 --offload-arch=gfx950 tools/order_bench.hip -o tools/bin/order_bench
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
#define G __attribute__((address_space(1)))
constexpr int N = 512, H = 2, E = N + 2 * H;
constexpr long NS = long(N) * N;  // spans

__global__ __launch_bounds__(256) void k(const char* f, char* buf, const long* off)
{
    const long gid = long(blockIdx.x) * 256 + threadIdx.x;
    const long s = gid >> 2, q = gid & 3;
    if (s >= NS) return;
    const v4 v = *(const G v4*)(f + off[s] + q * 16);
    *(G v4*)(buf + gid * 16) = v;
}

int main()
{
    const long pitches[3] = {long(E) * 8, 4224, 4160};
    const long fbytes = long(E) * E * 4224 + 8192;
    char *f, *buf;
    long* doff;
    CK(hipMalloc(&f, fbytes));
    CK(hipMalloc(&buf, NS * 64));
    CK(hipMalloc(&doff, NS * 8));
    CK(hipMemset(f, 1, fbytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::mt19937_64 rng(7);
    const char* names[6] = {"natural", "zfast", "random", "uniform", "pitch4224", "pitch4160"};
    for (int m = 0; m < 6; ++m)
    {
        const long SY = m == 4 ? pitches[1] : m == 5 ? pitches[2] : pitches[0];
        const long SZ = SY * E;
        std::vector<long> off(NS);
        for (long s = 0; s < NS; ++s)
        {
            long y = s % N, z = s / N;
            if (m == 1) std::swap(y, z);
            // span around the right halo of row (y, z): interior x = 512,513 .. next row x = 3
            off[s] = (z + H) * SZ + (y + H) * SY + 4096;
        }
        if (m == 2) std::shuffle(off.begin(), off.end(), rng);
        if (m == 3)
        {
            std::uniform_int_distribution<long> d(0, long(E) * E * E * 8 / 64 - 2);
            for (auto& o : off) o = d(rng) * 64;
        }
        CK(hipMemcpy(doff, off.data(), NS * 8, hipMemcpyHostToDevice));
        float us = 0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r)
        {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k, dim3(unsigned(NS * 4 / 256)), dim3(256), 0, 0, f, buf, doff);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) us += ms * 1000.f / reps;
        }
        printf("{\"order\":\"%s\",\"us\":%.2f,\"Gspans_per_s\":%.1f}\n", names[m], us, NS / us / 1e3);
    }
    return 0;
}
