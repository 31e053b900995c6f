// row_scatter_ab.hip — developer measurement (not product): why config 5's levels-8 scatter
// (500k random 64-B rows of an 84 MB x 8 field, levels first) runs slower than the index-list
// floor probe. Variants of the same scatter (buffer lane-linear -> field rows at random lids),
// each timed by its own events (median of 21), warm:
//   gs8     grid-stride, 8 B per lane (the probe, tools/pack_floor.hip k_iscatter)
//   gs16    grid-stride, 16 B per lane
//   t16_U   tiles of 16 KiB per workgroup, 16 B per lane, U vectors per lane in flight (the
//           product's copy_tile shape: lid loads, buffer loads, then stores)
//   t8_U    the same with 8 B per lane
// One JSON line per variant.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                \
    do                                                                       \
    {                                                                        \
        if ((x) != hipSuccess)                                               \
        {                                                                    \
            printf("{\"error\": \"HIP error at line %d\"}\n", __LINE__);     \
            return 1;                                                        \
        }                                                                    \
    } while (0)

using v2 = unsigned __attribute__((ext_vector_type(2)));
using v4 = unsigned __attribute__((ext_vector_type(4)));

template<typename V>
__global__ __launch_bounds__(256) void k_gs(char* __restrict__ f, const int* __restrict__ lids,
                                            const char* __restrict__ buf, uint64_t bytes)
{
    constexpr int W = sizeof(V);
    for (uint64_t p = (uint64_t(blockIdx.x) * 256 + threadIdx.x) * W; p < bytes;
         p += uint64_t(gridDim.x) * 256 * W)
    {
        const uint64_t row = p / 64, col = p % 64;
        *(V*)(f + uint64_t(lids[row]) * 64 + col) = *(const V*)(buf + p);
    }
}

template<typename V, int U>
__global__ __launch_bounds__(256) void k_tile(char* __restrict__ f, const int* __restrict__ lids,
                                              const char* __restrict__ buf, uint64_t bytes,
                                              uint32_t tile)
{
    constexpr int W = sizeof(V);
    const uint64_t start = uint64_t(blockIdx.x) * tile;
    const uint64_t end = std::min<uint64_t>(bytes, start + tile);
    for (uint64_t base = start + threadIdx.x * W; base < end; base += uint64_t(U) * 256 * W)
    {
        V v[U];
        uint64_t fo[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint64_t p = base + uint64_t(u) * 256 * W;
            if (p < end) fo[u] = uint64_t(lids[p / 64]) * 64 + p % 64;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint64_t p = base + uint64_t(u) * 256 * W;
            if (p < end) v[u] = *(const V*)(buf + p);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint64_t p = base + uint64_t(u) * 256 * W;
            if (p < end) *(V*)(f + fo[u]) = v[u];
        }
    }
}

int main()
{
    const size_t cells = 10500000, n = 500000, bytes = n * 64;
    std::vector<int> h(cells);
    for (size_t i = 0; i < cells; ++i) h[i] = int(i);
    unsigned long long x = 20260715ull;
    for (size_t i = cells - 1; i > 0; --i)
    {
        x += 0x9e3779b97f4a7c15ull;
        unsigned long long z = x;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        z ^= z >> 31;
        std::swap(h[i], h[size_t(z % (i + 1))]);
    }
    char *f, *buf;
    int* lids;
    CK(hipMalloc(&f, cells * 64));
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&lids, n * 4));
    CK(hipMemcpy(lids, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(f, 1, cells * 64));
    CK(hipMemset(buf, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) -> int {
        std::vector<float> t;
        for (int i = 0; i < 21; ++i)
        {
            launch(hipEvent_t(nullptr), hipEvent_t(nullptr));
            launch(e0, e1);
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        printf("{\"variant\": \"%s\", \"us\": %.2f}\n", name, t[t.size() / 2]);
        fflush(stdout);
        return 0;
    };
    const int grid = 256 * 16;
    run("gs8", [&](hipEvent_t a, hipEvent_t b) {
        hipExtLaunchKernelGGL(k_gs<v2>, dim3(grid), dim3(256), 0, 0, a, b, 0, f, (const int*)lids,
                              (const char*)buf, uint64_t(bytes));
    });
    run("gs16", [&](hipEvent_t a, hipEvent_t b) {
        hipExtLaunchKernelGGL(k_gs<v4>, dim3(grid), dim3(256), 0, 0, a, b, 0, f, (const int*)lids,
                              (const char*)buf, uint64_t(bytes));
    });
    for (uint32_t tile : {8192u, 16384u, 32768u})
    {
        char name[64];
        const unsigned blocks = unsigned((bytes + tile - 1) / tile);
        snprintf(name, sizeof name, "t16_U4_tile%u", tile);
        run(name, [&](hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL((k_tile<v4, 4>), dim3(blocks), dim3(256), 0, 0, a, b, 0, f,
                                  (const int*)lids, (const char*)buf, uint64_t(bytes), tile);
        });
        snprintf(name, sizeof name, "t8_U4_tile%u", tile);
        run(name, [&](hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL((k_tile<v2, 4>), dim3(blocks), dim3(256), 0, 0, a, b, 0, f,
                                  (const int*)lids, (const char*)buf, uint64_t(bytes), tile);
        });
        snprintf(name, sizeof name, "t16_U1_tile%u", tile);
        run(name, [&](hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernelGGL((k_tile<v4, 1>), dim3(blocks), dim3(256), 0, 0, a, b, 0, f,
                                  (const int*)lids, (const char*)buf, uint64_t(bytes), tile);
        });
    }
    return 0;
}
