// sorted_gather.hip — developer micro-benchmark (not product): does visiting an unstructured
// index list in field-address order make config 5's 8-B gathers / scatters cheaper?
// Field: F doubles (10M cells + 5 % outer cells, 84 MB); list: n = 500,000 distinct random lids
// (the pack's send lids, in the pattern's order). Variants, one lane per element:
//   rand        buf[i] = f[lid[i]]                 (what k_copy<seg_u> does: buffer order)
//   sorted_perm buf[pos[k]] = f[slid[k]]           (field order, buffer written at its position)
//   sorted_lin  buf[k] = f[slid[k]]                (field order, buffer linear: an upper bound)
// and the same three for the scatter (f[...] = buf[...]). slid = lids sorted, pos = their buffer
// positions (one int2 {lid, pos} per element). Warm (repeated) and cold (a 1 GiB read sweep
// before every launch, which also evicts the 256 MB MALL). Output: one JSON line per variant,
// the median of 25 launches by events. Build: make -C tools bin/sorted_gather
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                     \
    do                                                                            \
    {                                                                             \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess)                                                     \
        {                                                                         \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

using v4 = unsigned __attribute__((ext_vector_type(4)));

template<bool PACK>
__global__ __launch_bounds__(256) void k_rand(double* f, double* buf, const int* lid, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (PACK) buf[i] = f[lid[i]];
    else f[lid[i]] = buf[i];
}

template<bool PACK, bool LIN>
__global__ __launch_bounds__(256) void k_sorted(double* f, double* buf, const int2* lp, int n)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const int2 e = lp[k];
    const int b = LIN ? k : e.y;
    if (PACK) buf[b] = f[e.x];
    else f[e.x] = buf[b];
}

__global__ __launch_bounds__(256) void k_flush(const v4* p, size_t n, unsigned* sink)
{
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
    {
        const v4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 500000;
    const int F = argc > 2 ? atoi(argv[2]) : 10500000;
    std::mt19937_64 rng(20260715);
    std::vector<int> all(F);
    std::iota(all.begin(), all.end(), 0);
    for (int i = 0; i < n; ++i) std::swap(all[i], all[i + rng() % (F - i)]);  // partial shuffle
    std::vector<int> lid(all.begin(), all.begin() + n);
    std::vector<int2> lp(n);
    for (int i = 0; i < n; ++i) lp[i] = make_int2(lid[i], i);
    std::sort(lp.begin(), lp.end(), [](int2 a, int2 b) { return a.x < b.x; });

    double *f, *buf;
    int* dlid;
    int2* dlp;
    v4* fl;
    unsigned* sink;
    const size_t flush_n = (size_t(1) << 30) / 16;
    CK(hipMalloc(&f, size_t(F) * 8));
    CK(hipMalloc(&buf, size_t(n) * 8));
    CK(hipMalloc(&dlid, size_t(n) * 4));
    CK(hipMalloc(&dlp, size_t(n) * 8));
    CK(hipMalloc(&fl, flush_n * 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(f, 1, size_t(F) * 8));
    CK(hipMemset(buf, 2, size_t(n) * 8));
    CK(hipMemset(fl, 3, flush_n * 16));
    CK(hipMemcpy(dlid, lid.data(), size_t(n) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlp, lp.data(), size_t(n) * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = (n + 255) / 256;

    auto run = [&](const char* name, auto launch) {
        for (int cold = 0; cold < 2; ++cold)
        {
            std::vector<float> t;
            for (int r = 0; r < 30; ++r)
            {
                if (cold) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, fl, flush_n, sink);
                else launch();
                CK(hipEventRecord(e0, 0));
                launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 5) t.push_back(ms * 1e3f);
            }
            std::sort(t.begin(), t.end());
            const double us = t[t.size() / 2];
            printf("{\"variant\": \"%s\", \"cold\": %d, \"n\": %d, \"cells\": %d, \"us\": %.2f, "
                   "\"GBps_values\": %.1f}\n",
                   name, cold, n, F, us, 2.0 * n * 8 / us * 1e-3);
        }
    };
    run("pack_rand", [&] { hipLaunchKernelGGL(k_rand<true>, dim3(grid), dim3(256), 0, 0, f, buf, dlid, n); });
    run("pack_sorted_perm", [&] { hipLaunchKernelGGL((k_sorted<true, false>), dim3(grid), dim3(256), 0, 0, f, buf, dlp, n); });
    run("pack_sorted_lin", [&] { hipLaunchKernelGGL((k_sorted<true, true>), dim3(grid), dim3(256), 0, 0, f, buf, dlp, n); });
    run("unpack_rand", [&] { hipLaunchKernelGGL(k_rand<false>, dim3(grid), dim3(256), 0, 0, f, buf, dlid, n); });
    run("unpack_sorted_perm", [&] { hipLaunchKernelGGL((k_sorted<false, false>), dim3(grid), dim3(256), 0, 0, f, buf, dlp, n); });
    run("unpack_sorted_lin", [&] { hipLaunchKernelGGL((k_sorted<false, true>), dim3(grid), dim3(256), 0, 0, f, buf, dlp, n); });
    CK(hipDeviceSynchronize());
    return 0;
}
