// req_ceiling.hip — developer micro-benchmark (not product): how many L2 -> fabric requests per
// second the chip retires for each access shape the halo kernels issue, so that DESIGN §4.3's
// request-bound model rests on measured ceilings instead of one copy figure. Request counts are
// known by construction (a 128-B line read = 1 read request, a 64-B aligned write = 1 write
// request, a 16-B write into a fresh 64-B block = 1 partial write request); each kernel is timed
// with events, median of `reps`, warm (its footprint stays in the 256 MiB Infinity Cache: the
// regime of the bench's back-to-back steps) and cold (after a 1 GiB read-only sweep).
//   read_stream   16 B/lane, lane-linear over S bytes                  S/128 reads
//   write_stream  16 B/lane, lane-linear                               S/64 writes
//   copy_stream   read + write lane-linear                             S/128 + S/64
//   read_lines    one 16-B load per 128-B line, lines `stride` apart   n reads
//   write_pieces  one 16-B store per 64-B block, blocks `stride` apart n partial writes
// Build: hipcc -O3 --offload-arch=gfx950 tools/req_ceiling.hip -o tools/bin/req_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

__global__ __launch_bounds__(256) void k_read(const v4* p, size_t n, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) acc ^= p[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

__global__ __launch_bounds__(256) void k_write(v4* p, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        p[i] = v4{unsigned(i), 1, 2, 3};
}

__global__ __launch_bounds__(256) void k_copy(const v4* a, v4* b, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) b[i] = a[i];
}

// one 16-B load per item, items `stride` bytes apart
__global__ __launch_bounds__(256) void k_read_lines(const char* p, size_t n, size_t stride, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        acc ^= *(const v4*)(p + i * stride);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

__global__ __launch_bounds__(256) void k_write_pieces(char* p, size_t n, size_t stride)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        *(v4*)(p + i * stride) = v4{unsigned(i), 1, 2, 3};
}

// config 5's shapes in their simplest form (round 5): one int32 index per lane (coalesced), one
// 8-B access at field + index * 8 (a random line of an 84 MB field), with or without the
// lane-linear buffer side of a gather / scatter
__global__ __launch_bounds__(256) void k_read_random(const double* f, const int* idx, size_t n,
                                                     unsigned* sink)
{
    double acc = 0;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        acc += f[idx[i]];
    if (acc == 1.2345) sink[0] = 1;
}

__global__ __launch_bounds__(256) void k_write_random(double* f, const int* idx, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        f[idx[i]] = double(i);
}

__global__ __launch_bounds__(256) void k_gather_random(const double* f, const int* idx,
                                                       double* buf, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        buf[i] = f[idx[i]];
}

__global__ __launch_bounds__(256) void k_scatter_random(double* f, const int* idx,
                                                        const double* buf, size_t n)
{
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
        f[idx[i]] = buf[i];
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 11;
    const size_t S = size_t(64) << 20;      // streaming footprint per buffer (64 MiB)
    const size_t big = size_t(1100) << 20;  // scattered footprint (the 512^3 field's size)
    const size_t flush_bytes = size_t(1) << 30;
    char *a, *b, *f, *fl;
    unsigned* sink;
    CK(hipMalloc(&a, S));
    CK(hipMalloc(&b, S));
    CK(hipMalloc(&f, big));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, S));
    CK(hipMemset(b, 2, S));
    CK(hipMemset(f, 3, big));
    CK(hipMemset(fl, 4, flush_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = 256 * 16;
    auto flush = [&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const v4*)fl, flush_bytes / 16, sink); };
    auto timed = [&](const std::function<void()>& f, bool cold) {
        std::vector<float> t;
        for (int i = 0; i < reps; ++i)
        {
            if (cold) flush();
            else f();
            CK(hipEventRecord(e0));
            f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return double(t[t.size() / 2]);
    };
    auto report = [&](const char* name, double reads, double writes, double bytes, const std::function<void()>& f) {
        for (int cold = 0; cold < 2; ++cold)
        {
            const double us = timed(f, cold);
            printf("{\"shape\": \"%s\", \"cold\": %d, \"us\": %.2f, \"read_req\": %.0f, \"write_req\": %.0f, "
                   "\"G_req_per_s\": %.1f, \"TBps\": %.2f}\n",
                   name, cold, us, reads, writes, (reads + writes) / us / 1e3, bytes / us / 1e6);
            fflush(stdout);
        }
    };
    report("read_stream_64MiB", double(S) / 128, 0, double(S),
           [&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const v4*)a, S / 16, sink); });
    report("write_stream_64MiB", 0, double(S) / 64, double(S),
           [&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (v4*)b, S / 16); });
    report("copy_stream_64MiB", double(S) / 128, double(S) / 64, 2.0 * double(S),
           [&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const v4*)a, (v4*)b, S / 16); });
    for (size_t stride : {size_t(128), size_t(4096), size_t(4128), size_t(4224)})
    {
        const size_t n = std::min<size_t>(size_t(262144) * 2, (big - 64) / stride);
        char name[64];
        snprintf(name, sizeof name, "read_lines_stride%zu", stride);
        report(name, double(n), 0, double(n) * 16,
               [&] { hipLaunchKernelGGL(k_read_lines, dim3(grid), dim3(256), 0, 0, f, n, stride, sink); });
        snprintf(name, sizeof name, "write_pieces_stride%zu", stride);
        report(name, 0, double(n), double(n) * 16,
               [&] { hipLaunchKernelGGL(k_write_pieces, dim3(grid), dim3(256), 0, 0, f, n, stride); });
    }
    {
        // config 5 (round 5): 500k distinct random cells of a 10.5M-cell fp64 field (84 MB)
        const size_t cells = 10500000, n = 500000;
        std::vector<int> h(cells);
        for (size_t i = 0; i < cells; ++i) h[i] = int(i);
        unsigned long long x = 20260715ull;
        for (size_t i = cells - 1; i > 0; --i)  // Fisher-Yates with splitmix64
        {
            x += 0x9e3779b97f4a7c15ull;
            unsigned long long z = x;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            z ^= z >> 31;
            std::swap(h[i], h[size_t(z % (i + 1))]);
        }
        int* idx;
        double* buf;
        CK(hipMalloc(&idx, 2 * n * sizeof(int)));  // [0, n): gather cells, [n, 2n): scatter cells
        CK(hipMalloc(&buf, n * sizeof(double)));
        CK(hipMemcpy(idx, h.data(), 2 * n * sizeof(int), hipMemcpyHostToDevice));
        CK(hipMemset(buf, 0, n * sizeof(double)));
        const double* fd = (const double*)f;
        report("read_random_8B_of_84MB", double(n), 0, double(n) * 8,
               [&] { hipLaunchKernelGGL(k_read_random, dim3(grid), dim3(256), 0, 0, fd, idx, n, sink); });
        report("write_random_8B_of_84MB", 0, double(n), double(n) * 8,
               [&] { hipLaunchKernelGGL(k_write_random, dim3(grid), dim3(256), 0, 0, (double*)f, idx, n); });
        report("gather_random_8B_of_84MB", double(n), double(n) / 8, double(n) * 16,
               [&] { hipLaunchKernelGGL(k_gather_random, dim3(grid), dim3(256), 0, 0, fd, idx, buf, n); });
        report("scatter_random_8B_of_84MB", double(n) / 16, double(n), double(n) * 16,
               [&] { hipLaunchKernelGGL(k_scatter_random, dim3(grid), dim3(256), 0, 0, (double*)f, idx, buf, n); });
        report("gather_then_scatter_random_8B_of_84MB", double(n) * 17 / 16, double(n) * 9 / 8,
               double(n) * 32, [&] {
                   hipLaunchKernelGGL(k_gather_random, dim3(grid), dim3(256), 0, 0, fd, idx, buf, n);
                   hipLaunchKernelGGL(k_scatter_random, dim3(grid), dim3(256), 0, 0, (double*)f, idx + n, buf, n);
               });
        CK(hipFree(idx));
        CK(hipFree(buf));
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(f));
    CK(hipFree(fl));
    CK(hipFree(sink));
    return 0;
}
