// granule_bench.hip — developer micro-benchmark (not product): what a scattered partial write
// costs once it leaves the caches. 262,144 rows at the 512^3 H=2 field's row pitch (4,128 B);
// per row one write of W bytes at byte offset O of the row (the x-face halo pair of row r and
// r+1 is 32 B at offset 4,112; composed with the adjacent interior cells it is 64 B at 4,096).
// Each variant is timed as  flush; [write; flush]  against  flush; [flush]  (events around the
// brackets), so the write-back of the lines it leaves dirty — done by the next flush, as an
// application's next sweep would — is charged to it. The flush is a 1 GiB read-only reduction.
// Output: one JSON line per variant. Build: hipcc -O3 --offload-arch=gfx950 tools/granule_bench.hip
//   -o tools/bin/granule_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do                                                                               \
    {                                                                                \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess)                                                        \
        {                                                                            \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);    \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

using v4 = unsigned __attribute__((ext_vector_type(4)));
constexpr unsigned ROWS = 512u * 512u;

// one lane per row; W in {16, 32, 64, 128}: W/16 vector stores of 16 B (a lane's stores to one
// row are consecutive, so the L2 merges them into the same line)
template<int W, bool READ>
__global__ __launch_bounds__(256) void k_write(char* base, unsigned pitch, unsigned off)
{
    const unsigned r = blockIdx.x * 256 + threadIdx.x;
    if (r >= ROWS) return;
    char* p = base + size_t(r) * pitch + off;
    v4 v[W / 16];
#pragma unroll
    for (int i = 0; i < W / 16; ++i)
        v[i] = READ ? *(const v4*)(p + 16 * i) + v4{1, 1, 1, 1} : v4{r, r + 1, r + 2, r + 3};
#pragma unroll
    for (int i = 0; i < W / 16; ++i) *(v4*)(p + 16 * i) = v[i];
}

// two lanes per row, each one 16-B piece: the two halves of a halo pair written by different
// lanes (as the unpack's +x and -x segments do), lane pairs adjacent
__global__ __launch_bounds__(256) void k_write_pair(char* base, unsigned pitch, unsigned off)
{
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const unsigned r = t >> 1;
    if (r >= ROWS) return;
    char* p = base + size_t(r) * pitch + off + 16 * (t & 1);
    *(v4*)p = v4{t, t + 1, t + 2, t + 3};
}

__global__ __launch_bounds__(256) void k_flush(const v4* p, size_t n, unsigned* sink)
{
    unsigned acc = 0;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256)
    {
        const v4 x = p[i];
        acc += x.x ^ x.y ^ x.z ^ x.w;
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;  // practically never: keeps the loads live
}

int main(int argc, char** argv)
{
    const unsigned pitch = argc > 1 ? unsigned(atoi(argv[1])) : 4128u;
    const int reps = argc > 2 ? atoi(argv[2]) : 9;
    const size_t region = size_t(ROWS + 4) * pitch;
    const size_t flush_bytes = size_t(1) << 30;
    char *base, *fl;
    unsigned* sink;
    CK(hipMalloc(&base, region));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&sink, 4096 * sizeof(unsigned)));
    CK(hipMemset(base, 0, region));
    CK(hipMemset(fl, 1, flush_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto flush = [&] { hipLaunchKernelGGL(k_flush, dim3(2048), dim3(256), 0, 0, (const v4*)fl, flush_bytes / 16, sink); };
    const unsigned g1 = (ROWS + 255) / 256, g2 = (2 * ROWS + 255) / 256;
    struct variant
    {
        const char* name;
        int w;
        unsigned off;
        int kind;  // 0 one lane per row, 1 two lanes per row (16 B each), 2 read-modify-write
    };
    const std::vector<variant> vs = {
        {"halo_pair_2x16_at_4112", 32, 4112, 1}, {"pair_32_at_4112", 32, 4112, 0},
        {"sector_32_at_4096", 32, 4096, 0},      {"sector_32_at_4128", 32, 4128, 0},
        {"span_64_at_4096", 64, 4096, 0},        {"one_16_at_4112", 16, 4112, 0},
        {"line_128_at_4032", 128, 4032, 0},      {"rmw_64_at_4096", 64, 4096, 2}};
    auto launch = [&](const variant& v) {
        if (v.kind == 1) hipLaunchKernelGGL(k_write_pair, dim3(g2), dim3(256), 0, 0, base, pitch, v.off);
        else if (v.kind == 2) hipLaunchKernelGGL((k_write<64, true>), dim3(g1), dim3(256), 0, 0, base, pitch, v.off);
        else if (v.w == 16) hipLaunchKernelGGL((k_write<16, false>), dim3(g1), dim3(256), 0, 0, base, pitch, v.off);
        else if (v.w == 32) hipLaunchKernelGGL((k_write<32, false>), dim3(g1), dim3(256), 0, 0, base, pitch, v.off);
        else if (v.w == 64) hipLaunchKernelGGL((k_write<64, false>), dim3(g1), dim3(256), 0, 0, base, pitch, v.off);
        else hipLaunchKernelGGL((k_write<128, false>), dim3(g1), dim3(256), 0, 0, base, pitch, v.off);
    };
    auto timed = [&](auto body) {
        std::vector<float> t;
        for (int i = 0; i < reps; ++i)
        {
            flush();
            CK(hipEventRecord(e0));
            body();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    const float t_flush = timed([&] { flush(); });
    for (const auto& v : vs)
    {
        const float t_wf = timed([&] { launch(v); flush(); });
        const float t_w = timed([&] { launch(v); });                    // cold write alone
        const float t_ww = timed([&] { launch(v); launch(v); });        // + a warm repeat
        printf("{\"pitch\": %u, \"variant\": \"%s\", \"bytes_per_row\": %d, \"offset\": %u, "
               "\"write_cold_us\": %.2f, \"write_warm_us\": %.2f, \"write_plus_writeback_us\": %.2f, "
               "\"flush_us\": %.2f}\n",
               pitch, v.name, v.w, v.off, t_w, t_ww - t_w, t_wf - t_flush, t_flush);
        fflush(stdout);
    }
    CK(hipFree(base));
    CK(hipFree(fl));
    CK(hipFree(sink));
    return 0;
}
