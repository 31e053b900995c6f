// pack_floor.hip — developer measurement (not product): the read floor of the 512^3 H=2 pack,
// and the write floor of the unpack (ghx_probe_unpack_floor: the halo rows' bytes written once,
// 16-B pieces where aligned, plus the buffer stream read).
// Builds, on the host, the exact set of 128-B field lines the pack must read (the 26 send boxes
// of one periodic 516^3 fp64 domain: every row's byte range -> the lines it touches, deduped),
// split into the x-face class (lines touched by rows of <= H cells: x faces, x edges, corners)
// and the long-row class (the rest), and times a kernel that does nothing but load ONE 16-B
// vector from each listed line (lane-linear over the list, 4 loads in flight per lane, no index
// math, no writes). That is the least the memory system can take to deliver the pack's reads in
// that class order, whatever a pack kernel does; the pack's own time is measured beside it by
// bench.py / tools/microbench.py on the same box.
//   xface    the x-face lines alone
//   long     the long-row lines alone
//   both     x-face lines first, then long-row lines, one launch (the pack's dispatch order)
//   both_rw  as both, plus the pack's buffer writes (25.4 MB, 16 B per lane, streamed by the
//            same grid after its loads)
// Warm (footprint resident in the 256 MiB Infinity Cache, as in the bench's back-to-back steps)
// and cold (right after a 1 GiB read-only sweep: nothing dirty to write back). Each launch timed
// by its own begin/end events (hipExtLaunchKernelGGL: the interval a rocprofv3 kernel trace
// reports, as bench.py's pack_kernel_us), median of `reps`.
// Built by tools/Makefile (from __graft_entry__.build()) as tools/bin/pack_floor (one JSON line
// per measurement; `pack_floor reps N H v` runs unpack variant v alone, warm, for the PMC passes
// of tools/pmc_floor.sh) and tools/lib/libpackfloor.so (ghx_probe_pack_floor, called by bench.py).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                   \
    do                          \
    {                           \
        if ((x) != hipSuccess)  \
        {                       \
            rc = __LINE__;      \
            goto done;          \
        }                       \
    } while (0)

using v4 = unsigned __attribute__((ext_vector_type(4)));
constexpr int kU = 4;

// lines[0, n): one 16-B load per line; optionally the grid then streams `wbytes` of writes.
// DEP: every written vector carries a loaded value, so a lane's writes wait for its loads, as a
// pack's buffer writes wait for the field reads they copy (the plain form's writes are
// independent of its reads and overlap them freely).
template<bool DEP = false>
__global__ __launch_bounds__(256) void k_lines(const uint32_t* __restrict__ lines, uint32_t n,
                                               const char* __restrict__ field, v4* __restrict__ buf,
                                               uint64_t wvec, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t base = blockIdx.x * 256u + threadIdx.x; base < n; base += kU * stride)
    {
        uint32_t l[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) l[u] = base + u * stride < n ? lines[base + u * stride] : 0xffffffffu;
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (l[u] != 0xffffffffu) acc ^= *(const v4*)(field + uint64_t(l[u]) * 128);
    }
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < wvec; i += uint64_t(stride))
        buf[i] = v4{unsigned(i), DEP ? acc.x : 1u, 2, 3};
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

// The unpack's mirror: the grid streams `rvec` vectors of the buffer in, then writes each listed
// halo piece (bit 31: 16 B, else 8 B; bits 0-30: byte address / 8) once.
__global__ __launch_bounds__(256) void k_pieces(const uint32_t* __restrict__ pieces, uint32_t n,
                                                char* __restrict__ field, const v4* __restrict__ buf,
                                                uint64_t rvec, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    const uint32_t stride = gridDim.x * 256u;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < rvec; i += uint64_t(stride)) acc ^= buf[i];
    for (uint32_t base = blockIdx.x * 256u + threadIdx.x; base < n; base += kU * stride)
    {
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            if (base + u * stride >= n) break;
            const uint32_t q = pieces[base + u * stride];
            char* a = field + uint64_t(q & 0x7fffffffu) * 8;
            if (q >> 31) *(v4*)a = v4{q, acc.x, 2, 3};
            else *(unsigned __attribute__((ext_vector_type(2)))*)a = {q, acc.y};
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

// The unpack's mirror with the buffer reads interleaved with the writes, as the unpack kernel
// issues them: per lane and step one list entry, the 16-B buffer vector of that position (the
// buffer streamed lane-linearly) and the piece's store, kU steps in flight per lane. A piece of
// 8 B takes a 16-B buffer slot (its second half unused): the stream is at most a few % longer
// than the buffer.
__global__ __launch_bounds__(256) void k_pieces_il(const uint32_t* __restrict__ pieces, uint32_t n,
                                                   char* __restrict__ field,
                                                   const v4* __restrict__ buf, unsigned* sink)
{
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t base = blockIdx.x * 256u + threadIdx.x; base < n; base += kU * stride)
    {
        uint32_t q[kU];
        v4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) q[u] = base + u * stride < n ? pieces[base + u * stride] : 0xffffffffu;
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (q[u] != 0xffffffffu) v[u] = buf[base + u * stride];
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            if (q[u] == 0xffffffffu) continue;
            char* a = field + uint64_t(q[u] & 0x7fffffffu) * 8;
            if (q[u] >> 31) *(v4*)a = v[u];
            else *(unsigned __attribute__((ext_vector_type(2)))*)a = {v[u].x, v[u].y};
        }
    }
    if (n == 0xffffffffu) sink[0] = 0;
}

// The fused self exchange's mirror: one grid loads one vector per pack line, streams the buffer
// writes and writes every halo piece (what k_self must do, with no index arithmetic).
__global__ __launch_bounds__(256) void k_fused(const uint32_t* __restrict__ lines, uint32_t nl,
                                               const uint32_t* __restrict__ pieces, uint32_t np,
                                               char* __restrict__ field, v4* __restrict__ buf,
                                               uint64_t wvec, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nl; i += stride)
        acc ^= *(const v4*)(field + uint64_t(lines[i]) * 128);
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < wvec; i += uint64_t(stride))
        buf[i] = v4{unsigned(i), acc.x, 2, 3};
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < np; i += stride)
    {
        const uint32_t q = pieces[i];
        char* a = field + uint64_t(q & 0x7fffffffu) * 8;
        if (q >> 31) *(v4*)a = v4{q, acc.y, 2, 3};
        else *(unsigned __attribute__((ext_vector_type(2)))*)a = {q, acc.z};
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

__global__ __launch_bounds__(256) void k_sweep(const v4* p, size_t n, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) acc ^= p[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

// The 26 send boxes of one periodic (N+2H)^3 fp64 domain: the 128-B lines their rows touch,
// x-face class (rows of <= H cells) first; useful = the pack's algorithmic read bytes.
static void line_sets(int N, int H, std::vector<uint32_t>& xf, std::vector<uint32_t>& lg, uint64_t& useful)
{
    const int E = N + 2 * H;
    const uint64_t pitch = uint64_t(E) * 8, plane = pitch * E;
    std::vector<uint8_t> cls(size_t(plane * E / 128 + 1), 0);  // 1 x-face, 2 long
    useful = 0;
    const int lo[3] = {H, H, N};  // dir -1, 0, +1: first interior coordinate of the box
    const int hi[3] = {2 * H - 1, N + H - 1, N + H - 1};
    for (int dz = 0; dz < 3; ++dz)
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx)
            {
                if (dx == 1 && dy == 1 && dz == 1) continue;
                const int x0 = lo[dx], x1 = hi[dx];
                const bool shortrow = x1 - x0 + 1 <= H;
                for (int z = lo[dz]; z <= hi[dz]; ++z)
                    for (int y = lo[dy]; y <= hi[dy]; ++y)
                    {
                        const uint64_t b = uint64_t(z) * plane + uint64_t(y) * pitch + uint64_t(x0) * 8;
                        const uint64_t e = b + uint64_t(x1 - x0 + 1) * 8;
                        useful += e - b;
                        for (uint64_t l = b / 128; l <= (e - 1) / 128; ++l)
                            if (shortrow) cls[l] = 1;
                            else if (!cls[l]) cls[l] = 2;
                    }
            }
    for (size_t l = 0; l < cls.size(); ++l)
        if (cls[l] == 1) xf.push_back(uint32_t(l));
        else if (cls[l] == 2) lg.push_back(uint32_t(l));
}

// The 26 receive boxes (halos) of the same domain as write pieces: each row's byte range in
// 16-B pieces where 16-B aligned, 8-B pieces at the edges; x-face class first.
static void piece_sets(int N, int H, std::vector<uint32_t>& xf, std::vector<uint32_t>& lg, uint64_t& useful)
{
    const int E = N + 2 * H;
    const uint64_t pitch = uint64_t(E) * 8, plane = pitch * E;
    useful = 0;
    const int lo[3] = {0, H, N + H};  // dir -1, 0, +1: first halo-box coordinate
    const int hi[3] = {H - 1, N + H - 1, N + 2 * H - 1};
    for (int dz = 0; dz < 3; ++dz)
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx)
            {
                if (dx == 1 && dy == 1 && dz == 1) continue;
                const int x0 = lo[dx], x1 = hi[dx];
                auto& out = x1 - x0 + 1 <= H ? xf : lg;
                for (int z = lo[dz]; z <= hi[dz]; ++z)
                    for (int y = lo[dy]; y <= hi[dy]; ++y)
                    {
                        uint64_t b = uint64_t(z) * plane + uint64_t(y) * pitch + uint64_t(x0) * 8;
                        const uint64_t e = b + uint64_t(x1 - x0 + 1) * 8;
                        useful += e - b;
                        while (b < e)
                        {
                            const bool w16 = b % 16 == 0 && e - b >= 16;
                            out.push_back(uint32_t(b / 8) | (w16 ? 0x80000000u : 0u));
                            b += w16 ? 16 : 8;
                        }
                    }
            }
    std::sort(xf.begin(), xf.end(), [](uint32_t a, uint32_t b) { return (a & 0x7fffffffu) < (b & 0x7fffffffu); });
    std::sort(lg.begin(), lg.end(), [](uint32_t a, uint32_t b) { return (a & 0x7fffffffu) < (b & 0x7fffffffu); });
}

// PMC runs (main's 4th argument): only this unpack variant, warm only (-1: all)
static int s_only_variant = -1;

// out_us[10]: {xface, long, both, both + buffer reads streamed first, both + buffer reads
// interleaved (k_pieces_il)} x {warm, cold} of the unpack's halo writes; counts[3]: x-face pieces,
// long-row pieces, useful bytes. Returns 0, or the failing source line.
extern "C" int ghx_probe_unpack_floor(int N, int H, int reps, double* out_us, int64_t* counts)
{
    int rc = 0;
    std::vector<uint32_t> xf, lg;
    uint64_t useful = 0;
    piece_sets(N, H, xf, lg, useful);
    std::vector<uint32_t> both(xf);
    both.insert(both.end(), lg.begin(), lg.end());
    const int E = N + 2 * H;
    const size_t fbytes = size_t(E) * E * E * 8, flush_bytes = size_t(1) << 30;
    char *field = nullptr, *fl = nullptr;
    v4* buf = nullptr;
    unsigned* sink = nullptr;
    uint32_t *d_xf = nullptr, *d_lg = nullptr, *d_both = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int grid = 256 * 8;
    counts[0] = int64_t(xf.size());
    counts[1] = int64_t(lg.size());
    counts[2] = int64_t(useful);
    if (fbytes / 8 >= (size_t(1) << 31)) return __LINE__;  // piece addresses are 31-bit / 8
    CK(hipMalloc(&field, fbytes));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&buf, both.size() * 16 + 64));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&d_xf, xf.size() * 4 + 4));
    CK(hipMalloc(&d_lg, lg.size() * 4 + 4));
    CK(hipMalloc(&d_both, both.size() * 4 + 4));
    CK(hipMemcpy(d_xf, xf.data(), xf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lg, lg.data(), lg.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_both, both.data(), both.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(field, 1, fbytes));
    CK(hipMemset(buf, 3, both.size() * 16 + 64));
    CK(hipMemset(fl, 2, flush_bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    {
        const uint32_t* lists[5] = {d_xf, d_lg, d_both, d_both, d_both};
        const size_t ns[5] = {xf.size(), lg.size(), both.size(), both.size(), both.size()};
        const uint64_t rv[5] = {0, 0, 0, useful / 16, 0};
        for (int j = 0; j < 5; ++j)
            for (int cold = 0; cold < 2; ++cold)
            {
                if (s_only_variant >= 0 && (j != s_only_variant || cold))
                {
                    out_us[2 * j + cold] = 0;
                    continue;
                }
                std::vector<float> t;
                for (int i = 0; i < reps; ++i)
                {
                    if (cold)
                        hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(256), 0, 0, (const v4*)fl,
                                           flush_bytes / 16, sink);
                    else if (j == 4)
                        hipLaunchKernelGGL(k_pieces_il, dim3(grid), dim3(256), 0, 0, lists[j],
                                           uint32_t(ns[j]), field, (const v4*)buf, sink);
                    else
                        hipLaunchKernelGGL(k_pieces, dim3(grid), dim3(256), 0, 0, lists[j], uint32_t(ns[j]),
                                           field, (const v4*)buf, rv[j], sink);
                    if (j == 4)
                        hipExtLaunchKernelGGL(k_pieces_il, dim3(grid), dim3(256), 0, 0, e0, e1, 0,
                                              lists[j], uint32_t(ns[j]), field, (const v4*)buf, sink);
                    else
                        hipExtLaunchKernelGGL(k_pieces, dim3(grid), dim3(256), 0, 0, e0, e1, 0, lists[j],
                                              uint32_t(ns[j]), field, (const v4*)buf, rv[j], sink);
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    t.push_back(ms * 1e3f);
                }
                std::sort(t.begin(), t.end());
                out_us[2 * j + cold] = t[t.size() / 2];
            }
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void* p : {(void*)field, (void*)fl, (void*)buf, (void*)sink, (void*)d_xf, (void*)d_lg, (void*)d_both})
        if (p) (void)hipFree(p);
    return rc;
}

// out_us[10]: {xface, long, both, both_rw, both_rw with dependent writes} x {warm, cold}
// (microseconds, kernel-own events);
// counts[3]: x-face lines, long-row lines, useful bytes. Returns 0, or the failing source line.
extern "C" int ghx_probe_pack_floor(int N, int H, int reps, double* out_us, int64_t* counts)
{
    int rc = 0;
    std::vector<uint32_t> xf, lg;
    uint64_t useful = 0;
    line_sets(N, H, xf, lg, useful);
    std::vector<uint32_t> both(xf);
    both.insert(both.end(), lg.begin(), lg.end());
    const int E = N + 2 * H;
    const size_t fbytes = size_t(E) * E * E * 8, flush_bytes = size_t(1) << 30;
    char *field = nullptr, *fl = nullptr;
    v4* buf = nullptr;
    unsigned* sink = nullptr;
    uint32_t *d_xf = nullptr, *d_lg = nullptr, *d_both = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int grid = 256 * 8;
    counts[0] = int64_t(xf.size());
    counts[1] = int64_t(lg.size());
    counts[2] = int64_t(useful);
    CK(hipMalloc(&field, fbytes));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&buf, useful + 64));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&d_xf, xf.size() * 4 + 4));
    CK(hipMalloc(&d_lg, lg.size() * 4 + 4));
    CK(hipMalloc(&d_both, both.size() * 4 + 4));
    CK(hipMemcpy(d_xf, xf.data(), xf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lg, lg.data(), lg.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_both, both.data(), both.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(field, 1, fbytes));
    CK(hipMemset(fl, 2, flush_bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    {
        const uint32_t* lists[5] = {d_xf, d_lg, d_both, d_both, d_both};
        const size_t ns[5] = {xf.size(), lg.size(), both.size(), both.size(), both.size()};
        const uint64_t wv[5] = {0, 0, 0, useful / 16, useful / 16};
        for (int j = 0; j < 5; ++j)
            for (int cold = 0; cold < 2; ++cold)
            {
                std::vector<float> t;
                for (int i = 0; i < reps; ++i)
                {
                    if (cold)
                        hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(256), 0, 0, (const v4*)fl,
                                           flush_bytes / 16, sink);
                    else if (j == 4)
                        hipLaunchKernelGGL(k_lines<true>, dim3(grid), dim3(256), 0, 0, lists[j],
                                           uint32_t(ns[j]), (const char*)field, buf, wv[j], sink);
                    else
                        hipLaunchKernelGGL(k_lines<>, dim3(grid), dim3(256), 0, 0, lists[j], uint32_t(ns[j]),
                                           (const char*)field, buf, wv[j], sink);
                    if (j == 4)
                        hipExtLaunchKernelGGL(k_lines<true>, dim3(grid), dim3(256), 0, 0, e0, e1, 0,
                                              lists[j], uint32_t(ns[j]), (const char*)field, buf,
                                              wv[j], sink);
                    else
                        hipExtLaunchKernelGGL(k_lines<>, dim3(grid), dim3(256), 0, 0, e0, e1, 0, lists[j],
                                              uint32_t(ns[j]), (const char*)field, buf, wv[j], sink);
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    t.push_back(ms * 1e3f);
                }
                std::sort(t.begin(), t.end());
                out_us[2 * j + cold] = t[t.size() / 2];
            }
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void* p : {(void*)field, (void*)fl, (void*)buf, (void*)sink, (void*)d_xf, (void*)d_lg, (void*)d_both})
        if (p) (void)hipFree(p);
    return rc;
}

// out_us[2]: {warm, cold} of the fused mirror (pack lines read + buffer written + halo pieces
// written, one launch). Returns 0, or the failing source line.
extern "C" int ghx_probe_fused_floor(int N, int H, int reps, double* out_us)
{
    int rc = 0;
    std::vector<uint32_t> xf, lg, pxf, plg;
    uint64_t useful = 0, useful2 = 0;
    line_sets(N, H, xf, lg, useful);
    piece_sets(N, H, pxf, plg, useful2);
    std::vector<uint32_t> lines(xf), pieces(pxf);
    lines.insert(lines.end(), lg.begin(), lg.end());
    pieces.insert(pieces.end(), plg.begin(), plg.end());
    const int E = N + 2 * H;
    const size_t fbytes = size_t(E) * E * E * 8, flush_bytes = size_t(1) << 30;
    char *field = nullptr, *fl = nullptr;
    v4* buf = nullptr;
    unsigned* sink = nullptr;
    uint32_t *d_l = nullptr, *d_p = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int grid = 256 * 8;
    if (fbytes / 8 >= (size_t(1) << 31)) return __LINE__;
    CK(hipMalloc(&field, fbytes));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&buf, useful + 64));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&d_l, lines.size() * 4 + 4));
    CK(hipMalloc(&d_p, pieces.size() * 4 + 4));
    CK(hipMemcpy(d_l, lines.data(), lines.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_p, pieces.data(), pieces.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(field, 1, fbytes));
    CK(hipMemset(fl, 2, flush_bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int cold = 0; cold < 2; ++cold)
    {
        std::vector<float> t;
        for (int i = 0; i < reps; ++i)
        {
            if (cold)
                hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(256), 0, 0, (const v4*)fl, flush_bytes / 16, sink);
            else
                hipLaunchKernelGGL(k_fused, dim3(grid), dim3(256), 0, 0, d_l, uint32_t(lines.size()), d_p,
                                   uint32_t(pieces.size()), field, buf, useful / 16, sink);
            hipExtLaunchKernelGGL(k_fused, dim3(grid), dim3(256), 0, 0, e0, e1, 0, d_l, uint32_t(lines.size()),
                                  d_p, uint32_t(pieces.size()), field, buf, useful / 16, sink);
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        out_us[cold] = t[t.size() / 2];
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void* p : {(void*)field, (void*)fl, (void*)buf, (void*)sink, (void*)d_l, (void*)d_p})
        if (p) (void)hipFree(p);
    return rc;
}


// Config 5's index-list floor (round 5): the simplest gather and scatter of the SAME lid lists
// the product runs (levels-first rows of `levels` fp64 values): one (lid, level) value per lane,
// buffer side lane-linear, no plan, no run detection, no tiles. What the memory system takes for
// those random rows; bench.py sets it beside the product's fused launches (floor_over_kernel).
__global__ __launch_bounds__(256) void k_igather(const double* __restrict__ f, const int* __restrict__ lids,
                                                 double* __restrict__ buf, uint64_t n, int L)
{
    for (uint64_t k = uint64_t(blockIdx.x) * 256 + threadIdx.x; k < n * uint64_t(L);
         k += uint64_t(gridDim.x) * 256)
        buf[k] = f[uint64_t(lids[k / L]) * L + k % L];
}

__global__ __launch_bounds__(256) void k_iscatter(double* __restrict__ f, const int* __restrict__ lids,
                                                  const double* __restrict__ buf, uint64_t n, int L)
{
    for (uint64_t k = uint64_t(blockIdx.x) * 256 + threadIdx.x; k < n * uint64_t(L);
         k += uint64_t(gridDim.x) * 256)
        f[uint64_t(lids[k / L]) * L + k % L] = buf[k];
}

// out_us[4]: {gather, scatter} x {warm, cold} (kernel-own events, median of reps).
extern "C" int ghx_probe_index_floor(int64_t cells, int levels, const int32_t* send_lids,
                                     int64_t n_send, const int32_t* recv_lids, int64_t n_recv,
                                     int reps, double* out_us)
{
    int rc = 0;
    const size_t flush_bytes = size_t(1) << 30;
    double *field = nullptr, *sbuf = nullptr, *rbuf = nullptr;
    int *d_s = nullptr, *d_r = nullptr;
    char* fl = nullptr;
    unsigned* sink = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int grid = 256 * 16;
    const int L = levels;
    CK(hipMalloc(&field, size_t(cells) * L * 8));
    CK(hipMalloc(&sbuf, size_t(n_send) * L * 8 + 8));
    CK(hipMalloc(&rbuf, size_t(n_recv) * L * 8 + 8));
    CK(hipMalloc(&d_s, size_t(n_send) * 4 + 4));
    CK(hipMalloc(&d_r, size_t(n_recv) * 4 + 4));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemcpy(d_s, send_lids, size_t(n_send) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_r, recv_lids, size_t(n_recv) * 4, hipMemcpyHostToDevice));
    CK(hipMemset(field, 1, size_t(cells) * L * 8));
    CK(hipMemset(rbuf, 2, size_t(n_recv) * L * 8 + 8));
    CK(hipMemset(fl, 3, flush_bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int j = 0; j < 2; ++j)
        for (int cold = 0; cold < 2; ++cold)
        {
            std::vector<float> t;
            auto launch = [&](hipEvent_t a, hipEvent_t b) {
                if (j == 0)
                    hipExtLaunchKernelGGL(k_igather, dim3(grid), dim3(256), 0, 0, a, b, 0,
                                          (const double*)field, (const int*)d_s, sbuf,
                                          uint64_t(n_send), L);
                else
                    hipExtLaunchKernelGGL(k_iscatter, dim3(grid), dim3(256), 0, 0, a, b, 0, field,
                                          (const int*)d_r, (const double*)rbuf, uint64_t(n_recv), L);
            };
            for (int i = 0; i < reps; ++i)
            {
                if (cold)
                    hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(256), 0, 0, (const v4*)fl,
                                       flush_bytes / 16, sink);
                else
                    launch(nullptr, nullptr);
                launch(e0, e1);
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                t.push_back(ms * 1e3f);
            }
            std::sort(t.begin(), t.end());
            out_us[2 * j + cold] = t[t.size() / 2];
        }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void* p : {(void*)field, (void*)sbuf, (void*)rbuf, (void*)d_s, (void*)d_r, (void*)fl, (void*)sink})
        if (p) (void)hipFree(p);
    return rc;
}



// Config 4's floors (round 5): several fields of element sizes es[k] (one (N+2H)^3 periodic
// domain each, layout_map<2,1,0>), placed in one allocation at 2 MiB-aligned offsets. Pack:
// one 16-B load per 128-B line the pack must read (x-face lines of every field first, as the
// plan dispatches short-row segments first), then the buffer writes (every field's halo bytes).
// Unpack: the buffer read, then every halo row's bytes written once in 16/8/4-B pieces
// (encoding: byte address / 4 in bits 0-29, size code in bits 30-31: 0 = 4 B, 1 = 8 B, 2 = 16 B).
static void field_lines(int N, int H, int es, uint64_t base, std::vector<uint8_t>& cls, uint64_t& useful)
{
    const int E = N + 2 * H;
    const uint64_t pitch = uint64_t(E) * es, plane = pitch * E;
    const int lo[3] = {H, H, N};
    const int hi[3] = {2 * H - 1, N + H - 1, N + H - 1};
    for (int dz = 0; dz < 3; ++dz)
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx)
            {
                if (dx == 1 && dy == 1 && dz == 1) continue;
                const int x0 = lo[dx], x1 = hi[dx];
                const bool shortrow = uint64_t(x1 - x0 + 1) * es < 64;
                for (int z = lo[dz]; z <= hi[dz]; ++z)
                    for (int y = lo[dy]; y <= hi[dy]; ++y)
                    {
                        const uint64_t b = base + uint64_t(z) * plane + uint64_t(y) * pitch + uint64_t(x0) * es;
                        const uint64_t e = b + uint64_t(x1 - x0 + 1) * es;
                        useful += e - b;
                        for (uint64_t l = b / 128; l <= (e - 1) / 128; ++l)
                            if (shortrow) cls[l] = 1;
                            else if (!cls[l]) cls[l] = 2;
                    }
            }
}

static void field_pieces(int N, int H, int es, uint64_t base, std::vector<uint32_t>& xf,
                         std::vector<uint32_t>& lg)
{
    const int E = N + 2 * H;
    const uint64_t pitch = uint64_t(E) * es, plane = pitch * E;
    const int lo[3] = {0, H, N + H};
    const int hi[3] = {H - 1, N + H - 1, N + 2 * H - 1};
    for (int dz = 0; dz < 3; ++dz)
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx)
            {
                if (dx == 1 && dy == 1 && dz == 1) continue;
                const int x0 = lo[dx], x1 = hi[dx];
                auto& out = uint64_t(x1 - x0 + 1) * es < 64 ? xf : lg;
                for (int z = lo[dz]; z <= hi[dz]; ++z)
                    for (int y = lo[dy]; y <= hi[dy]; ++y)
                    {
                        uint64_t b = base + uint64_t(z) * plane + uint64_t(y) * pitch + uint64_t(x0) * es;
                        const uint64_t e = b + uint64_t(x1 - x0 + 1) * es;
                        while (b < e)
                        {
                            uint32_t code = 0, w = 4;
                            if (b % 16 == 0 && e - b >= 16) code = 2, w = 16;
                            else if (b % 8 == 0 && e - b >= 8) code = 1, w = 8;
                            out.push_back(uint32_t(b / 4) | (code << 30));
                            b += w;
                        }
                    }
            }
}

__global__ __launch_bounds__(256) void k_pieces4(const uint32_t* __restrict__ pieces, uint32_t n,
                                                 char* __restrict__ field, const v4* __restrict__ buf,
                                                 uint64_t rvec, unsigned* sink)
{
    v4 acc{0, 0, 0, 0};
    const uint32_t stride = gridDim.x * 256u;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < rvec; i += uint64_t(stride)) acc ^= buf[i];
    for (uint32_t base = blockIdx.x * 256u + threadIdx.x; base < n; base += kU * stride)
    {
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            if (base + u * stride >= n) break;
            const uint32_t q = pieces[base + u * stride];
            char* a = field + uint64_t(q & 0x3fffffffu) * 4;
            const uint32_t code = q >> 30;
            if (code == 2) *(v4*)a = v4{q, acc.x, 2, 3};
            else if (code == 1) *(unsigned __attribute__((ext_vector_type(2)))*)a = {q, acc.y};
            else *(unsigned*)a = q ^ acc.z;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
}

// out_us[6]: {pack floor warm, cold, unpack (buffer read + halo writes) warm, cold, halo writes
// alone warm, cold}; counts[3]: lines, pieces, useful bytes. Returns 0, or the failing source line.
extern "C" int ghx_probe_multi_floor(int N, int H, int n_fields, const int* es, int reps,
                                     double* out_us, int64_t* counts)
{
    int rc = 0;
    const int E = N + 2 * H;
    std::vector<uint64_t> base(static_cast<size_t>(n_fields));
    uint64_t total = 0;
    for (int k = 0; k < n_fields; ++k)
    {
        base[size_t(k)] = total;
        total += (uint64_t(E) * E * E * es[k] + (uint64_t(2) << 20) - 1) / (uint64_t(2) << 20) * (uint64_t(2) << 20);
    }
    std::vector<uint8_t> cls(size_t(total / 128 + 1), 0);
    uint64_t useful = 0;
    for (int k = 0; k < n_fields; ++k) field_lines(N, H, es[k], base[size_t(k)], cls, useful);
    std::vector<uint32_t> lines;
    for (int pass = 1; pass <= 2; ++pass)
        for (size_t l = 0; l < cls.size(); ++l)
            if (cls[l] == pass) lines.push_back(uint32_t(l));
    std::vector<uint32_t> pxf, plg;
    for (int k = 0; k < n_fields; ++k) field_pieces(N, H, es[k], base[size_t(k)], pxf, plg);
    std::vector<uint32_t> pieces(pxf);
    pieces.insert(pieces.end(), plg.begin(), plg.end());
    counts[0] = int64_t(lines.size());
    counts[1] = int64_t(pieces.size());
    counts[2] = int64_t(useful);
    const size_t flush_bytes = size_t(1) << 30;
    char *field = nullptr, *fl = nullptr;
    v4* buf = nullptr;
    unsigned* sink = nullptr;
    uint32_t *d_l = nullptr, *d_p = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int grid = 256 * 8;
    if (total / 4 >= (uint64_t(1) << 30)) return __LINE__;
    CK(hipMalloc(&field, total));
    CK(hipMalloc(&fl, flush_bytes));
    CK(hipMalloc(&buf, useful + 64));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&d_l, lines.size() * 4 + 4));
    CK(hipMalloc(&d_p, pieces.size() * 4 + 4));
    CK(hipMemcpy(d_l, lines.data(), lines.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_p, pieces.data(), pieces.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(field, 1, total));
    CK(hipMemset(buf, 3, useful + 64));
    CK(hipMemset(fl, 2, flush_bytes));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int j = 0; j < 3; ++j)
        for (int cold = 0; cold < 2; ++cold)
        {
            auto go = [&](hipEvent_t a, hipEvent_t b) {
                if (j == 0)
                    hipExtLaunchKernelGGL(k_lines<>, dim3(grid), dim3(256), 0, 0, a, b, 0, d_l,
                                          uint32_t(lines.size()), (const char*)field, buf,
                                          uint64_t(useful / 16), sink);
                else  // j = 2: the halo writes alone (the unpack's write set), no buffer read
                    hipExtLaunchKernelGGL(k_pieces4, dim3(grid), dim3(256), 0, 0, a, b, 0, d_p,
                                          uint32_t(pieces.size()), field, (const v4*)buf,
                                          j == 1 ? uint64_t(useful / 16) : uint64_t(0), sink);
            };
            std::vector<float> t;
            for (int i = 0; i < reps; ++i)
            {
                if (cold)
                    hipLaunchKernelGGL(k_sweep, dim3(grid), dim3(256), 0, 0, (const v4*)fl,
                                       flush_bytes / 16, sink);
                else
                    go(nullptr, nullptr);
                go(e0, e1);
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                t.push_back(ms * 1e3f);
            }
            std::sort(t.begin(), t.end());
            out_us[2 * j + cold] = t[t.size() / 2];
        }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    for (void* p : {(void*)field, (void*)fl, (void*)buf, (void*)sink, (void*)d_l, (void*)d_p})
        if (p) (void)hipFree(p);
    return rc;
}

#ifdef PACK_FLOOR_MAIN
int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 21;
    const int N = argc > 2 ? atoi(argv[2]) : 512, H = argc > 3 ? atoi(argv[3]) : 2;
    double us[10];
    int64_t c[3];
    if (argc > 4)
    {
        // one unpack variant alone, warm (for rocprofv3 --pmc passes: tools/pmc_floor.sh)
        s_only_variant = atoi(argv[4]);
        const int rcv = ghx_probe_unpack_floor(N, H, reps, us, c);
        printf("{\"unpack_variant\": %d, \"us\": %.2f, \"rc\": %d}\n", s_only_variant,
               rcv ? -1.0 : us[2 * s_only_variant], rcv);
        return rcv ? 1 : 0;
    }
    const int rc = ghx_probe_pack_floor(N, H, reps, us, c);
    if (rc)
    {
        printf("{\"error\": \"HIP call failed at pack_floor.hip:%d\"}\n", rc);
        return 1;
    }
    printf("{\"config\": \"%d^3 fp64 H=%d pack read set\", \"useful_bytes\": %lld, \"xface_lines\": %lld, "
           "\"long_lines\": %lld}\n", N, H, (long long)c[2], (long long)c[0], (long long)c[1]);
    const char* names[4] = {"xface", "long", "both", "both_rw"};
    for (int j = 0; j < 4; ++j)
        for (int cold = 0; cold < 2; ++cold)
            printf("{\"set\": \"%s\", \"cold\": %d, \"us\": %.2f}\n", names[j], cold, us[2 * j + cold]);
    const int rc2 = ghx_probe_unpack_floor(N, H, reps, us, c);
    if (rc2)
    {
        printf("{\"error\": \"HIP call failed at pack_floor.hip:%d\"}\n", rc2);
        return 1;
    }
    printf("{\"config\": \"%d^3 fp64 H=%d unpack write set\", \"useful_bytes\": %lld, \"xface_pieces\": %lld, "
           "\"long_pieces\": %lld}\n", N, H, (long long)c[2], (long long)c[0], (long long)c[1]);
    const char* unames[5] = {"xface_writes", "long_writes", "writes", "writes_plus_buffer_reads",
                             "writes_buffer_reads_interleaved"};
    for (int j = 0; j < 5; ++j)
        for (int cold = 0; cold < 2; ++cold)
            printf("{\"set\": \"%s\", \"cold\": %d, \"us\": %.2f}\n", unames[j], cold, us[2 * j + cold]);
    const int rc3 = ghx_probe_fused_floor(N, H, reps, us);
    if (rc3)
    {
        printf("{\"error\": \"HIP call failed at pack_floor.hip:%d\"}\n", rc3);
        return 1;
    }
    for (int cold = 0; cold < 2; ++cold)
        printf("{\"set\": \"fused_reads_buffer_halos\", \"cold\": %d, \"us\": %.2f}\n", cold, us[cold]);
    return 0;
}
#endif
