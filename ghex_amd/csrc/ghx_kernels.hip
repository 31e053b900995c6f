// ghx_kernels.hip — gfx950 (CDNA4) pack / unpack kernels for the halo path.
//
// One launch covers every (field, iteration space, buffer) of a plan. Work is cut in the
// BUFFER's byte space: a workgroup tile is tile_bytes (default 8 KiB) of one segment's buffer
// range, so the buffer side is always a linear, fully coalesced 16 B/lane stream, and the field
// side is linear within each contiguous row. Each lane decodes its buffer byte position into
// (row, column) and the row into field coordinates with magic-number division, so no launch
// depends on the shape of an iteration space: face, edge and corner spaces of all fields share
// the one grid (the reference launches one kernel per iteration space per field,
// include/ghex/structured/pack_kernels.hpp:216-241, with a per-element 32-bit divide chain,
// include/ghex/structured/field_utils.hpp:128-159).
//
// Vector width per segment: the widest W in {16,8,4,2,1} bytes dividing the row length, the
// row offsets/strides (planner) and the runtime base pointers (checked per tile here), so the
// same plan is correct for any pointer alignment. No MFMA: this path is pure data movement.
//
// Variants (tuning, selected at launch): U = vectors in flight per lane per loop trip,
// NT = cache policy (0 default, 1 non-temporal stores, 2 non-temporal loads and stores).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>
#include <vector>

#include "ghx_internal.hpp"

namespace ghx
{
tuning g_tune{};

// Per-launch kernel timing (ghx_launch_timing): while enabled on a thread, every launch from that
// thread goes through hipExtLaunchKernelGGL with a start and a stop event, which the runtime
// records at the kernel's own begin and end (the interval rocprofv3's kernel trace reports),
// not around the host call. Eager launches only (not during stream capture).
thread_local std::vector<std::pair<hipEvent_t, hipEvent_t>>* t_timing = nullptr;

template<typename K, typename... A>
static void launch(K kernel, uint32_t grid, hipStream_t s, A... args)
{
    if (t_timing)
    {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess)
        {
            hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, s, e0, e1, 0, args...);
            t_timing->emplace_back(e0, e1);
            return;
        }
        if (e0) (void)hipEventDestroy(e0);
    }
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, s, args...);
}

namespace
{
__device__ __forceinline__ uint32_t fastdiv(uint32_t n, magic_u32 m)
{
    const uint32_t t = __umulhi(m.m, n);
    return (t + ((n - t) >> m.s1)) >> m.s2;
}

template<int W>
struct vec_t;
template<>
struct vec_t<16>
{
    using type = unsigned __attribute__((ext_vector_type(4)));
};
template<>
struct vec_t<8>
{
    using type = unsigned __attribute__((ext_vector_type(2)));
};
template<>
struct vec_t<4>
{
    using type = unsigned;
};
template<>
struct vec_t<2>
{
    using type = unsigned short;
};
template<>
struct vec_t<1>
{
    using type = unsigned char;
};

// Fields and buffers are device (global) memory: address-space-1 pointers make the compiler
// emit global_load/global_store instead of flat_* (no aperture check, and no lgkmcnt coupling
// that forces every store to wait for all outstanding loads).
#define GHX_GLOBAL __attribute__((address_space(1)))

template<typename V, bool NTL>
__device__ __forceinline__ V vload(const char* p)
{
    const GHX_GLOBAL V* g = (const GHX_GLOBAL V*)(p);
    if constexpr (NTL) return __builtin_nontemporal_load(g);
    else return *g;
}

template<typename V, bool NTS>
__device__ __forceinline__ void vstore(char* p, V v)
{
    GHX_GLOBAL V* g = (GHX_GLOBAL V*)(p);
    if constexpr (NTS) __builtin_nontemporal_store(v, g);
    else *g = v;
}

// Field-side accesses under the segment's cache policy (seg_s::fpol, uniform per tile):
// bit 0 = non-temporal load ("nt"), bit 1 = store with sc1 (gfx950 cache-policy bit; the
// compiler exposes no builtin for it, hence the asm). Short rows are the request-bound part of a
// halo; nt loads keep their 128-B line fills from allocating in the Infinity Cache, sc1 stores
// issue each masked row write once (tools/cpol_bench.hip).
template<typename V, bool NTL>
__device__ __forceinline__ V fload(const char* p, uint32_t pol)
{
    if (!NTL && (pol & 1u)) return __builtin_nontemporal_load((const GHX_GLOBAL V*)(p));
    return vload<V, NTL>(p);
}

template<typename V, bool NTS>
__device__ __forceinline__ void fstore(char* p, V v, uint32_t pol)
{
    if constexpr (sizeof(V) == 16)
    {
        if (!NTS && (pol & 2u))
        {
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            return;
        }
    }
    else if constexpr (sizeof(V) == 8)
    {
        if (!NTS && (pol & 2u))
        {
            asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            return;
        }
    }
    else if constexpr (sizeof(V) == 4)
    {
        if (!NTS && (pol & 2u))
        {
            asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            return;
        }
    }
    vstore<V, NTS>(p, v);
}

template<typename Seg>
__device__ __forceinline__ uint32_t fpol_of(const Seg& s)
{
    return s.fpol;
}

// field byte offset of segment-relative buffer position p (structured)
__device__ __forceinline__ int64_t field_offset_s(const seg_s& s, uint32_t p)
{
    const uint32_t row = fastdiv(p, s.mag_row);
    const uint32_t col = p - row * s.row_bytes;
    const uint32_t q0 = fastdiv(row, s.mag_ext[0]);
    const uint32_t c0 = row - q0 * s.ext[0];
    const uint32_t q1 = fastdiv(q0, s.mag_ext[1]);
    const uint32_t c1 = q0 - q1 * s.ext[1];
    const uint32_t q2 = fastdiv(q1, s.mag_ext[2]);
    const uint32_t c2 = q1 - q2 * s.ext[2];
    return s.field_off + int64_t(c0) * s.stride[0] + int64_t(c1) * s.stride[1] +
           int64_t(c2) * s.stride[2] + int64_t(q2) * s.stride[3] + int64_t(col);
}

__device__ __forceinline__ int64_t load_lid(const seg_u& s, uint32_t i)
{
    if (s.lid64) return ((const GHX_GLOBAL int64_t*)(s.lids))[i];
    return ((const GHX_GLOBAL int32_t*)(s.lids))[i];
}

// field byte offset of segment-relative buffer position p (unstructured: rows from lids)
__device__ __forceinline__ int64_t field_offset_u(const seg_u& s, uint32_t p)
{
    const uint32_t row = fastdiv(p, s.mag_row);
    const uint32_t col = p - row * s.row_bytes;
    uint32_t i, l;
    if (s.mode == 0)
    {
        i = row;
        l = 0;
    }
    else if (s.mode == 1)
    {
        i = fastdiv(row, s.mag_inner);
        l = row - i * s.row_levels;
    }
    else
    {
        l = fastdiv(row, s.mag_inner);
        i = row - l * s.n;
    }
    return load_lid(s, i) * s.index_stride_b + int64_t(l) * s.level_stride_b + int64_t(col);
}

// buffer byte position of segment-relative position p: p itself, except for sorted unstructured
// segments (lids visited in ascending field order; perm maps back to the buffer row)
__device__ __forceinline__ uint32_t buf_pos(const seg_s&, uint32_t p)
{
    return p;
}

__device__ __forceinline__ uint32_t buf_pos(const seg_u& s, uint32_t p)
{
    if (!s.perm) return p;
    const uint32_t row = fastdiv(p, s.mag_row);
    const uint32_t col = p - row * s.row_bytes;
    return ((const GHX_GLOBAL uint32_t*)(s.perm))[row] * s.row_bytes + col;
}

template<typename Seg>
__device__ __forceinline__ int64_t field_offset(const Seg& s, uint32_t p);
template<>
__device__ __forceinline__ int64_t field_offset<seg_s>(const seg_s& s, uint32_t p)
{
    return field_offset_s(s, p);
}
template<>
__device__ __forceinline__ int64_t field_offset<seg_u>(const seg_u& s, uint32_t p)
{
    return field_offset_u(s, p);
}

// Copy one tile [start, end) of a segment. Lane-linear in buffer space: lanes of a wave touch
// consecutive W-byte vectors of the buffer; U independent vectors in flight per lane.
template<bool PACK, int W, int U, int NT, typename Seg>
__device__ __forceinline__ void copy_tile(const Seg& s, char* __restrict__ field,
                                          char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    constexpr bool NTL = NT >= 2;             // 2, 3: non-temporal loads
    constexpr bool NTS = NT == 1 || NT == 2;  // 1, 2: non-temporal stores
    const uint32_t tid = threadIdx.x;
    const uint32_t pol = fpol_of(s);
    for (uint32_t base = start + tid * W; base < end; base += U * kBlock * W)
    {
        V v[U];
        int64_t fo[U];
        uint32_t bp[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                fo[u] = field_offset<Seg>(s, p);
                bp[u] = buf_pos(s, p);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if (PACK) v[u] = fload<V, NTL>(field + fo[u], pol);
                else v[u] = vload<V, NTL>(buf + bp[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if (PACK) vstore<V, NTS>(buf + bp[u], v[u]);
                else fstore<V, NTS>(field + fo[u], v[u], pol);
            }
        }
    }
}

// Unstructured rows of L = 4 or 8 bytes with run detection (seg_u::runs): lane t of a wave moves
// the 16-B buffer chunk [p, p+16) = rows r0 .. r0+K-1 (K = 16/L). It loads the chunk's K lids
// with one vector load and tests whether they form a run (lid[j] = lid[0] + j): then the K rows
// are 16 contiguous field bytes and move as ONE 16-B field access; otherwise as K L-byte
// accesses assembled into the same 16-B buffer vector. The buffer side is a lane-linear
// 16 B/lane stream either way (the one-row-per-lane path moves 4-8 B per lane instruction).
// A wave whose lids are all runs issues the per-row instructions with an empty EXEC mask, which
// the hardware skips; mixed waves execute both, masked. Field accesses of a run are only
// L-aligned: the HSA runtime runs kernels in unaligned-access mode, so a 16-B access at a 4-B
// aligned address is legal (split by the TA where it crosses a line).
using v4_a4 = unsigned __attribute__((ext_vector_type(4), aligned(4)));

template<int K>
__device__ __forceinline__ void load_lids(const seg_u& s, uint32_t r0, int64_t (&l)[K])
{
    if (s.lid64)
    {
        const GHX_GLOBAL vec_t<16>::type* p =
            (const GHX_GLOBAL vec_t<16>::type*)((const int64_t*)(s.lids) + r0);
#pragma unroll
        for (int j = 0; j < K; j += 2)
        {
            const auto q = p[j / 2];
            l[j] = int64_t(uint64_t(q.x) | (uint64_t(q.y) << 32));
            l[j + 1] = int64_t(uint64_t(q.z) | (uint64_t(q.w) << 32));
        }
    }
    else if constexpr (K == 2)
    {
        const auto q = *(const GHX_GLOBAL vec_t<8>::type*)((const int32_t*)(s.lids) + r0);
        l[0] = int32_t(q.x);
        l[1] = int32_t(q.y);
    }
    else
    {
        const auto q = *(const GHX_GLOBAL vec_t<16>::type*)((const int32_t*)(s.lids) + r0);
        l[0] = int32_t(q.x);
        l[1] = int32_t(q.y);
        l[2] = int32_t(q.z);
        l[3] = int32_t(q.w);
    }
}

template<int L>
__device__ __forceinline__ vec_t<16>::type assemble(const typename vec_t<L>::type (&w)[16 / L])
{
    if constexpr (L == 8) return vec_t<16>::type{w[0].x, w[0].y, w[1].x, w[1].y};
    else return vec_t<16>::type{w[0], w[1], w[2], w[3]};
}

template<int L>
__device__ __forceinline__ void split(vec_t<16>::type v, typename vec_t<L>::type (&w)[16 / L])
{
    if constexpr (L == 8)
    {
        w[0] = vec_t<8>::type{v.x, v.y};
        w[1] = vec_t<8>::type{v.z, v.w};
    }
    else
    {
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
    }
}

template<bool PACK, int L, int U, int NT>
__device__ __forceinline__ void copy_runs(const seg_u& s, char* __restrict__ field,
                                          char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<16>::type;
    using R = typename vec_t<L>::type;
    constexpr int K = 16 / L;
    constexpr bool NTL = NT >= 2;
    constexpr bool NTS = NT == 1 || NT == 2;
    const uint32_t pol = s.fpol;
    for (uint32_t base = start + threadIdx.x * 16; base < end; base += U * kBlock * 16)
    {
        int64_t fo[U][K];
        uint32_t full = 0, run = 0;  // bit u: chunk u holds K rows / ... that form a run
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * 16;
            if (p >= end) continue;
            const uint32_t r0 = p / L;
            int64_t l[K];
            if (p + 16 <= end)
            {
                full |= 1u << u;
                load_lids<K>(s, r0, l);
                bool c = true;
#pragma unroll
                for (int j = 1; j < K; ++j) c = c && l[j] == l[0] + j;
                if (c) run |= 1u << u;
            }
            else
            {
#pragma unroll
                for (int j = 0; j < K; ++j) l[j] = p + j * L < end ? load_lid(s, r0 + j) : 0;
            }
#pragma unroll
            for (int j = 0; j < K; ++j) fo[u][j] = l[j] * L;  // index stride = L (planner)
        }
        V v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * 16;
            if (p >= end || !(full >> u & 1u)) continue;
            if (PACK)
            {
                if (run >> u & 1u)
                {
                    const v4_a4 x = fload<v4_a4, NTL>(field + fo[u][0], pol);
                    v[u] = V{x.x, x.y, x.z, x.w};
                }
                else
                {
                    R w[K];
#pragma unroll
                    for (int j = 0; j < K; ++j) w[j] = fload<R, NTL>(field + fo[u][j], pol);
                    v[u] = assemble<L>(w);
                }
            }
            else
                v[u] = vload<V, NTL>(buf + p);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * 16;
            if (p >= end) continue;
            if (!(full >> u & 1u))
            {
                // segment tail: fewer than K rows left, row by row
#pragma unroll
                for (int j = 0; j < K; ++j)
                {
                    if (p + j * L >= end) break;
                    if (PACK) vstore<R, NTS>(buf + p + j * L, fload<R, NTL>(field + fo[u][j], pol));
                    else fstore<R, NTS>(field + fo[u][j], vload<R, NTL>(buf + p + j * L), pol);
                }
                continue;
            }
            if (PACK)
                vstore<V, NTS>(buf + p, v[u]);
            else if (run >> u & 1u)
                fstore<v4_a4, NTS>(field + fo[u][0], v4_a4{v[u].x, v[u].y, v[u].z, v[u].w}, pol);
            else
            {
                R w[K];
                split<L>(v[u], w);
#pragma unroll
                for (int j = 0; j < K; ++j) fstore<R, NTS>(field + fo[u][j], w[j], pol);
            }
        }
    }
}

// Paired segments (planner: pair_segments): lane moves row r of the primary and row r-1 of the
// partner, whose field pieces share a cache line; both buffer streams stay lane-linear.
template<bool PACK, int W, int U, int NT>
__device__ __forceinline__ void copy_tile_pair(const seg_s& s, const seg_s& q,
                                               char* __restrict__ field, char* __restrict__ buf,
                                               char* __restrict__ qbuf, uint32_t start,
                                               uint32_t end)
{
    using V = typename vec_t<W>::type;
    constexpr bool NTL = NT >= 2;
    constexpr bool NTS = NT == 1 || NT == 2;
    const uint32_t tid = threadIdx.x;
    const uint32_t L = s.row_bytes;
    for (uint32_t base = start + tid * W; base < end; base += U * kBlock * W)
    {
        V v[U], w[U];
        int64_t fo[U], fq[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                fo[u] = field_offset_s(s, p);
                if (p >= L) fq[u] = field_offset_s(q, p - L);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if (PACK)
                {
                    v[u] = vload<V, NTL>(field + fo[u]);
                    if (p >= L) w[u] = vload<V, NTL>(field + fq[u]);
                }
                else
                {
                    v[u] = vload<V, NTL>(buf + p);
                    if (p >= L) w[u] = vload<V, NTL>(qbuf + (p - L));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if (PACK)
                {
                    vstore<V, NTS>(buf + p, v[u]);
                    if (p >= L) vstore<V, NTS>(qbuf + (p - L), w[u]);
                }
                else
                {
                    vstore<V, NTS>(field + fo[u], v[u]);
                    if (p >= L) vstore<V, NTS>(field + fq[u], w[u]);
                }
            }
        }
    }
}

// Interleaved pairs (knob pair = 2): the rows of the primary P and of its line partner Q (row r
// of P shares a cache line with row r-1 of Q: the -x piece of row y+1 and the +x piece of row y
// of a unit-stride field) are dealt to ALTERNATE lanes — lane 2i moves row i of P, lane 2i+1
// row i-1 of Q — so the two pieces of one line are requested by ONE wave instruction, which the
// texture addresser merges into one request per line (per-lane pairing issues them in two
// instructions). Each buffer side stays a contiguous stream (even lanes into P's range, odd
// lanes into Q's). Rows of exactly one vector (L == W: 8 or 16 B, halo 1 or 2 of fp64).
template<bool PACK, int W, int U, int NT>
__device__ __forceinline__ void copy_tile_ilv(const seg_s& s, const seg_s& q,
                                              char* __restrict__ field, char* __restrict__ buf,
                                              char* __restrict__ qbuf, uint32_t start,
                                              uint32_t end)
{
    using V = typename vec_t<W>::type;
    constexpr bool NTL = NT >= 2;
    constexpr bool NTS = NT == 1 || NT == 2;
    const uint32_t total = 2 * ((end - start) / W);  // whole rows per tile (planner)
    for (uint32_t e0 = threadIdx.x; e0 < total; e0 += U * kBlock)
    {
        V v[U];
        int64_t fo[U];
        char* bp[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t e = e0 + uint32_t(u) * kBlock;
            const uint32_t side = e & 1u;
            const uint32_t p = start + (e >> 1) * W;  // primary row position
            ok[u] = e < total && (side == 0 || p >= W);
            const uint32_t pp = side ? p - W : p;
            // P and Q have the same shape: only their bases differ
            fo[u] = field_offset_s(s, pp) - s.field_off + (side ? q.field_off : s.field_off);
            bp[u] = (side ? qbuf : buf) + pp;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u]) v[u] = PACK ? vload<V, NTL>(field + fo[u]) : vload<V, NTL>(bp[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u])
            {
                if (PACK) vstore<V, NTS>(bp[u], v[u]);
                else vstore<V, NTS>(field + fo[u], v[u]);
            }
    }
}

template<bool PACK, int U, int NT>
__device__ __forceinline__ void dispatch_pair(const seg_s& s, const seg_s& q, char* field,
                                              char* buf, char* qbuf, uint32_t start, uint32_t end,
                                              int w)
{
    switch (w)
    {
        case 4: copy_tile_pair<PACK, 16, U, NT>(s, q, field, buf, qbuf, start, end); break;
        case 3: copy_tile_pair<PACK, 8, U, NT>(s, q, field, buf, qbuf, start, end); break;
        case 2: copy_tile_pair<PACK, 4, U, NT>(s, q, field, buf, qbuf, start, end); break;
        case 1: copy_tile_pair<PACK, 2, U, NT>(s, q, field, buf, qbuf, start, end); break;
        default: copy_tile_pair<PACK, 1, U, NT>(s, q, field, buf, qbuf, start, end); break;
    }
}

template<bool PACK, int U, int NT, bool ILV, typename Seg>
__device__ __forceinline__ bool try_pair(const Seg&, const Seg*, const kargs&, char*, char*,
                                         uint32_t, uint32_t, int)
{
    return false;
}

template<bool PACK, int U, int NT, bool ILV>
__device__ __forceinline__ bool try_pair(const seg_s& s, const seg_s* segs, const kargs& a,
                                         char* field, char* buf, uint32_t start, uint32_t end,
                                         int w)
{
    if (s.partner < 0) return false;
    const seg_s q = segs[s.partner];
    char* qbuf = reinterpret_cast<char*>(a.buf_ptr[q.buf_slot]) + q.buf_off;
    w = min(w, int(__builtin_ctzll(reinterpret_cast<uint64_t>(qbuf) | 16ull)));
    if constexpr (ILV)
    {
        if (w == 4 && s.row_bytes == 16)
        {
            copy_tile_ilv<PACK, 16, U, NT>(s, q, field, buf, qbuf, start, end);
            return true;
        }
        if (w == 3 && s.row_bytes == 8)
        {
            copy_tile_ilv<PACK, 8, U, NT>(s, q, field, buf, qbuf, start, end);
            return true;
        }
    }
    dispatch_pair<PACK, U, NT>(s, q, field, buf, qbuf, start, end, w);
    return true;
}

// LDS-staged pack of a short-row tile (knob "lds"; the north star's stride -> linear transpose
// through LDS, kept as a measured alternative): each wave takes 64 rows per trip. Phase 1 reads,
// for each row, the whole aligned 64-B block that holds it, four lanes per block (16 rows per
// wave instruction, every access a full 16-B vector at a 16-B boundary) and stages the blocks in
// the wave's LDS slice; phase 2 gives one row per lane: the lane extracts its R-byte piece from
// LDS and stores it to the lane-linear buffer. The fabric sees the same line requests as the
// direct form (the blocks are the rows' own lines); L1/TA traffic is 64/R times the direct form's.
// Rows of R = 8 or 16 bytes whose field offsets are R-aligned (checked by the caller). Blocks are
// read whole: an aligned 64-B block never crosses a page, so bytes outside the rows are readable.
constexpr uint32_t kLdsRows = 64;   // rows per wave per trip
constexpr uint32_t kLdsPitch = 80;  // staged bytes per row: the block + 16 B (spreads LDS banks)

template<int R>
__device__ __forceinline__ void copy_tile_lds(const seg_s& s, char* __restrict__ field,
                                              char* __restrict__ buf, uint32_t start, uint32_t end,
                                              char* lds)
{
    using V = vec_t<16>::type;
    using VR = typename vec_t<R>::type;
    const uint32_t lane = threadIdx.x & 63u;
    char* slice = lds + (threadIdx.x >> 6) * (kLdsRows * kLdsPitch);
    const uint32_t r1 = end / R;
    for (uint32_t base = start / R + (threadIdx.x >> 6) * kLdsRows; base < r1;
         base += (kBlock / 64) * kLdsRows)
    {
        V v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            const uint32_t row = base + u * 16 + (lane >> 2);
            if (row < r1)
            {
                const uintptr_t a = reinterpret_cast<uintptr_t>(field + field_offset_s(s, row * R));
                v[u] = vload<V, false>(reinterpret_cast<const char*>(a & ~uintptr_t(63)) + (lane & 3u) * 16);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (base + u * 16 + (lane >> 2) < r1)
                *reinterpret_cast<V*>(slice + (u * 16 + (lane >> 2)) * kLdsPitch + (lane & 3u) * 16) = v[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t row = base + lane;
        if (row < r1)
        {
            const uintptr_t a = reinterpret_cast<uintptr_t>(field + field_offset_s(s, row * R));
            const VR x = *reinterpret_cast<const VR*>(slice + lane * kLdsPitch + (a & 63u));
            vstore<VR, false>(buf + row * R, x);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next trip
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

__device__ __forceinline__ int ptr_wlog2(uint64_t p)
{
    return __builtin_ctzll(p | 16ull);  // log2 of the largest power of two (<= 16) dividing p
}

// RUNS (unstructured only): every segment of the plan takes the run path (copy_runs); the host
// (uplan::execute) launches this variant only when runs_ok holds for all of them, so the
// general path's registers do not weigh on it and vice versa. PAIR (structured only): the plan
// holds paired segments (knob "pair"); the pair path more than doubles the kernel's VGPRs
// (156 vs 73 at U=4), so plans without pairs launch the variant that leaves it out.
template<bool PACK, int U, int NT, typename Seg, bool RUNS = false, bool PAIR = false,
         bool ILV = false, bool LDS = false>
__global__ __launch_bounds__(kBlock) void k_copy(kargs a)
{
    const Seg* __restrict__ segs = static_cast<const Seg*>(a.segs);
    char* lds = nullptr;
    if constexpr (LDS)
    {
        __shared__ __attribute__((aligned(16))) char stage[(kBlock / 64) * kLdsRows * kLdsPitch];
        lds = stage;
    }
    for (uint32_t t = blockIdx.x; t < a.n_tiles; t += gridDim.x)
    {
        const uint32_t si = a.tile_seg[2 * t];
        const uint32_t ti = a.tile_seg[2 * t + 1];
        const Seg s = segs[si];
        const uint32_t start = ti * s.tile_bytes;
        const uint32_t end = min(start + s.tile_bytes, s.bytes);
        char* field = reinterpret_cast<char*>(a.field_ptr[s.field_slot]);
        char* buf = reinterpret_cast<char*>(a.buf_ptr[s.buf_slot]) + s.buf_off;
        int w = s.wlog2;
        w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(field)));
        w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(buf)));
        if constexpr (RUNS)
        {
            if (s.row_bytes == 8) copy_runs<PACK, 8, U, NT>(s, field, buf, start, end);
            else copy_runs<PACK, 4, U, NT>(s, field, buf, start, end);
            continue;
        }
        if constexpr (PAIR)
        {
            if (try_pair<PACK, U, NT, ILV>(s, segs, a, field, buf, start, end, w)) continue;
        }
        if constexpr (LDS && PACK && std::is_same_v<Seg, seg_s>)
        {
            if (s.row_bytes == 16 && w >= 4)
            {
                copy_tile_lds<16>(s, field, buf, start, end, lds);
                continue;
            }
            if (s.row_bytes == 8 && w >= 3)
            {
                copy_tile_lds<8>(s, field, buf, start, end, lds);
                continue;
            }
        }
        switch (w)
        {
            case 4: copy_tile<PACK, 16, U, NT>(s, field, buf, start, end); break;
            case 3: copy_tile<PACK, 8, U, NT>(s, field, buf, start, end); break;
            case 2: copy_tile<PACK, 4, U, NT>(s, field, buf, start, end); break;
            case 1: copy_tile<PACK, 2, U, NT>(s, field, buf, start, end); break;
            default: copy_tile<PACK, 1, U, NT>(s, field, buf, start, end); break;
        }
    }
}

template<bool PACK, int U, int NT>
__device__ __forceinline__ void copy_any(const seg_s& s, char* field, char* buf, uint32_t start,
                                         uint32_t end, int w)
{
    switch (w)
    {
        case 4: copy_tile<PACK, 16, U, NT>(s, field, buf, start, end); break;
        case 3: copy_tile<PACK, 8, U, NT>(s, field, buf, start, end); break;
        case 2: copy_tile<PACK, 4, U, NT>(s, field, buf, start, end); break;
        case 1: copy_tile<PACK, 2, U, NT>(s, field, buf, start, end); break;
        default: copy_tile<PACK, 1, U, NT>(s, field, buf, start, end); break;
    }
}

// Software-pipelined self tile (pack and unpack of one tile with the same vector width W): trip j
// loads the field rows of chunk j (pack) and the buffer bytes of chunk j-1 (unpack), stores
// chunk j to the buffer, waits for ITS OWN memory operations, passes the workgroup barrier (chunk
// j's buffer bytes are then complete for every wave), and only then stores chunk j-1 into the
// halos. Those halo stores — the scattered writes of the x-faces — are left in flight under the
// next trip's scattered field loads instead of being drained by every barrier, so the x-face reads
// and writes overlap inside each workgroup (with plain __syncthreads between a whole pack half and
// a whole unpack half, all x-face workgroups read, then all of them write).
template<int W, int U>
__device__ __forceinline__ void self_pipelined(const seg_s& s, const seg_s& q,
                                               char* __restrict__ fp, char* __restrict__ fu,
                                               char* __restrict__ buf, uint32_t start,
                                               uint32_t end)
{
    using V = typename vec_t<W>::type;
    constexpr uint32_t K = uint32_t(U) * kBlock * W;  // buffer bytes per trip
    const uint32_t lane = threadIdx.x * W;
    const uint32_t pol_p = s.fpol, pol_u = q.fpol;
    const uint32_t n = (end - start + K - 1) / K;
    for (uint32_t j = 0; j <= n; ++j)
    {
        const uint32_t cp = start + j * K;  // pack chunk (j < n)
        const uint32_t cu = cp - K;         // unpack chunk (j > 0)
        V pv[U], uv[U];
        int64_t fo[U];
        if (j < n)
        {
#pragma unroll
            for (int u = 0; u < U; ++u)
            {
                const uint32_t p = cp + uint32_t(u) * kBlock * W + lane;
                if (p < end) pv[u] = fload<V, false>(fp + field_offset_s(s, p), pol_p);
            }
        }
        if (j > 0)
        {
#pragma unroll
            for (int u = 0; u < U; ++u)
            {
                const uint32_t p = cu + uint32_t(u) * kBlock * W + lane;
                if (p < end)
                {
                    uv[u] = vload<V, false>(buf + p);
                    fo[u] = field_offset_s(q, p);
                }
            }
        }
        if (j < n)
        {
#pragma unroll
            for (int u = 0; u < U; ++u)
            {
                const uint32_t p = cp + uint32_t(u) * kBlock * W + lane;
                if (p < end) vstore<V, false>(buf + p, pv[u]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's buffer stores landed
        __builtin_amdgcn_s_barrier();                      // ... and every other wave's
        if (j > 0)
        {
#pragma unroll
            for (int u = 0; u < U; ++u)
            {
                const uint32_t p = cu + uint32_t(u) * kBlock * W + lane;
                if (p < end) fstore<V, false>(fu + fo[u], uv[u], pol_u);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // lanes are reused by the next tile of a grid-stride loop
}

// Lane-local self tile with store-to-load forwarding: the unpack half needs exactly the buffer
// bytes this lane has just stored (same positions, same width), so it takes them from the
// registers instead of loading them back: field interior -> register -> buffer store AND halo
// store. Every buffer byte and every halo byte is still written; what disappears is the
// buffer read-back (which the lane-local form served from L2, or, for ~20 % of it, from HBM:
// TCC_EA0_RDREQ 573k against 461k for the field reads alone).
template<int W, int U, int NT>
__device__ __forceinline__ void self_forward(const seg_s& s, const seg_s& q,
                                             char* __restrict__ fp, char* __restrict__ fu,
                                             char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    constexpr bool NTL = NT >= 2;
    constexpr bool NTS = NT == 1 || NT == 2;
    const uint32_t pol_p = s.fpol, pol_u = q.fpol;
    for (uint32_t base = start + threadIdx.x * W; base < end; base += U * kBlock * W)
    {
        V v[U];
        int64_t op[U], ou[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                op[u] = field_offset_s(s, p);
                ou[u] = field_offset_s(q, p);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end) v[u] = fload<V, NTL>(fp + op[u], pol_p);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                vstore<V, NTS>(buf + p, v[u]);
                fstore<V, NTS>(fu + ou[u], v[u], pol_u);
            }
        }
    }
}

// Fused self exchange: every message is a self message, so pack segment k and unpack segment k
// cover the same buffer bytes. A workgroup packs its tile (field interior -> buffer), waits at a
// workgroup barrier (its own stores are visible to its own waves), then unpacks the same bytes
// (buffer -> field halo). All bytes of pack and unpack move; the hand-off never leaves the CU.
// PIPE: the software-pipelined variant (knob "self_pipe") is compiled into its own kernel, so
// its registers (148 vs 116 VGPRs at U=4) do not cost the default kernel occupancy.
template<int U, int NT, bool PIPE = false>
__global__ __launch_bounds__(kBlock) void k_self(kargs a)
{
    const seg_s* __restrict__ ps = static_cast<const seg_s*>(a.segs);
    const seg_s* __restrict__ us = static_cast<const seg_s*>(a.segs2);
    for (uint32_t t = blockIdx.x; t < a.n_tiles; t += gridDim.x)
    {
        const uint32_t si = a.tile_seg[2 * t];
        const uint32_t ti = a.tile_seg[2 * t + 1];
        const seg_s s = ps[si];
        const seg_s q = us[si];
        const uint32_t start = ti * s.tile_bytes;
        const uint32_t end = min(start + s.tile_bytes, s.bytes);
        char* field_p = reinterpret_cast<char*>(a.field_ptr[s.field_slot]);
        char* field_u = reinterpret_cast<char*>(a.field_ptr[q.field_slot]);
        char* buf = reinterpret_cast<char*>(a.buf_ptr[s.buf_slot]) + s.buf_off;
        int wp = min(int(s.wlog2), ptr_wlog2(reinterpret_cast<uint64_t>(field_p)));
        wp = min(wp, ptr_wlog2(reinterpret_cast<uint64_t>(buf)));
        int wu = min(int(q.wlog2), ptr_wlog2(reinterpret_cast<uint64_t>(field_u)));
        wu = min(wu, ptr_wlog2(reinterpret_cast<uint64_t>(buf)));
        if (q.bytes == 0)
        {
            // a peer message of a mixed exchange (ghx_exchange_pack_self): pack only
            copy_any<true, U, NT>(s, field_p, buf, start, end, wp);
            continue;
        }
        if constexpr (PIPE)
        {
            if (wp == wu && s.row_bytes < a.pipe)
            {
                switch (wp)
                {
                    case 4: self_pipelined<16, U>(s, q, field_p, field_u, buf, start, end); break;
                    case 3: self_pipelined<8, U>(s, q, field_p, field_u, buf, start, end); break;
                    case 2: self_pipelined<4, U>(s, q, field_p, field_u, buf, start, end); break;
                    case 1: self_pipelined<2, U>(s, q, field_p, field_u, buf, start, end); break;
                    default: self_pipelined<1, U>(s, q, field_p, field_u, buf, start, end); break;
                }
                continue;
            }
        }
        // Whole tile, or in chunks of a.chunk buffer bytes (g_tune.self_chunk, a knob: keeping
        // the re-read bytes in L2 this way measured no faster).
        if (wp == wu && a.lane_local == 2)
        {
            switch (wp)
            {
                case 4: self_forward<16, U, NT>(s, q, field_p, field_u, buf, start, end); break;
                case 3: self_forward<8, U, NT>(s, q, field_p, field_u, buf, start, end); break;
                case 2: self_forward<4, U, NT>(s, q, field_p, field_u, buf, start, end); break;
                case 1: self_forward<2, U, NT>(s, q, field_p, field_u, buf, start, end); break;
                default: self_forward<1, U, NT>(s, q, field_p, field_u, buf, start, end); break;
            }
            continue;
        }
        if (wp == wu && a.lane_local)
        {
            // Same vector width on both sides: every lane unpacks exactly the buffer bytes it
            // packed (same lane -> position map), so the hand-off is program order within the
            // lane (its own stores, then its own loads of the same addresses) and no workgroup
            // barrier is needed: waves run free, and one wave's halo writes overlap other waves'
            // field reads instead of every wave of the tile reading first and writing after.
            copy_any<true, U, NT>(s, field_p, buf, start, end, wp);
            asm volatile("" ::: "memory");  // keep the unpack's buffer loads after the stores
            copy_any<false, U, NT>(q, field_u, buf, start, end, wu);
            continue;
        }
        const uint32_t chunk = a.chunk ? a.chunk : s.tile_bytes;
        for (uint32_t c = start; c < end; c += chunk)
        {
            const uint32_t ce = min(c + chunk, end);
            copy_any<true, U, NT>(s, field_p, buf, c, ce, wp);
            __syncthreads();  // workgroup release/acquire: the chunk's buffer bytes are complete
            copy_any<false, U, NT>(q, field_u, buf, c, ce, wu);
            __syncthreads();  // the next chunk / tile reuses the lanes
        }
    }
}

// Zero-copy put: element p of the virtual message is read from the source field through the
// pack segment's addressing and written to the target field (peer memory or local) through the
// unpack segment's addressing, register to register — no buffer.
template<int W, int U>
__device__ __forceinline__ void copy_direct(const seg_s& s, const seg_s& q,
                                            const char* __restrict__ src, char* __restrict__ dst,
                                            uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    for (uint32_t base = start + threadIdx.x * W; base < end; base += U * kBlock * W)
    {
        V v[U];
        int64_t fd[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                v[u] = vload<V, false>(src + field_offset_s(s, p));
                fd[u] = field_offset_s(q, p);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end) vstore<V, false>(dst + fd[u], v[u]);
        }
    }
}

template<int U>
__global__ __launch_bounds__(kBlock) void k_put(kargs a)
{
    const seg_s* __restrict__ ps = static_cast<const seg_s*>(a.segs);
    const seg_s* __restrict__ qs = static_cast<const seg_s*>(a.segs2);
    for (uint32_t t = blockIdx.x; t < a.n_tiles; t += gridDim.x)
    {
        const uint32_t si = a.tile_seg[2 * t];
        const uint32_t ti = a.tile_seg[2 * t + 1];
        const seg_s s = ps[si];
        const seg_s q = qs[si];
        const uint32_t start = ti * s.tile_bytes;
        const uint32_t end = min(start + s.tile_bytes, s.bytes);
        const char* src = reinterpret_cast<const char*>(a.field_ptr[s.field_slot]);
        char* dst = reinterpret_cast<char*>(a.buf_ptr[q.field_slot]);
        int w = min(int(s.wlog2), int(q.wlog2));
        w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(src)));
        w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(dst)));
        switch (w)
        {
            case 4: copy_direct<16, U>(s, q, src, dst, start, end); break;
            case 3: copy_direct<8, U>(s, q, src, dst, start, end); break;
            case 2: copy_direct<4, U>(s, q, src, dst, start, end); break;
            case 1: copy_direct<2, U>(s, q, src, dst, start, end); break;
            default: copy_direct<1, U>(s, q, src, dst, start, end); break;
        }
    }
}

template<typename Seg, bool PACK, int U>
void launch_nt(const kargs& a, hipStream_t s, uint32_t grid)
{
    // nt_dir: 0 the policy applies to both directions, 1 to the pack only, 2 to the unpack only
    const int nt = (g_tune.nt_dir == 0 || (g_tune.nt_dir == 1) == PACK) ? g_tune.nt : 0;
    switch (nt)
    {
        case 1: launch((k_copy<PACK, U, 1, Seg>), grid, s, a); break;
        case 2: launch((k_copy<PACK, U, 2, Seg>), grid, s, a); break;
        case 3: launch((k_copy<PACK, U, 3, Seg>), grid, s, a); break;
        default: launch((k_copy<PACK, U, 0, Seg>), grid, s, a); break;
    }
}

template<typename Seg, bool PACK>
void launch_variant(const kargs& a, hipStream_t s, uint32_t grid)
{
    if (g_tune.unroll == 8) launch_nt<Seg, PACK, 8>(a, s, grid);
    else if (g_tune.unroll == 2) launch_nt<Seg, PACK, 2>(a, s, grid);
    else launch_nt<Seg, PACK, 4>(a, s, grid);
}
}  // namespace

void timing_enable(bool on)
{
    if (on && !t_timing) t_timing = new std::vector<std::pair<hipEvent_t, hipEvent_t>>();
    if (!on && t_timing)
    {
        for (auto& e : *t_timing)
        {
            (void)hipEventSynchronize(e.second);
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        delete t_timing;
        t_timing = nullptr;
    }
}

int timing_read(float* ms, int32_t cap, int32_t* n)
{
    int32_t k = 0;
    hipError_t bad = hipSuccess;
    if (t_timing)
    {
        for (auto& e : *t_timing)
        {
            float t = 0.f;
            hipError_t r = hipEventSynchronize(e.second);
            if (r == hipSuccess) r = hipEventElapsedTime(&t, e.first, e.second);
            if (r != hipSuccess && bad == hipSuccess) bad = r;
            if (ms && k < cap) ms[k] = t;
            ++k;
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        t_timing->clear();
    }
    if (n) *n = k;
    if (bad != hipSuccess)
    {
        set_error(std::string("launch timing: ") + hipGetErrorString(bad));
        return GHX_ERR_HIP;
    }
    return GHX_OK;
}

uint32_t grid_for_tiles(uint32_t n_tiles)
{
    uint32_t cap = g_tune.grid_cap > 0 ? uint32_t(g_tune.grid_cap) : (1u << 20);
    return n_tiles < cap ? n_tiles : cap;
}

int launch_structured(const kargs& a, int direction, void* stream, uint32_t grid, int pairs)
{
    if (a.n_tiles == 0) return GHX_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // plans with paired segments (knob "pair"): one variant, U = 4, default cache policy;
    // pairs == 2: the two rows of a line on alternate lanes of one instruction
    if (pairs == 2 && direction == 0)
        launch((k_copy<true, 4, 0, seg_s, false, true, true>), grid, s, a);
    else if (pairs == 2)
        launch((k_copy<false, 4, 0, seg_s, false, true, true>), grid, s, a);
    else if (!pairs && g_tune.lds && direction == 0)  // LDS-staged short rows (knob "lds")
        launch((k_copy<true, 4, 0, seg_s, false, false, false, true>), grid, s, a);
    else if (pairs && direction == 0)
        launch((k_copy<true, 4, 0, seg_s, false, true>), grid, s, a);
    else if (pairs)
        launch((k_copy<false, 4, 0, seg_s, false, true>), grid, s, a);
    else if (direction == 0) launch_variant<seg_s, true>(a, s, grid);
    else launch_variant<seg_s, false>(a, s, grid);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
    {
        set_error(std::string("structured kernel launch failed: ") + hipGetErrorString(e));
        return GHX_ERR_HIP;
    }
    return GHX_OK;
}

int launch_self(const kargs& a, void* stream, uint32_t grid)
{
    if (a.n_tiles == 0) return GHX_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (a.pipe)  // software-pipelined tiles (a developer knob): one variant, U = 4
        launch((k_self<4, 0, true>), grid, s, a);
    else if (g_tune.unroll == 8) launch((k_self<8, 0>), grid, s, a);
    else if (g_tune.unroll == 2) launch((k_self<2, 0>), grid, s, a);
    else launch((k_self<4, 0>), grid, s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
    {
        set_error(std::string("self-exchange kernel launch failed: ") + hipGetErrorString(e));
        return GHX_ERR_HIP;
    }
    return GHX_OK;
}

int launch_put(const kargs& a, void* stream, uint32_t grid)
{
    if (a.n_tiles == 0) return GHX_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (g_tune.unroll == 8) launch((k_put<8>), grid, s, a);
    else if (g_tune.unroll == 2) launch((k_put<2>), grid, s, a);
    else launch((k_put<4>), grid, s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
    {
        set_error(std::string("put kernel launch failed: ") + hipGetErrorString(e));
        return GHX_ERR_HIP;
    }
    return GHX_OK;
}

int launch_unstructured(const kargs& a, int direction, void* stream, uint32_t grid, bool runs)
{
    if (a.n_tiles == 0) return GHX_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (runs && direction == 0)
        launch((k_copy<true, 4, 0, seg_u, true>), grid, s, a);
    else if (runs)
        launch((k_copy<false, 4, 0, seg_u, true>), grid, s, a);
    else if (direction == 0) launch_variant<seg_u, true>(a, s, grid);
    else launch_variant<seg_u, false>(a, s, grid);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
    {
        set_error(std::string("unstructured kernel launch failed: ") + hipGetErrorString(e));
        return GHX_ERR_HIP;
    }
    return GHX_OK;
}

}  // namespace ghx
