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
// Four vectors in flight per lane per loop trip (U = 4; 2 and 8 measured slower).
//
// The variants that lost their A/Bs in rounds 1-2 (paired / interleaved / LDS-staged short rows,
// software-pipelined and chunked self tiles, non-temporal policies) were removed from this file
// in round 3; their code and numbers are in tools/kernel_variants_r02.hip.
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
constexpr int kU = 4;  // vectors in flight per lane per loop trip

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

template<typename V>
__device__ __forceinline__ V vload(const char* p)
{
    return *(const GHX_GLOBAL V*)(p);
}

template<typename V>
__device__ __forceinline__ void vstore(char* p, V v)
{
    *(GHX_GLOBAL V*)(p) = v;
}

// Field-side accesses under the segment's cache policy (seg_s::fpol, uniform per tile; knob
// "short_pol" sets it on short-row segments): bit 0 = non-temporal load, bit 1 = store with sc1
// (gfx950 cache-policy bit; the compiler exposes no builtin for it, hence the asm). Measured
// neutral-to-worse warm; kept for the cold-cache A/Bs.
template<typename V>
__device__ __forceinline__ V fload(const char* p, uint32_t pol)
{
    if (pol & 1u) return __builtin_nontemporal_load((const GHX_GLOBAL V*)(p));
    return vload<V>(p);
}

template<typename V>
__device__ __forceinline__ void fstore(char* p, V v, uint32_t pol)
{
    if constexpr (sizeof(V) == 16)
    {
        if (pol & 2u)
        {
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            return;
        }
    }
    else if constexpr (sizeof(V) == 8)
    {
        if (pol & 2u)
        {
            asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            return;
        }
    }
    else if constexpr (sizeof(V) == 4)
    {
        if (pol & 2u)
        {
            asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
            return;
        }
    }
    vstore<V>(p, v);
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

// The short form (seg_s::amode 1 / 2, planner short_addressing): the offset of buffer position
// p RELATIVE to s.field_off, in 32 bits. Every product has both operands below 2^24 and a result
// below 2^32, so the full-rate v_mul_u32_u24 is exact; the last outer coordinate is the quotient
// itself (rows < ext[0]*ext[1](*ext[2])), so NDIV = n_outer - 1 divisions (at least one).
template<int NDIV>
__device__ __forceinline__ uint32_t field_offset_f(const seg_s& s, uint32_t p)
{
    const uint32_t row = fastdiv(p, s.mag_row);
    uint32_t off = p - __umul24(row, s.row_bytes);
    const uint32_t q0 = fastdiv(row, s.mag_ext[0]);
    off += __umul24(row - __umul24(q0, s.ext[0]), uint32_t(s.stride[0]));
    if constexpr (NDIV == 1)
        off += __umul24(q0, uint32_t(s.stride[1]));
    else
    {
        const uint32_t q1 = fastdiv(q0, s.mag_ext[1]);
        off += __umul24(q0 - __umul24(q1, s.ext[1]), uint32_t(s.stride[1]));
        off += __umul24(q1, uint32_t(s.stride[2]));
    }
    return off;
}

__device__ __forceinline__ int64_t load_lid(const seg_u& s, uint32_t i)
{
    if (s.lid64) return ((const GHX_GLOBAL int64_t*)(s.lids))[i];
    return ((const GHX_GLOBAL int32_t*)(s.lids))[i];
}

template<typename Seg>
__device__ __forceinline__ int64_t field_offset(const Seg& s, uint32_t p);
template<>
__device__ __forceinline__ int64_t field_offset<seg_s>(const seg_s& s, uint32_t p)
{
    return field_offset_s(s, p);
}

// Copy one tile [start, end) of a segment. Lane-linear in buffer space: lanes of a wave touch
// consecutive W-byte vectors of the buffer; kU independent vectors in flight per lane.
// AM: the segment's offset arithmetic (seg_s::amode): 0 general; 1 / 2 the short form, field
// addressed as (field + field_off) + a 32-bit offset.
template<bool PACK, int W, typename Seg, int AM = 0, int kU = ghx::kU>
__device__ __forceinline__ void copy_tile(const Seg& s, char* __restrict__ field,
                                          char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    const uint32_t tid = threadIdx.x;
    const uint32_t pol = s.fpol;
    if constexpr (AM != 0) field += s.field_off;
    for (uint32_t base = start + tid * W; base < end; base += kU * kBlock * W)
    {
        V v[kU];
        using off_t = std::conditional_t<AM == 0, int64_t, uint32_t>;
        off_t fo[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if constexpr (AM == 0)
            {
                if (p < end) fo[u] = field_offset<Seg>(s, p);
            }
            else if (p < end)
                fo[u] = field_offset_f<AM>(s, p);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if (PACK) v[u] = fload<V>(field + fo[u], pol);
                else v[u] = vload<V>(buf + p);
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if (PACK) vstore<V>(buf + p, v[u]);
                else fstore<V>(field + fo[u], v[u], pol);
            }
        }
    }
}

// The unpack of a tile of several steps (unpack plans with long-row tiles above 8 KiB,
// g_tune.unpack_tile_bytes), software-pipelined: each lane issues the buffer loads of step k+1
// before the field stores of step k, so a workgroup keeps its reads in flight while its writes
// drain (the unpack is bound by its writes, §4.4 of DESIGN.md); kP vectors per lane per step.
template<int W, typename Seg>
__device__ __forceinline__ void unpack_tile_pipelined(const Seg& s, char* __restrict__ field,
                                                      char* __restrict__ buf, uint32_t start,
                                                      uint32_t end)
{
    using V = typename vec_t<W>::type;
    constexpr int kP = 2;
    const uint32_t pol = s.fpol;
    const uint32_t step = kP * kBlock * W;
    uint32_t base = start + threadIdx.x * W;
    if (base >= end) return;
    V v[kP];
    int64_t fo[kP];
#pragma unroll
    for (int u = 0; u < kP; ++u)
    {
        const uint32_t p = base + u * kBlock * W;
        if (p < end)
        {
            fo[u] = field_offset<Seg>(s, p);
            v[u] = vload<V>(buf + p);
        }
    }
    for (;;)
    {
        const uint32_t nb = base + step;
        const bool more = nb < end;
        V w[kP];
        int64_t fn[kP];
        if (more)
        {
#pragma unroll
            for (int u = 0; u < kP; ++u)
            {
                const uint32_t p = nb + u * kBlock * W;
                if (p < end)
                {
                    fn[u] = field_offset<Seg>(s, p);
                    w[u] = vload<V>(buf + p);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kP; ++u)
            if (base + u * kBlock * W < end) fstore<V>(field + fo[u], v[u], pol);
        if (!more) break;
        base = nb;
        for (int u = 0; u < kP; ++u)  // register renaming (fully unrolled by the compiler)
        {
            v[u] = w[u];
            fo[u] = fn[u];
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

template<bool PACK, int L>
__device__ __forceinline__ void copy_runs(const seg_u& s, char* __restrict__ field,
                                          char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<16>::type;
    using R = typename vec_t<L>::type;
    constexpr int K = 16 / L;
    const uint32_t pol = s.fpol;
    for (uint32_t base = start + threadIdx.x * 16; base < end; base += kU * kBlock * 16)
    {
        int64_t fo[kU][K];
        uint32_t full = 0, run = 0;  // bit u: chunk u holds K rows / ... that form a run
#pragma unroll
        for (int u = 0; u < kU; ++u)
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
            for (int j = 0; j < K; ++j) fo[u][j] = s.field_off + l[j] * L;  // index stride = L (planner)
        }
        V v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * 16;
            if (p >= end || !(full >> u & 1u)) continue;
            if (PACK)
            {
                if (run >> u & 1u)
                {
                    const v4_a4 x = fload<v4_a4>(field + fo[u][0], pol);
                    v[u] = V{x.x, x.y, x.z, x.w};
                }
                else
                {
                    R w[K];
#pragma unroll
                    for (int j = 0; j < K; ++j) w[j] = fload<R>(field + fo[u][j], pol);
                    v[u] = assemble<L>(w);
                }
            }
            else
                v[u] = vload<V>(buf + p);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
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
                    if (PACK) vstore<R>(buf + p + j * L, fload<R>(field + fo[u][j], pol));
                    else fstore<R>(field + fo[u][j], vload<R>(buf + p + j * L), pol);
                }
                continue;
            }
            if (PACK)
                vstore<V>(buf + p, v[u]);
            else if (run >> u & 1u)
                fstore<v4_a4>(field + fo[u][0], v4_a4{v[u].x, v[u].y, v[u].z, v[u].w}, pol);
            else
            {
                R w[K];
                split<L>(v[u], w);
#pragma unroll
                for (int j = 0; j < K; ++j) fstore<R>(field + fo[u][j], w[j], pol);
            }
        }
    }
}

__device__ __forceinline__ int ptr_wlog2(uint64_t p)
{
    return __builtin_ctzll(p | 16ull);  // log2 of the largest power of two (<= 16) dividing p
}

// Unstructured tile, general path (rows that are not 4/8-B runs, e.g. config 5's 64-B
// levels-first rows): all kU index loads of a lane, then all kU value loads, are issued
// together. Written branch-free per vector: the uniform choices (index width, row mode, cache
// policy) are hoisted out of the per-vector code, and a vector position past the tile's end is
// clamped to the tile's last vector, which moves the same bytes again (a duplicate store of
// identical bytes by another lane of this workgroup). Per-vector branches made the compiler wait
// for each index load before issuing the next (s_waitcnt vmcnt(0) inside every branch): four
// dependent round trips per lane instead of one.
template<bool PACK, int W, int kU>
__device__ __forceinline__ void copy_tile_u(const seg_u& s, char* __restrict__ field,
                                            char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    const uint32_t last = end - W;  // tiles hold whole rows: end - start is a multiple of W
    const uint32_t pol = s.fpol;
    for (uint32_t base = start + threadIdx.x * W; base < end; base += kU * kBlock * W)
    {
        uint32_t p[kU], idx[kU];
        int64_t extra[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) p[u] = min(base + uint32_t(u) * kBlock * W, last);
        V v[kU];
        if (!PACK)
        {
#pragma unroll
            for (int u = 0; u < kU; ++u) v[u] = vload<V>(buf + p[u]);
        }
        if (s.mode == 0)
        {
#pragma unroll
            for (int u = 0; u < kU; ++u)
            {
                const uint32_t row = fastdiv(p[u], s.mag_row);
                idx[u] = row;
                extra[u] = int64_t(p[u] - row * s.row_bytes);
            }
        }
        else if (s.mode == 1)
        {
#pragma unroll
            for (int u = 0; u < kU; ++u)
            {
                const uint32_t row = fastdiv(p[u], s.mag_row);
                const uint32_t i = fastdiv(row, s.mag_inner);
                idx[u] = i;
                extra[u] = int64_t(row - i * s.row_levels) * s.level_stride_b +
                           int64_t(p[u] - row * s.row_bytes);
            }
        }
        else
        {
#pragma unroll
            for (int u = 0; u < kU; ++u)
            {
                const uint32_t row = fastdiv(p[u], s.mag_row);
                const uint32_t l = fastdiv(row, s.mag_inner);
                idx[u] = row - l * s.n;
                extra[u] = int64_t(l) * s.level_stride_b + int64_t(p[u] - row * s.row_bytes);
            }
        }
        int64_t lid[kU];
        if (s.lid64)
        {
#pragma unroll
            for (int u = 0; u < kU; ++u) lid[u] = ((const GHX_GLOBAL int64_t*)(s.lids))[idx[u]];
        }
        else
        {
#pragma unroll
            for (int u = 0; u < kU; ++u) lid[u] = ((const GHX_GLOBAL int32_t*)(s.lids))[idx[u]];
        }
        int64_t fo[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) fo[u] = s.field_off + lid[u] * s.index_stride_b + extra[u];
        if (PACK)
        {
            if (pol & 1u)
            {
#pragma unroll
                for (int u = 0; u < kU; ++u) v[u] = fload<V>(field + fo[u], 1u);
            }
            else
            {
#pragma unroll
                for (int u = 0; u < kU; ++u) v[u] = vload<V>(field + fo[u]);
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) vstore<V>(buf + p[u], v[u]);
        }
        else if (pol & 2u)
        {
#pragma unroll
            for (int u = 0; u < kU; ++u) fstore<V>(field + fo[u], v[u], 2u);
        }
        else
        {
#pragma unroll
            for (int u = 0; u < kU; ++u) vstore<V>(field + fo[u], v[u]);
        }
    }
}

template<bool PACK, int UU>
__device__ __forceinline__ void copy_any(const seg_u& s, char* field, char* buf, uint32_t start,
                                         uint32_t end, int w)
{
    switch (w)
    {
        case 4: copy_tile_u<PACK, 16, UU>(s, field, buf, start, end); break;
        case 3: copy_tile_u<PACK, 8, UU>(s, field, buf, start, end); break;
        case 2: copy_tile_u<PACK, 4, UU>(s, field, buf, start, end); break;
        case 1: copy_tile_u<PACK, 2, UU>(s, field, buf, start, end); break;
        default: copy_tile_u<PACK, 1, UU>(s, field, buf, start, end); break;
    }
}

template<bool PACK, int UU, typename Seg>
__device__ __forceinline__ void copy_any(const Seg& s, char* field, char* buf, uint32_t start,
                                         uint32_t end, int w)
{
    if constexpr (!PACK)
        if (s.pipe && w == 4)  // long rows in tiles of several steps (planner: unpack_tile_bytes)
        {
            unpack_tile_pipelined<16>(s, field, buf, start, end);
            return;
        }
    if constexpr (std::is_same_v<Seg, seg_s>)
    {
        if (s.amode == 1)  // the short form for the widths fp32/fp64 fields give
        {
            switch (w)
            {
                case 4: copy_tile<PACK, 16, Seg, 1, UU>(s, field, buf, start, end); return;
                case 3: copy_tile<PACK, 8, Seg, 1, UU>(s, field, buf, start, end); return;
                case 2: copy_tile<PACK, 4, Seg, 1, UU>(s, field, buf, start, end); return;
                default: break;
            }
        }
        else if (s.amode == 2 && w == 4)
        {
            copy_tile<PACK, 16, Seg, 2>(s, field, buf, start, end);
            return;
        }
    }
    switch (w)
    {
        case 4: copy_tile<PACK, 16>(s, field, buf, start, end); break;
        case 3: copy_tile<PACK, 8>(s, field, buf, start, end); break;
        case 2: copy_tile<PACK, 4>(s, field, buf, start, end); break;
        case 1: copy_tile<PACK, 2>(s, field, buf, start, end); break;
        default: copy_tile<PACK, 1>(s, field, buf, start, end); break;
    }
}

// RUNS (unstructured only): every segment of the plan takes the run path (copy_runs); the host
// (uplan::execute) launches this variant only when runs_ok holds for all of them, so the
// general path's registers do not weigh on it and vice versa.
// DBL (double-buffered buffers, the direct exchange's one-launch epochs): the launch uses, for
// every buffer slot with a second copy, the copy of this exchange's parity, read once per
// workgroup from the epoch counter in device memory (a captured graph alternates on replay).
__device__ __forceinline__ bool odd_parity(const kargs& a)
{
    return ((__hip_atomic_load(a.parity_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
             a.parity_add) & 1) != 0;
}

// REC (tile records, g_tune.tile_records): the workgroup's first load is its own record at
// tile_recs[blockIdx.x] (the segment, with the tile's index in first_tile), so the chain ahead
// of the first data load is one table load instead of tile table -> segment. The grid never
// exceeds n_tiles (grid_for_tiles), so the first tile needs no bound check either.
template<bool PACK, typename Seg, bool RUNS = false, bool DBL = false, int UU = kU, bool REC = false>
__global__ __launch_bounds__(kBlock) void k_copy(kargs a)
{
    const Seg* __restrict__ segs = static_cast<const Seg*>(REC ? a.tile_recs : a.segs);
    bool odd = false;
    if constexpr (DBL) odd = odd_parity(a);
    uint32_t t = blockIdx.x;
    do
    {
        Seg s;
        uint32_t ti;
        if constexpr (REC)
        {
            s = segs[t];
            ti = s.first_tile;
        }
        else
        {
            const uint32_t si = a.tile_seg[2 * t];
            ti = a.tile_seg[2 * t + 1];
            s = segs[si];
        }
        const uint32_t start = ti * s.tile_bytes;
        const uint32_t end = min(start + s.tile_bytes, s.bytes);
        char* field = reinterpret_cast<char*>(a.field_ptr[s.field_slot]);
        char* buf = reinterpret_cast<char*>(a.buf_ptr[s.buf_slot]) + s.buf_off;
        if constexpr (DBL)
            if (odd) buf += a.dbl_off[s.buf_slot];
        if constexpr (RUNS)
        {
            if (s.row_bytes == 8) copy_runs<PACK, 8>(s, field, buf, start, end);
            else copy_runs<PACK, 4>(s, field, buf, start, end);
        }
        else
        {
            int w = s.wlog2;
            w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(field)));
            w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(buf)));
            copy_any<PACK, UU>(s, field, buf, start, end, w);
        }
        t += gridDim.x;
    } while (t < a.n_tiles);
}

// Lane-local self tile with store-to-load forwarding: the unpack half needs exactly the buffer
// bytes this lane has just stored (same positions, same width), so it takes them from the
// registers instead of loading them back: field interior -> register -> buffer store AND halo
// store. Every buffer byte and every halo byte is still written; what disappears is the
// buffer read-back (which a lane-local read-back served from L2, or, for ~20 % of it, from HBM:
// TCC_EA0_RDREQ 573k against 461k for the field reads alone).
// AM: 0 general; 1 both segments in the short form with one division (copy_tile's AM 1).
template<int W, int AM = 0>
__device__ __forceinline__ void self_forward(const seg_s& s, const seg_s& q,
                                             char* __restrict__ fp, char* __restrict__ fu,
                                             char* __restrict__ buf, uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    using off_t = std::conditional_t<AM == 0, int64_t, uint32_t>;
    const uint32_t pol_p = s.fpol, pol_u = q.fpol;
    if constexpr (AM != 0)
    {
        fp += s.field_off;
        fu += q.field_off;
    }
    for (uint32_t base = start + threadIdx.x * W; base < end; base += kU * kBlock * W)
    {
        V v[kU];
        off_t op[kU], ou[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if constexpr (AM == 0)
                {
                    op[u] = field_offset_s(s, p);
                    ou[u] = field_offset_s(q, p);
                }
                else
                {
                    op[u] = field_offset_f<AM>(s, p);
                    ou[u] = field_offset_f<AM>(q, p);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end) v[u] = fload<V>(fp + op[u], pol_p);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                vstore<V>(buf + p, v[u]);
                fstore<V>(fu + ou[u], v[u], pol_u);
            }
        }
    }
}

// Fused self exchange: every message is a self message, so pack segment k and unpack segment k
// cover the same buffer bytes with the same tiling. When both halves of a tile use the same
// vector width (always, for aligned fields) every lane unpacks exactly the bytes it packed:
// it writes the halo from the registers it stored the buffer from (self_forward), no barrier.
// Otherwise the workgroup packs its tile (field interior -> buffer), passes a workgroup barrier
// (its own stores are visible to its own waves), then unpacks the same bytes (buffer -> halo).
// REC: pair records (upload_pair_records) — the workgroup loads its tile's pack and unpack
// segments side by side at tile_recs[2 * blockIdx.x], no tile-table load ahead of them.
template<bool DBL = false, bool REC = false>
__global__ __launch_bounds__(kBlock) void k_self(kargs a)
{
    const seg_s* __restrict__ ps = static_cast<const seg_s*>(a.segs);
    const seg_s* __restrict__ us = static_cast<const seg_s*>(a.segs2);
    const seg_s* __restrict__ rec = static_cast<const seg_s*>(a.tile_recs);
    bool odd = false;
    if constexpr (DBL) odd = odd_parity(a);
    for (uint32_t t = blockIdx.x; t < a.n_tiles; t += gridDim.x)
    {
        seg_s s, q;
        uint32_t ti;
        if constexpr (REC)
        {
            s = rec[2 * t];
            q = rec[2 * t + 1];
            ti = s.first_tile;
        }
        else
        {
            const uint32_t si = a.tile_seg[2 * t];
            ti = a.tile_seg[2 * t + 1];
            s = ps[si];
            q = us[si];
        }
        const uint32_t start = ti * s.tile_bytes;
        const uint32_t end = min(start + s.tile_bytes, s.bytes);
        char* field_p = reinterpret_cast<char*>(a.field_ptr[s.field_slot]);
        char* field_u = reinterpret_cast<char*>(a.field_ptr[q.field_slot]);
        char* buf = reinterpret_cast<char*>(a.buf_ptr[s.buf_slot]) + s.buf_off;
        if constexpr (DBL)
            if (odd) buf += a.dbl_off[s.buf_slot];
        int wp = min(int(s.wlog2), ptr_wlog2(reinterpret_cast<uint64_t>(field_p)));
        wp = min(wp, ptr_wlog2(reinterpret_cast<uint64_t>(buf)));
        int wu = min(int(q.wlog2), ptr_wlog2(reinterpret_cast<uint64_t>(field_u)));
        wu = min(wu, ptr_wlog2(reinterpret_cast<uint64_t>(buf)));
        if (q.bytes == 0)
        {
            // a peer message of a mixed exchange (ghx_exchange_pack_self): pack only
            copy_any<true, kU>(s, field_p, buf, start, end, wp);
            continue;
        }
        if (wp == wu && s.amode == 1 && q.amode == 1 && wp >= 3)
        {
            if (wp == 4) self_forward<16, 1>(s, q, field_p, field_u, buf, start, end);
            else self_forward<8, 1>(s, q, field_p, field_u, buf, start, end);
            continue;
        }
        if (wp == wu)
        {
            switch (wp)
            {
                case 4: self_forward<16>(s, q, field_p, field_u, buf, start, end); break;
                case 3: self_forward<8>(s, q, field_p, field_u, buf, start, end); break;
                case 2: self_forward<4>(s, q, field_p, field_u, buf, start, end); break;
                case 1: self_forward<2>(s, q, field_p, field_u, buf, start, end); break;
                default: self_forward<1>(s, q, field_p, field_u, buf, start, end); break;
            }
            continue;
        }
        copy_any<true, kU>(s, field_p, buf, start, end, wp);
        __syncthreads();  // workgroup release/acquire: the tile's buffer bytes are complete
        copy_any<false, kU>(q, field_u, buf, start, end, wu);
        __syncthreads();  // the next tile of a grid-stride loop reuses the lanes
    }
}

// Zero-copy put: element p of the virtual message is read from the source field through the
// pack segment's addressing and written to the target field (peer memory or local) through the
// unpack segment's addressing, register to register — no buffer.
template<int W, int AM = 0>
__device__ __forceinline__ void copy_direct(const seg_s& s, const seg_s& q,
                                            const char* __restrict__ src, char* __restrict__ dst,
                                            uint32_t start, uint32_t end)
{
    using V = typename vec_t<W>::type;
    using off_t = std::conditional_t<AM == 0, int64_t, uint32_t>;
    if constexpr (AM != 0)
    {
        src += s.field_off;
        dst += q.field_off;
    }
    for (uint32_t base = start + threadIdx.x * W; base < end; base += kU * kBlock * W)
    {
        V v[kU];
        off_t fd[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end)
            {
                if constexpr (AM == 0)
                {
                    v[u] = vload<V>(src + field_offset_s(s, p));
                    fd[u] = field_offset_s(q, p);
                }
                else
                {
                    v[u] = vload<V>(src + field_offset_f<AM>(s, p));
                    fd[u] = field_offset_f<AM>(q, p);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
        {
            const uint32_t p = base + u * kBlock * W;
            if (p < end) vstore<V>(dst + fd[u], v[u]);
        }
    }
}

template<bool REC = false>
__global__ __launch_bounds__(kBlock) void k_put(kargs a)
{
    const seg_s* __restrict__ ps = static_cast<const seg_s*>(a.segs);
    const seg_s* __restrict__ qs = static_cast<const seg_s*>(a.segs2);
    const seg_s* __restrict__ rec = static_cast<const seg_s*>(a.tile_recs);
    for (uint32_t t = blockIdx.x; t < a.n_tiles; t += gridDim.x)
    {
        seg_s s, q;
        uint32_t ti;
        if constexpr (REC)
        {
            s = rec[2 * t];
            q = rec[2 * t + 1];
            ti = s.first_tile;
        }
        else
        {
            const uint32_t si = a.tile_seg[2 * t];
            ti = a.tile_seg[2 * t + 1];
            s = ps[si];
            q = qs[si];
        }
        const uint32_t start = ti * s.tile_bytes;
        const uint32_t end = min(start + s.tile_bytes, s.bytes);
        const char* src = reinterpret_cast<const char*>(a.field_ptr[s.field_slot]);
        char* dst = reinterpret_cast<char*>(a.buf_ptr[q.field_slot]);
        int w = min(int(s.wlog2), int(q.wlog2));
        w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(src)));
        w = min(w, ptr_wlog2(reinterpret_cast<uint64_t>(dst)));
        if (s.amode == 1 && q.amode == 1 && w >= 3)
        {
            if (w == 4) copy_direct<16, 1>(s, q, src, dst, start, end);
            else copy_direct<8, 1>(s, q, src, dst, start, end);
            continue;
        }
        switch (w)
        {
            case 4: copy_direct<16>(s, q, src, dst, start, end); break;
            case 3: copy_direct<8>(s, q, src, dst, start, end); break;
            case 2: copy_direct<4>(s, q, src, dst, start, end); break;
            case 1: copy_direct<2>(s, q, src, dst, start, end); break;
            default: copy_direct<1>(s, q, src, dst, start, end); break;
        }
    }
}

int launched(const char* what)
{
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
    {
        set_error(std::string(what) + " kernel launch failed: " + hipGetErrorString(e));
        return GHX_ERR_HIP;
    }
    return GHX_OK;
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

template<bool REC>
void launch_s(const kargs& a, int direction, hipStream_t s, uint32_t grid)
{
    if (a.parity_word)
    {
        if (direction == 0) launch((k_copy<true, seg_s, false, true, kU, REC>), grid, s, a);
        else launch((k_copy<false, seg_s, false, true, kU, REC>), grid, s, a);
    }
    else if (direction == 0) launch((k_copy<true, seg_s, false, false, kU, REC>), grid, s, a);
    else launch((k_copy<false, seg_s, false, false, kU, REC>), grid, s, a);
}

int launch_structured(const kargs& a, int direction, void* stream, uint32_t grid)
{
    if (a.n_tiles == 0) return GHX_OK;
    grid = min(grid, a.n_tiles);  // k_copy's first tile is unchecked: never more groups than tiles
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (a.tile_recs) launch_s<true>(a, direction, s, grid);
    else launch_s<false>(a, direction, s, grid);
    return launched("structured");
}

int launch_self(const kargs& a, void* stream, uint32_t grid)
{
    if (a.n_tiles == 0) return GHX_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (a.parity_word)
    {
        if (a.tile_recs) launch((k_self<true, true>), grid, s, a);
        else launch((k_self<true, false>), grid, s, a);
    }
    else if (a.tile_recs) launch((k_self<false, true>), grid, s, a);
    else launch((k_self<false, false>), grid, s, a);
    return launched("self-exchange");
}

int launch_put(const kargs& a, void* stream, uint32_t grid)
{
    if (a.n_tiles == 0) return GHX_OK;
    if (a.tile_recs) launch(k_put<true>, grid, static_cast<hipStream_t>(stream), a);
    else launch(k_put<false>, grid, static_cast<hipStream_t>(stream), a);
    return launched("put");
}

template<bool DBL, bool REC>
void launch_u(const kargs& a, int direction, hipStream_t s, uint32_t grid, bool runs)
{
    if (runs && direction == 0) launch((k_copy<true, seg_u, true, DBL, kU, REC>), grid, s, a);
    else if (runs) launch((k_copy<false, seg_u, true, DBL, kU, REC>), grid, s, a);
    else if (direction == 0) launch((k_copy<true, seg_u, false, DBL, kU, REC>), grid, s, a);
    else launch((k_copy<false, seg_u, false, DBL, kU, REC>), grid, s, a);
}

int launch_unstructured(const kargs& a, int direction, void* stream, uint32_t grid, bool runs)
{
    if (a.n_tiles == 0) return GHX_OK;
    grid = min(grid, a.n_tiles);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (a.parity_word)
    {
        if (a.tile_recs) launch_u<true, true>(a, direction, s, grid, runs);
        else launch_u<true, false>(a, direction, s, grid, runs);
    }
    else if (a.tile_recs) launch_u<false, true>(a, direction, s, grid, runs);
    else launch_u<false, false>(a, direction, s, grid, runs);
    return launched("unstructured");
}

}  // namespace ghx
