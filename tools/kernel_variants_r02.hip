// kernel_variants_r02.hip — device code REMOVED from the product kernel (ghex_amd/csrc/
// ghx_kernels.hip) in round 3, kept here as the record behind the round-2 A/B measurements.
// NOT compiled or linked by anything; it refers to the product's types (seg_s, kargs, vload,
// vstore, field_offset_s, kBlock) as they were at commit d116055, where it last built and ran.
//
// Every variant measured slower than the default (direct k_copy, register-forwarded k_self):
//   copy_tile_pair / dispatch_pair / try_pair  knob "pair" = 1: one lane moves both pieces of a
//       shared 128-B line — 40.4 us step vs 33.2-33.6 (profiles/r02_pack_unpack_ab.jsonl)
//   copy_tile_ilv  knob "pair" = 2: the two pieces on adjacent lanes of one instruction —
//       38.5-38.7 us step (35.0 with 2048-row tiles)
//   copy_tile_lds  knob "lds": the north star's LDS-staged stride->linear transpose of 8/16-B
//       rows — pack 20.1 -> 38.7 us (profiles/r02_lds_ab.jsonl)
//   self_pipelined  knob "self_pipe": software-pipelined fused self tiles — H=2 within noise,
//       H=1 +3 %, H=3 +12 %
// Also removed with them (host side): the chunked self tile ("self_chunk": 4 KiB 34.8 us, no
// faster), non-temporal policies "nt" 1-3 / "nt_dir" (nt=3 54.7 us step), the XCD placement
// knobs "short_xcds" (X=7..1: 43.5-110.9 us step, profiles/r02_short_xcds_ab.jsonl) and
// "xcd_rotate" (step unchanged, profiles/r02_l2_channels.jsonl), dispatch orders 2-4
// (36.6-46.0 us), "unroll" 2/8 and the ascending-index visit order "usort" (500 -> 337 GB/s).

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
