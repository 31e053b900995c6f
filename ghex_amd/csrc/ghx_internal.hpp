// ghx_internal.hpp — structures shared by the host planner and the gfx950 kernels.
//
// Data layout in HBM: a plan is a flat table of segments (one per field x
// iteration space) plus a tile table (uint32 segment index per workgroup tile). A segment is a
// set of equal-length contiguous byte runs ("rows") of the field that map, in order, onto ONE
// contiguous byte range of the buffer — the dense buffer box of make_buffer_desc
// (include/ghex/structured/regular/field_descriptor.hpp:114-129) is row-major in the field's
// layout order, so row r occupies buffer bytes [r*L, (r+1)*L). Rows are decoded from the
// buffer byte position by magic-number division (no hardware divide on the hot path).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ghx.h"

namespace ghx
{
// Bytes of buffer covered by one workgroup tile (default 256 threads x 4 vectors x 16 B); the
// tile size is a plan-time tuning knob bounded by kMaxTileBytes.
constexpr uint32_t kTileBytes = 8192;
constexpr uint32_t kMaxTileBytes = 1u << 20;
constexpr int kBlock = 256;

// Launch / planning knobs (ghx_tune). Defaults are the measured best. The knobs
// whose every setting but the default lost its A/B were removed in round 3
// (tools/kernel_variants_r02.hip lists them with their numbers).
struct tuning
{
    int grid_cap = 0;               // >0: at most this many workgroups (grid-stride beyond)
    uint32_t tile_bytes = kTileBytes;  // tile of segments with long rows
    uint32_t unpack_tile_bytes = 0;    // the same for unpack plans (0: tile_bytes); above 8 KiB
                                       // the unpack kernel pipelines a tile's steps
    uint32_t self_tile_bytes = kTileBytes;  // the same for the fused self exchange (separate
                                       // self plans are built when it differs). Medians of 4
                                       // interleaved A/B runs with register forwarding:
                                       // H=2 8 KiB 26.4 vs 4 KiB 27.9 us; H=1 18.6 vs 19.9;
                                       // H=3 32.8 vs 32.0 (profiles/r01c_fwd_tile_ab.jsonl)
    uint32_t small_tile_rows = 0;      // rows per tile of segments with short rows (0: by the
                                       // plan's short-row count, ghx_plan.cpp short_tile_rows)
    uint32_t pack_tile_rows = 0;       // rows per short-row tile of PACK plans only (0: as
                                       // small_tile_rows / the plan's rule)
    uint32_t unpack_tile_rows = 0;     // the same for UNPACK plans
    uint32_t small_row_bytes = 64;     // rows shorter than this are "short" (request-bound)
    uint32_t u_tile_rows = 512;        // rows per tile of short-row unstructured segments
    uint32_t u_tile_bytes = 16384;     // tile of unstructured segments with long rows (config 5's
                                       // 64-B levels-first rows: scatter 16.8 -> 14.0 us against
                                       // 8 KiB, tools/u_tile_sweep.py, profiles/r05_u_tile_sweep*)
    int order = 1;                     // tile dispatch order: 0 segment order, 1 short-row
                                       // segments first (2-4 lost: tools/kernel_variants_r02.hip)
    int urun = 1;                      // unstructured 4/8-B-row segments: 16-B lane chunks with
                                       // run detection (copy_runs)
    uint32_t u_run_tile_rows = 2048;   // rows per tile of run-heavy index-list segments
    int short_pol = 0;                 // field-side cache policy of short-row segments:
                                       // bit 0 non-temporal loads (pack), bit 1 sc1 stores
                                       // (unpack)
    int xcd_pair = 1;                  // dispatch the tiles of line-sharing short-row segment
                                       // pairs in lock-step groups of 8, so tile t of both
                                       // halves lands on the same XCD (blocks are dealt
                                       // round-robin over the 8 XCDs) at the same time
    int mixed_always = 0;              // build the mixed self/peer plans even when the self
                                       // messages hold no short rows (tests, measurements)
    int tile_records = 1;              // k_copy reads per tile ONE record (its segment with the
                                       // tile index in first_tile) at blockIdx: no dependent
                                       // tile-table load ahead of the segment load
    int fast_addr = 1;                 // structured segments whose offsets fit the short form
                                       // (seg_s::amode) decode rows with 1-2 divisions and
                                       // full-rate 24-bit products instead of int64 ones
};
extern tuning g_tune;

// Unsigned 32-bit division by an invariant d via multiply-high (Granlund-Montgomery; the
// round-up variant valid for every n < 2^32): q = (t + ((n - t) >> s1)) >> s2, t = mulhi(m, n).
struct magic_u32
{
    uint32_t m;
    uint8_t s1, s2;
    uint16_t pad;
};

inline magic_u32 make_magic(uint32_t d)
{
    magic_u32 r{};
    if (d == 0) d = 1;
    int l = 0;
    while ((uint64_t(1) << l) < d) ++l;  // l = ceil(log2 d)
    uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1;
    r.m = uint32_t(m);
    r.s1 = uint8_t(l < 1 ? l : 1);
    r.s2 = uint8_t(l > 1 ? l - 1 : 0);
    return r;
}

// Structured segment (128 B, read once per workgroup tile with scalar loads).
struct alignas(16) seg_s
{
    int64_t field_off;    // byte offset (from the field base) of the segment's first row
    uint64_t buf_off;     // byte offset (from the buffer base) of the segment's first byte
    int64_t stride[4];    // field byte stride of outer dim k (k = 0 varies fastest over rows)
    uint32_t ext[4];      // outer extents (1 for unused dims)
    magic_u32 mag_row;    // division by row_bytes
    magic_u32 mag_ext[3]; // division by ext[0], ext[1], ext[2]
    uint32_t row_bytes;   // L: bytes per contiguous run
    uint32_t bytes;       // rows * L
    uint32_t first_tile;  // 0 in a segment table; in a tile record, the tile's index in its
                          // segment
    uint16_t field_slot;
    uint16_t buf_slot;
    uint8_t wlog2;        // log2 of the widest vector (<= 16 B) that divides L, offsets, strides
    uint8_t n_outer;
    uint8_t fpol;         // field-side cache policy: bit 0 nt loads, bit 1 sc1 stores
    uint8_t pipe;         // unpack of long rows in tiles of several steps: software-pipelined
    uint32_t tile_bytes;  // this segment's tile size (a multiple of the row length or 16 KiB)
    uint8_t amode;        // field-offset arithmetic (planner, set_amode): 0 general (int64, 3
                          // divisions), 1 / 2: 32-bit offsets relative to field_off from 24-bit
                          // products, 1 / 2 divisions (n_outer <= 2 / == 3), see field_offset_f
    uint8_t pad[7];
};
static_assert(sizeof(seg_s) == 128, "seg_s layout");

// Unstructured segment: rows come from an index list.
struct alignas(16) seg_u
{
    uint64_t buf_off;
    const void* lids;          // device array, int32 or int64
    int64_t index_stride_b;    // bytes
    int64_t level_stride_b;    // bytes
    magic_u32 mag_row;         // division by row_bytes
    magic_u32 mag_inner;       // levels_first: division by levels_per_row-group; else by n
    uint32_t n;                // number of indices
    uint32_t row_levels;       // levels per row group when rows are per (i,l); see planner
    uint32_t row_bytes;
    uint32_t bytes;
    uint32_t first_tile;
    uint16_t field_slot;
    uint16_t buf_slot;
    uint8_t wlog2;
    uint8_t mode;              // 0: row = index i (levels contiguous, L = levels*elem)
                               // 1: rows (i,l) i-major (levels_first, strided levels)
                               // 2: rows (l,i) l-major (levels_last)
    uint8_t lid64;
    uint8_t fpol;              // field-side cache policy (as seg_s)
    uint32_t tile_bytes;
    int64_t field_off;         // added to every field offset (a level of a split levels-last list)
    uint8_t runs;              // mode 0, rows of 4 or 8 B, rows of consecutive lids contiguous
                               // in the field: lanes move 16-B chunks (16/L rows), one 16-B
                               // field access where the chunk's lids form a run (copy_runs);
                               // 2: at least half the chunks are runs (u_run_tile_rows tiles)
    uint8_t pad2[7];
};
static_assert(sizeof(seg_u) == 96, "seg_u layout");

// Kernel arguments (passed by value: <= 1.7 KB of kernarg).
struct kargs
{
    const void* segs;
    const void* segs2;         // fused self exchange: the unpack segments (1:1 with segs)
    const uint32_t* tile_seg;  // per tile: {segment index, tile index within the segment}
    const void* tile_recs;     // or per tile one record (k_copy; null: use segs + tile_seg)
    uint32_t n_tiles;
    uint32_t parity_add;       // double-buffered launches: parity = (*parity_word + add) & 1
    const uint64_t* parity_word;  // null: single-buffered (the kernels' plain variants)
    uint64_t field_ptr[GHX_MAX_SLOTS];
    uint64_t buf_ptr[GHX_MAX_SLOTS];
    int64_t dbl_off[GHX_MAX_SLOTS];  // per buffer slot: byte offset of its odd-parity copy (0: none)
};

// Double-buffered buffers (the direct exchange's one-launch epochs, ghx_epochs.hip): a buffer
// exists twice, its odd-parity copy `offset` bytes after the even one, and a launch uses the copy
// of the exchange's parity, read on the device from the epoch counter (so that a captured graph
// alternates on replay). Per caller buffer index: the offset (0 = one copy only).
struct parity_cfg
{
    const uint64_t* word = nullptr;
    uint32_t add = 0;
    std::vector<int64_t> offset;
    // fill a launch's parity fields; map: local slot -> caller buffer index (empty: identity)
    void apply(kargs& a, const std::vector<int32_t>& map, int n_identity) const
    {
        if (!word) return;
        a.parity_word = word;
        a.parity_add = add;
        const int n = map.empty() ? n_identity : int(map.size());
        for (int i = 0; i < n; ++i)
        {
            const size_t c = size_t(map.empty() ? i : map[size_t(i)]);
            a.dbl_off[i] = c < offset.size() ? offset[c] : 0;
        }
    }
};

// thread-local last error
void set_error(const std::string& msg);
const char* get_error();

// kernel launchers (ghx_kernels.hip)
int launch_structured(const kargs& a, int direction, void* stream, uint32_t grid);
int launch_unstructured(const kargs& a, int direction, void* stream, uint32_t grid, bool runs);
int launch_self(const kargs& a, void* stream, uint32_t grid);
int launch_put(const kargs& a, void* stream, uint32_t grid);
uint32_t grid_for_tiles(uint32_t n_tiles);
void timing_enable(bool on);                            // ghx_launch_timing
int timing_read(float* ms, int32_t cap, int32_t* n);    // ghx_launch_timing_read

}  // namespace ghx
