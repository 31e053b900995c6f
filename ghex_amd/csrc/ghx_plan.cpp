// ghx_plan.cpp — host-side planner: iteration spaces -> device segment + tile tables.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "ghx_plan.hpp"

namespace ghx
{
namespace
{
int ctz64(uint64_t v) { return v ? __builtin_ctzll(v) : 64; }

int wlog2_of(uint64_t v)  // log2 of the largest power of two <= 16 dividing v
{
    return std::min(4, ctz64(v));
}

uint32_t tiles_of(uint32_t bytes, uint32_t tb) { return (bytes + tb - 1) / tb; }

// Short-row segments of one field whose rows interleave in memory: row r of `a` and row r-1 of
// `b` share a 128-B line (0 < a.field_off + a.stride[0] - b.field_off < 128, the pieces disjoint).
// For a unit-stride field these are the two x-normal faces (and x-edges) of a halo: the -x piece
// of row y+1 sits right after the +x piece of row y. Returns partner[i] (or -1), symmetric.
std::vector<int32_t> line_partners(const std::vector<seg_s>& segs)
{
    std::vector<int32_t> partner(segs.size(), -1);
    for (size_t i = 0; i < segs.size(); ++i)
    {
        const auto& a = segs[i];
        if (partner[i] >= 0 || a.row_bytes >= g_tune.small_row_bytes ||
            a.n_outer < 1 || a.bytes / a.row_bytes < 2)
            continue;
        for (size_t j = 0; j < segs.size(); ++j)
        {
            if (j == i || partner[j] >= 0) continue;
            const auto& b = segs[j];
            bool same = b.field_slot == a.field_slot && b.row_bytes == a.row_bytes &&
                        b.n_outer == a.n_outer && b.bytes == a.bytes;
            for (int k = 0; same && k < 4; ++k)
                same = b.ext[k] == a.ext[k] && b.stride[k] == a.stride[k];
            if (!same) continue;
            const int64_t d = a.field_off + a.stride[0] - b.field_off;
            if (d <= 0 || d >= 128 || d < int64_t(a.row_bytes)) continue;
            partner[i] = int32_t(j);
            partner[j] = int32_t(i);
            break;
        }
    }
    return partner;
}

std::vector<int32_t> line_partners(const std::vector<seg_u>& segs)
{
    return std::vector<int32_t>(segs.size(), -1);
}

// Rows per tile of a short-row segment. Structured short rows (x-normal faces, edges, corners
// of a unit-stride field) are request-bound: a plan's R short rows are cut so that they make
// about R/128 tiles when each row is one 16-B lane access (16-B rows: H=2 fp64), R/256 otherwise,
// a power of two in [512, 4096] (knob small_tile_rows > 0 overrides). Measured with the
// graph-timed two-launch step over N = 256..640 and H = 1..3 (profiles/r03_tile_rows_sweep.jsonl,
// DESIGN §4): a fixed 4096 rows — the round-1 choice, made at 512^3 H=2 where it still wins — left
// small cubes with a few dozen x-face workgroups (256^3 H=3: 35.4 us vs 14.9 us at 1024 rows) and
// was 15-17 % slower at 512^3 H=1/H=3 than 2048 rows. Index-list gathers are latency-bound
// random accesses and want many workgroups in flight (512 rows), except run-heavy lists on the
// run path, which stream (2048 rows: tools/urun_bench.py, contiguous lids 40 -> 33 us).
// Pack plans whose short rows take several vector accesses each (24-B rows of fp64 at H=3, 12-B
// rows of fp32) cut four times finer (round 6): the pack at 384^3 / 512^3 / 640^3 H=3 takes 12.6 ->
// 11.5 / 19.7 -> 18.5 / 34.3 -> 31.8-33.9 us with 512-row tiles against the old rule's 1024-2048
// rows, 256^3 H=3 equal; single-access rows (H=1, H=2 fp64) keep the old rule, which wins there
// (interleaved A/B, profiles/r06an_pack_tile_rows_ab.jsonl; sweep r06am_pack_tile_rows_sweep.jsonl).
uint32_t short_tile_rows(const seg_s& s, uint64_t short_rows, int dir)
{
    if (dir == 0 && g_tune.pack_tile_rows) return g_tune.pack_tile_rows;
    if (dir == 1 && g_tune.unpack_tile_rows) return g_tune.unpack_tile_rows;
    if (g_tune.small_tile_rows) return g_tune.small_tile_rows;
    // several vector accesses per row (whatever the pointers' alignment allows)
    const bool multi = s.row_bytes > 16 || (s.row_bytes & (s.row_bytes - 1)) != 0;
    const uint64_t want = short_rows / (dir == 0 && multi ? 1024 : s.row_bytes == 16 ? 128 : 256);
    uint32_t r = 512;
    while (r < 4096 && uint64_t(r) * 2 <= want) r *= 2;
    return r;
}
uint32_t short_tile_rows(const seg_u& s, uint64_t, int)
{
    return s.runs == 2 ? g_tune.u_run_tile_rows : g_tune.u_tile_rows;
}
// tile of segments with long rows: structured / unstructured
uint32_t long_tile_bytes(const seg_s&, int dir)
{
    return dir == 1 && g_tune.unpack_tile_bytes ? g_tune.unpack_tile_bytes : g_tune.tile_bytes;
}
uint32_t long_tile_bytes(const seg_u& s, int)
{
    // whole rows per tile (at least one)
    const uint32_t tb = std::max<uint32_t>(g_tune.u_tile_bytes, s.row_bytes);
    return tb - tb % s.row_bytes;
}

// The short form of a segment's field-offset arithmetic (seg_s::amode, field_offset_f in
// ghx_kernels.hip): a row's offset RELATIVE to field_off is computed in 32 bits from full-rate
// 24-bit products (v_mul_u32_u24) with one division per outer dim beyond the last, instead of
// the general form's three divisions and four int64 products (about 16 quarter-rate
// multiplies per vector, the launch's VALU time at small shapes). Exact when every operand of a
// product is below 2^24 and the relative offsets below 2^32: rows, row length, the decoded outer
// extents and the strides (non-negative) of the outer dims in use.
uint8_t short_addressing(const seg_s& s)
{
    if (!g_tune.fast_addr || s.n_outer > 3) return 0;
    constexpr uint64_t k24 = uint64_t(1) << 24;
    const uint64_t rows = s.row_bytes ? s.bytes / s.row_bytes : 0;
    if (rows >= k24 || s.row_bytes >= k24) return 0;
    uint64_t span = s.row_bytes;
    for (int k = 0; k < s.n_outer; ++k)
    {
        if (s.stride[k] < 0 || uint64_t(s.stride[k]) >= k24 || s.ext[k] >= k24) return 0;
        span += uint64_t(s.ext[k] - 1) * uint64_t(s.stride[k]);
    }
    if (span >= (uint64_t(1) << 32)) return 0;
    return s.n_outer == 3 ? 2 : 1;
}

void set_pipe(seg_s& s, bool on) { s.pipe = on ? 1 : 0; }
void set_pipe(seg_u&, bool) {}

// Tile table: per tile {segment, tile index within the segment}. Segments with short rows
// (request-bound: one memory request per row) may use a different tile size from streaming
// segments; the dispatch order of tiles is a tuning knob (hardware dispatches in blockIdx order).
template<typename Seg>
std::vector<uint32_t> build_tiles(std::vector<Seg>& segs, int dir)
{
    std::vector<std::vector<uint32_t>> per(segs.size());
    // each field's short rows (its request-bound work): a field's short-row tiles are sized by
    // its own rows, not the plan's, so a plan of several fields keeps each field's tiling
    // (config 4, five 256^3 fields at H=3: 2048-row tiles by the plan's 686k short rows vs 512
    // by each field's 137k, pack 23.7 -> 21.4 us, profiles/r05_config4_sweep.jsonl)
    std::map<int32_t, uint64_t> short_rows;
    for (const auto& sg : segs)
        if (sg.row_bytes < g_tune.small_row_bytes) short_rows[sg.field_slot] += sg.bytes / sg.row_bytes;
    for (uint32_t i = 0; i < segs.size(); ++i)
    {
        const bool small = segs[i].row_bytes < g_tune.small_row_bytes;
        uint32_t tb = long_tile_bytes(segs[i], dir);
        if (small)
        {
            const uint32_t rows = short_tile_rows(segs[i], short_rows[segs[i].field_slot], dir);
            const uint64_t want = uint64_t(rows) * segs[i].row_bytes;
            tb = uint32_t(std::max<uint64_t>(segs[i].row_bytes, std::min<uint64_t>(want, kMaxTileBytes)));
            tb -= tb % segs[i].row_bytes;  // whole rows per tile
        }
        segs[i].tile_bytes = tb;
        segs[i].fpol = small ? uint8_t(g_tune.short_pol) : uint8_t(0);
        set_pipe(segs[i], !small && dir == 1 && g_tune.unpack_tile_bytes > kTileBytes);
        segs[i].first_tile = 0;
        const uint32_t nt = tiles_of(segs[i].bytes, tb);
        for (uint32_t t = 0; t < nt; ++t) per[i].push_back(t);
    }
    std::vector<uint32_t> out;
    auto emit = [&](uint32_t i, uint32_t t) {
        out.push_back(i);
        out.push_back(t);
    };
    std::vector<uint32_t> idx(segs.size());
    for (uint32_t i = 0; i < segs.size(); ++i) idx[i] = i;
    if (g_tune.order == 1)
        std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
            return (segs[a].row_bytes < g_tune.small_row_bytes) >
                   (segs[b].row_bytes < g_tune.small_row_bytes);
        });
    std::vector<int32_t> partner(segs.size(), -1);
    if (g_tune.order == 1 && g_tune.xcd_pair) partner = line_partners(segs);
    // Line-sharing pairs first, in lock-step groups of 8 tiles: tile t of one half at block
    // 16k + i, tile t of the other at 16k + 8 + i -> the same XCD (blocks are dealt
    // round-robin over the 8 XCDs) at about the same time, so each shared line is fetched
    // once into that XCD's L2 and both halves' partial writes merge there. A short group is
    // padded with tiles of the other segments so the alignment holds.
    std::vector<std::pair<uint32_t, uint32_t>> rest;
    for (uint32_t i : idx)
        if (partner[i] < 0)
            for (uint32_t t : per[i]) rest.emplace_back(i, t);
    size_t next = 0;
    for (uint32_t i : idx)
    {
        const int32_t j = partner[i];
        if (j < 0 || uint32_t(j) < i) continue;
        const size_t n = per[i].size();  // == per[j].size(): partners have equal bytes
        for (size_t k = 0; k < n; k += 8)
        {
            const size_t m = std::min<size_t>(8, n - k);
            for (size_t u = 0; u < m; ++u) emit(uint32_t(j), per[size_t(j)][k + u]);
            for (size_t u = m; u < 8 && next < rest.size(); ++u, ++next)
                emit(rest[next].first, rest[next].second);
            for (size_t u = 0; u < m; ++u) emit(i, per[i][k + u]);
        }
    }
    for (; next < rest.size(); ++next) emit(rest[next].first, rest[next].second);
    return out;
}

bool have_device()
{
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

// Upload a plan's host tables to device memory (synchronous: plan creation is setup time).
// Without a HIP device (the CPU build container) the plan stays host-only: its metadata can be
// inspected, executing it reports GHX_ERR_HIP.
template<typename Seg>
void upload(device_tables& dt, const std::vector<Seg>& segs, const std::vector<uint32_t>& tiles)
{
    dt.release();
    if (segs.empty() || !have_device()) return;
    const size_t sb = segs.size() * sizeof(Seg), tb = tiles.size() * sizeof(uint32_t);
    if (hipMalloc(&dt.segs, sb) != hipSuccess) throw hip_error("hipMalloc(segments)");
    if (hipMalloc(reinterpret_cast<void**>(&dt.tiles), tb) != hipSuccess)
        throw hip_error("hipMalloc(tiles)");
    if (hipMemcpy(dt.segs, segs.data(), sb, hipMemcpyHostToDevice) != hipSuccess)
        throw hip_error("hipMemcpy(segments)");
    if (hipMemcpy(dt.tiles, tiles.data(), tb, hipMemcpyHostToDevice) != hipSuccess)
        throw hip_error("hipMemcpy(tiles)");
    if (g_tune.tile_records && !tiles.empty())
    {
        // one record per tile, in dispatch order: the tile's segment with first_tile = the
        // tile's index in it (a workgroup loads its record from blockIdx alone)
        std::vector<Seg> rec(tiles.size() / 2);
        for (size_t t = 0; t < rec.size(); ++t)
        {
            rec[t] = segs[tiles[2 * t]];
            rec[t].first_tile = tiles[2 * t + 1];
        }
        const size_t rb = rec.size() * sizeof(Seg);
        if (hipMalloc(&dt.recs, rb) != hipSuccess) throw hip_error("hipMalloc(tile records)");
        if (hipMemcpy(dt.recs, rec.data(), rb, hipMemcpyHostToDevice) != hipSuccess)
            throw hip_error("hipMemcpy(tile records)");
    }
}
// Cut segments (in order) into launch groups of at most GHX_MAX_SLOTS distinct field and buffer
// slots each; local[k] = segment k's slots inside its group. One group with identity maps
// (empty) when every caller slot is already below GHX_MAX_SLOTS.
struct slot_partition
{
    std::vector<std::vector<uint32_t>> segs;
    std::vector<std::vector<int32_t>> fmap, bmap;
    std::vector<int32_t> lf, lb;
};

slot_partition partition_slots(const std::vector<int32_t>& gf, const std::vector<int32_t>& gb)
{
    slot_partition p;
    const size_t n = gf.size();
    p.lf = gf;
    p.lb = gb;
    int32_t mf = -1, mb = -1;
    for (size_t k = 0; k < n; ++k)
    {
        mf = std::max(mf, gf[k]);
        mb = std::max(mb, gb[k]);
    }
    if (mf < GHX_MAX_SLOTS && mb < GHX_MAX_SLOTS)
    {
        p.segs.emplace_back();
        for (size_t k = 0; k < n; ++k) p.segs[0].push_back(uint32_t(k));
        p.fmap.emplace_back();
        p.bmap.emplace_back();
        return p;
    }
    std::map<int32_t, int32_t> cf, cb;  // current group: caller slot -> local slot
    for (size_t k = 0; k < n; ++k)
    {
        const bool nf = !cf.count(gf[k]), nb = !cb.count(gb[k]);
        if (p.segs.empty() || cf.size() + nf > size_t(GHX_MAX_SLOTS) ||
            cb.size() + nb > size_t(GHX_MAX_SLOTS))
        {
            p.segs.emplace_back();
            p.fmap.emplace_back();
            p.bmap.emplace_back();
            cf.clear();
            cb.clear();
        }
        auto slot = [](std::map<int32_t, int32_t>& m, std::vector<int32_t>& map, int32_t g) {
            auto it = m.find(g);
            if (it != m.end()) return it->second;
            const int32_t l = int32_t(map.size());
            m.emplace(g, l);
            map.push_back(g);
            return l;
        };
        p.lf[k] = slot(cf, p.fmap.back(), gf[k]);
        p.lb[k] = slot(cb, p.bmap.back(), gb[k]);
        p.segs.back().push_back(uint32_t(k));
    }
    return p;
}

// Fill a launch's pointer slots from the caller's arrays through a group's maps.
void fill_slots(uint64_t (&dst)[GHX_MAX_SLOTS], void* const* src, const std::vector<int32_t>& map,
                int n_identity, const char* what)
{
    const int n = map.empty() ? n_identity : int(map.size());
    for (int i = 0; i < n; ++i)
    {
        void* p = src[map.empty() ? i : map[size_t(i)]];
        if (!p) throw invalid(std::string("null ") + what + " pointer");
        dst[i] = reinterpret_cast<uint64_t>(p);
    }
}
}  // namespace

void device_tables::release()
{
    if (segs) (void)hipFree(segs);
    if (tiles) (void)hipFree(tiles);
    if (recs) (void)hipFree(recs);
    if (lids) (void)hipFree(lids);
    segs = nullptr;
    tiles = nullptr;
    recs = nullptr;
    lids = nullptr;
}

void upload_segments(device_tables& dt, const std::vector<seg_s>& segs)
{
    dt.release();
    if (segs.empty() || !have_device()) return;
    const size_t sb = segs.size() * sizeof(seg_s);
    if (hipMalloc(&dt.segs, sb) != hipSuccess) throw hip_error("hipMalloc(segments)");
    if (hipMemcpy(dt.segs, segs.data(), sb, hipMemcpyHostToDevice) != hipSuccess)
        throw hip_error("hipMemcpy(segments)");
}

void upload_pair_records(device_tables& dt, const std::vector<seg_s>& primary,
                         const std::vector<seg_s>& companion, const std::vector<uint32_t>& tiles)
{
    dt.release();
    if (!g_tune.tile_records || tiles.empty() || !have_device()) return;
    if (primary.size() != companion.size()) throw invalid("pair records: segment counts differ");
    std::vector<seg_s> rec(tiles.size());  // 2 per tile
    for (size_t t = 0; t < tiles.size() / 2; ++t)
    {
        const uint32_t si = tiles[2 * t];
        rec[2 * t] = primary[si];
        rec[2 * t].first_tile = tiles[2 * t + 1];
        rec[2 * t + 1] = companion[si];
    }
    const size_t rb = rec.size() * sizeof(seg_s);
    if (hipMalloc(&dt.recs, rb) != hipSuccess) throw hip_error("hipMalloc(pair records)");
    if (hipMemcpy(dt.recs, rec.data(), rb, hipMemcpyHostToDevice) != hipSuccess)
        throw hip_error("hipMemcpy(pair records)");
}

// ---------------------------------------------------------------------------------------------
// structured
// ---------------------------------------------------------------------------------------------
void validate_field(const ghx_field_desc& f)
{
    if (f.dim < 1 || f.dim > GHX_MAX_DIM) throw invalid("field dim must be in [1, 4]");
    if (f.elem_size < 1) throw invalid("elem_size must be >= 1");
    if (f.num_components < 1) throw invalid("number of components must be greater than 0");
    if (!f.has_components && f.num_components > 1)
        throw invalid("this field cannot have more than 1 components");
    if (f.has_components && f.dim < 2) throw invalid("component axis needs dim >= 2");
    bool seen[GHX_MAX_DIM] = {false, false, false, false};
    for (int d = 0; d < f.dim; ++d)
    {
        if (f.layout[d] < 0 || f.layout[d] >= f.dim || seen[f.layout[d]])
            throw invalid("layout must be a permutation of 0..dim-1");
        seen[f.layout[d]] = true;
    }
}

// Append the segments of one iteration space (`box`, spatial dims only).
// Mirrors make_pack_is / make_buffer_desc / make_is (regular/field_descriptor.hpp:114-150):
// the buffer box is dense in the field's layout order; row = run along the layout's stride-1
// dim. Returns the buffer bytes of the space (is.size() * num_components * sizeof(T)).
uint64_t add_box_segments(std::vector<seg_s>& out, const ghx_field_desc& f, const ghx_box& box,
                          uint16_t field_slot, uint16_t buf_slot, uint64_t buf_off)
{
    const int D = f.dim;
    const int spatial = D - (f.has_components ? 1 : 0);
    int64_t first[GHX_MAX_DIM], ext[GHX_MAX_DIM];
    for (int d = 0; d < D; ++d)
    {
        if (d < spatial)
        {
            first[d] = box.first[d];
            ext[d] = int64_t(box.last[d]) - box.first[d] + 1;
        }
        else
        {
            first[d] = 0;
            ext[d] = f.num_components;
        }
        if (ext[d] <= 0) throw invalid("iteration space: first must be <= last");
        // bounds against the declared extents (the reference does not check; a GPU fault here
        // would take the whole node down, so the planner refuses instead)
        const int64_t off = d < spatial ? f.offsets[d] : 0;
        if (f.extents[d] > 0 && (first[d] + off < 0 || first[d] + ext[d] - 1 + off >= f.extents[d]))
            throw invalid("iteration space outside the field extents");
    }
    int64_t n = 1;
    for (int d = 0; d < D; ++d) n *= ext[d];
    const int64_t elem = f.elem_size;
    // dims sorted by layout value, fastest (value D-1) first
    int by_speed[GHX_MAX_DIM];
    for (int d = 0; d < D; ++d) by_speed[D - 1 - f.layout[d]] = d;
    const int cont = by_speed[0];
    int64_t L;
    int outer[GHX_MAX_DIM + 1];
    int n_outer = 0;
    if (f.byte_strides[cont] == elem)
    {
        L = ext[cont] * elem;
        for (int k = 1; k < D; ++k) outer[n_outer++] = by_speed[k];
    }
    else
    {
        // strided fastest dim: every element is its own row (element-wise semantics of the GPU
        // reference, pack_kernels.hpp:161-183)
        L = elem;
        for (int k = 0; k < D; ++k) outer[n_outer++] = by_speed[k];
    }
    int64_t ostride[GHX_MAX_DIM], oext[GHX_MAX_DIM];
    for (int k = 0; k < n_outer; ++k)
    {
        ostride[k] = f.byte_strides[outer[k]];
        oext[k] = ext[outer[k]];
    }
    // merge rows that are contiguous in the field too (box spans the full padded run)
    while (n_outer > 0 && ostride[0] == L && oext[0] * L < (int64_t(1) << 30))
    {
        L *= oext[0];
        for (int k = 1; k < n_outer; ++k)
        {
            ostride[k - 1] = ostride[k];
            oext[k - 1] = oext[k];
        }
        --n_outer;
    }
    if (n_outer > 4) throw invalid("too many outer dims");
    if (L >= (int64_t(1) << 31)) throw invalid("row too long");
    int64_t field_off = 0;
    for (int d = 0; d < D; ++d)
    {
        const int64_t off = d < spatial ? f.offsets[d] : 0;
        field_off += (first[d] + off) * f.byte_strides[d];
    }
    // split along the slowest outer dim so that one segment stays below 2^31 bytes
    int64_t rows_per_slowest = 1;
    for (int k = 0; k + 1 < n_outer; ++k) rows_per_slowest *= oext[k];
    const int64_t slab = rows_per_slowest * L;  // bytes per unit of the slowest outer dim
    const int64_t nslow = n_outer > 0 ? oext[n_outer - 1] : 1;
    const int64_t max_bytes = (int64_t(1) << 31) - kMaxTileBytes;
    int64_t chunk = n_outer > 0 ? std::max<int64_t>(1, max_bytes / slab) : 1;
    if (n_outer == 0 && L > max_bytes) throw invalid("segment too large");
    if (n_outer > 0 && slab > max_bytes) throw invalid("segment row block too large");
    for (int64_t s0 = 0; s0 < nslow; s0 += chunk)
    {
        const int64_t cnt = std::min(chunk, nslow - s0);
        seg_s s{};
        s.field_slot = field_slot;
        s.buf_slot = buf_slot;
        s.row_bytes = uint32_t(L);
        s.n_outer = uint8_t(n_outer);
        int64_t rows = 1;
        for (int k = 0; k < 4; ++k)
        {
            if (k < n_outer)
            {
                s.stride[k] = ostride[k];
                s.ext[k] = uint32_t(k == n_outer - 1 ? cnt : oext[k]);
            }
            else
            {
                s.stride[k] = 0;
                s.ext[k] = 1;
            }
            rows *= s.ext[k];
        }
        s.field_off = field_off + (n_outer > 0 ? s0 * ostride[n_outer - 1] : 0);
        s.buf_off = buf_off + uint64_t(s0 * slab);
        s.bytes = uint32_t(rows * L);
        s.mag_row = make_magic(uint32_t(L));
        for (int k = 0; k < 3; ++k) s.mag_ext[k] = make_magic(s.ext[k]);
        const int wb = std::min(wlog2_of(uint64_t(L)), wlog2_of(s.buf_off));  // buffer side
        int wf = wlog2_of(uint64_t(s.field_off));                             // field side
        for (int k = 0; k < n_outer; ++k)
            if (s.ext[k] > 1) wf = std::min(wf, wlog2_of(uint64_t(s.stride[k] < 0 ? -s.stride[k] : s.stride[k])));
        s.wlog2 = uint8_t(std::min(wb, wf));
        s.amode = short_addressing(s);
        out.push_back(s);
    }
    return uint64_t(n * elem);
}

splan::splan(const ghx_pack_entry* entries, int n_entries, int dir) : direction(dir)
{
    tile_bytes = g_tune.tile_bytes;
    if (dir != 0 && dir != 1) throw invalid("direction must be 0 (pack) or 1 (unpack)");
    std::vector<seg_s> segs;
    std::vector<int32_t> gf, gb;  // caller slots per segment
    for (int e = 0; e < n_entries; ++e)
    {
        const auto& en = entries[e];
        validate_field(en.field);
        if (en.field_slot < 0 || en.buffer_slot < 0) throw invalid("negative slot");
        if (en.n_boxes < 0 || (en.n_boxes > 0 && !en.boxes)) throw invalid("bad boxes");
        max_field_slot = std::max(max_field_slot, en.field_slot);
        max_buf_slot = std::max(max_buf_slot, en.buffer_slot);
        uint64_t off = en.buffer_offset;
        for (int b = 0; b < en.n_boxes; ++b)
            off += add_box_segments(segs, en.field, en.boxes[b], 0, 0, off);
        gf.resize(segs.size(), en.field_slot);
        gb.resize(segs.size(), en.buffer_slot);
        bytes += off - en.buffer_offset;
    }
    n_segments = int32_t(segs.size());
    const slot_partition part = partition_slots(gf, gb);
    for (size_t g = 0; g < part.segs.size(); ++g)
    {
        std::vector<seg_s> gs;
        for (uint32_t k : part.segs[g])
        {
            seg_s x = segs[k];
            x.field_slot = uint16_t(part.lf[k]);
            x.buf_slot = uint16_t(part.lb[k]);
            gs.push_back(x);
        }
        std::vector<uint32_t> tiles = build_tiles(gs, direction);
        if (g == 0)
        {
            n_tiles = uint32_t(tiles.size() / 2);
            host_segs = gs;
            host_tiles = tiles;
            fmap = part.fmap[0];
            bmap = part.bmap[0];
            upload(dev, gs, tiles);
            continue;
        }
        auto grp = std::make_unique<slot_group<seg_s>>();
        grp->fmap = part.fmap[g];
        grp->bmap = part.bmap[g];
        grp->n_tiles = uint32_t(tiles.size() / 2);
        grp->host_segs = gs;
        upload(grp->dev, gs, tiles);
        more.push_back(std::move(grp));
    }
}

uint32_t splan::total_tiles() const
{
    uint32_t t = n_tiles;
    for (const auto& g : more) t += g->n_tiles;
    return t;
}

int splan::execute(void* const* fptr, int nf, void* const* bptr, int nb, void* stream) const
{
    if (total_tiles() == 0) return GHX_OK;
    if (nf <= max_field_slot || nb <= max_buf_slot) throw invalid("pointer arrays do not cover the plan's slots");
    auto run = [&](const device_tables& dt, uint32_t nt, const std::vector<int32_t>& fm,
                   const std::vector<int32_t>& bm) {
        if (nt == 0) return int(GHX_OK);
        if (!dt.segs) throw hip_error("plan has no device tables (no HIP device at creation)");
        kargs a{};
        a.segs = dt.segs;
        a.tile_seg = dt.tiles;
        a.tile_recs = dt.recs;
        a.n_tiles = nt;
        fill_slots(a.field_ptr, fptr, fm, max_field_slot + 1, "field");
        fill_slots(a.buf_ptr, bptr, bm, max_buf_slot + 1, "buffer");
        parity.apply(a, bm, max_buf_slot + 1);
        return launch_structured(a, direction, stream, grid_for_tiles(nt));
    };
    int rc = run(dev, n_tiles, fmap, bmap);
    for (size_t g = 0; rc == GHX_OK && g < more.size(); ++g)
        rc = run(more[g]->dev, more[g]->n_tiles, more[g]->fmap, more[g]->bmap);
    return rc;
}

// ---------------------------------------------------------------------------------------------
// unstructured
// ---------------------------------------------------------------------------------------------
uplan::uplan(const ghx_upack_entry* entries, int n_entries, int dir) : direction(dir)
{
    tile_bytes = g_tune.tile_bytes;
    if (dir != 0 && dir != 1) throw invalid("direction must be 0 (pack) or 1 (unpack)");
    std::vector<seg_u> segs;
    // all index lists in one device allocation: int32 where they fit
    struct pending
    {
        size_t seg;
        size_t off;  // the segment's list in the device allocation
    };
    struct lid_upload
    {
        const int64_t* lids;
        int64_t n;
        bool wide;
        size_t off;
    };
    std::vector<pending> pend;
    std::vector<lid_upload> uploads;
    std::map<std::pair<const int64_t*, int64_t>, size_t> lid_off;
    std::vector<int32_t> gf, gb;  // caller slots per segment
    size_t lid_bytes = 0;
    for (int e = 0; e < n_entries; ++e)
    {
        const auto& en = entries[e];
        const auto& d = en.data;
        if (d.elem_size < 1 || d.levels < 1) throw invalid("bad unstructured data descriptor");
        if (en.field_slot < 0 || en.buffer_slot < 0) throw invalid("negative slot");
        if (en.n_lids < 0 || (en.n_lids > 0 && !en.lids)) throw invalid("bad index list");
        max_field_slot = std::max(max_field_slot, en.field_slot);
        max_buf_slot = std::max(max_buf_slot, en.buffer_slot);
        if (en.n_lids == 0) continue;
        const int64_t elem = d.elem_size;
        bool wide = false;
        for (int64_t i = 0; i < en.n_lids; ++i)
        {
            if (en.lids[i] < 0) throw invalid("negative local index");
            if (en.lids[i] >= (int64_t(1) << 31)) wide = true;
        }
        int mode;
        int64_t L;
        if (d.levels == 1 || (d.levels_first && d.level_stride == 1))
        {
            mode = 0;  // one row per index: all levels contiguous on both sides
            L = d.levels * elem;
        }
        else
        {
            mode = d.levels_first ? 1 : 2;  // rows (i, l) i-major / rows (l, i) l-major
            L = elem;
        }
        // one segment of index range [a, a + n) of the list (mode 2 split: one level `lev`, as
        // a mode-0 segment of elem-byte rows at field offset lev * level stride)
        auto add = [&](int64_t a, int64_t n, int m, int64_t lev, uint64_t buf_off) {
            seg_u s{};  // slots: set per launch group below
            s.buf_off = buf_off;
            s.n = uint32_t(n);
            s.index_stride_b = d.index_stride * elem;
            s.level_stride_b = d.level_stride * elem;
            s.field_off = lev >= 0 ? lev * s.level_stride_b : 0;
            s.lid64 = wide ? 1 : 0;
            s.mode = uint8_t(m);
            const int64_t Ls = m == 0 && lev < 0 ? L : elem;
            if (m == 1)
            {
                s.row_levels = uint32_t(d.levels);
                s.mag_inner = make_magic(uint32_t(d.levels));
            }
            else if (m == 2)
                s.mag_inner = make_magic(uint32_t(n));
            const int64_t seg_bytes = n * (m == 0 ? Ls : int64_t(d.levels) * elem);
            s.row_bytes = uint32_t(Ls);
            s.bytes = uint32_t(seg_bytes);
            s.mag_row = make_magic(uint32_t(Ls));
            int w = wlog2_of(uint64_t(Ls));
            w = std::min(w, wlog2_of(s.buf_off));
            w = std::min(w, wlog2_of(uint64_t(s.field_off < 0 ? -s.field_off : s.field_off)));
            if (n > 1) w = std::min(w, wlog2_of(uint64_t(s.index_stride_b < 0 ? -s.index_stride_b : s.index_stride_b)));
            if (m != 0) w = std::min(w, wlog2_of(uint64_t(s.level_stride_b < 0 ? -s.level_stride_b : s.level_stride_b)));
            s.wlog2 = uint8_t(w);
            // 4/8-B rows whose consecutive lids are adjacent in the field (index stride = row
            // length): 16-B lane chunks, one field access per run of 16/L lids (copy_runs)
            s.runs = (g_tune.urun && m == 0 && (Ls == 4 || Ls == 8) && s.index_stride_b == Ls &&
                      s.buf_off % 16 == 0) ? 1 : 0;
            if (s.runs)
            {
                // run-heavy: at least half of the 16-B chunks hold 16/L consecutive lids
                const int64_t K = 16 / Ls, chunks = n / K;
                const int64_t* li = en.lids + a;
                int64_t hits = 0;
                for (int64_t c = 0; c < chunks; ++c)
                {
                    bool run = true;
                    for (int64_t j = 1; j < K && run; ++j) run = li[c * K + j] == li[c * K] + j;
                    hits += run ? 1 : 0;
                }
                if (chunks > 0 && 2 * hits >= chunks) s.runs = 2;
            }
            // index lists shared by the segments that read the same range (split levels)
            const auto key = std::make_pair(en.lids + a, n);
            auto it = lid_off.find(key);
            size_t off;
            if (it != lid_off.end()) off = it->second;
            else
            {
                lid_bytes = (lid_bytes + 15) & ~size_t(15);
                off = lid_bytes;
                lid_bytes += size_t(n) * (wide ? 8 : 4);
                lid_off.emplace(key, off);
                uploads.push_back({en.lids + a, n, wide, off});
            }
            pend.push_back({segs.size(), off});
            segs.push_back(s);
            gf.push_back(en.field_slot);
            gb.push_back(en.buffer_slot);
        };
        // a segment addresses its bytes with 32-bit offsets: lists of more than kSegLimit bytes
        // are planned as several segments (index ranges; a levels-last list level by level)
        constexpr int64_t kSegLimit = int64_t(1) << 30;
        const int64_t per_index = int64_t(d.levels) * elem;
        const int64_t total = en.n_lids * per_index;
        if (per_index > kSegLimit) throw invalid("unstructured row of more than 1 GiB");
        if (total <= kSegLimit && en.n_lids < (int64_t(1) << 32))
            add(0, en.n_lids, mode, -1, en.buffer_offset);
        else if (mode != 2)
        {
            const int64_t step = kSegLimit / per_index;
            for (int64_t a = 0; a < en.n_lids; a += step)
                add(a, std::min(step, en.n_lids - a), mode, -1,
                    en.buffer_offset + uint64_t(a * per_index));
        }
        else
        {
            const int64_t step = kSegLimit / elem;
            for (int64_t lev = 0; lev < d.levels; ++lev)
                for (int64_t a = 0; a < en.n_lids; a += step)
                    add(a, std::min(step, en.n_lids - a), 0, lev,
                        en.buffer_offset + uint64_t((lev * en.n_lids + a) * elem));
        }
        bytes += uint64_t(total);
    }
    n_segments = int32_t(segs.size());
    if (!segs.empty() && have_device())
    {
        std::vector<unsigned char> host(lid_bytes);
        for (auto& p : uploads)
        {
            if (p.wide)
            {
                int64_t* dst = reinterpret_cast<int64_t*>(host.data() + p.off);
                for (int64_t i = 0; i < p.n; ++i) dst[i] = p.lids[i];
            }
            else
            {
                int32_t* dst = reinterpret_cast<int32_t*>(host.data() + p.off);
                for (int64_t i = 0; i < p.n; ++i) dst[i] = int32_t(p.lids[i]);
            }
        }
        if (hipMalloc(&dev.lids, lid_bytes) != hipSuccess) throw hip_error("hipMalloc(lids)");
        if (hipMemcpy(dev.lids, host.data(), lid_bytes, hipMemcpyHostToDevice) != hipSuccess)
            throw hip_error("hipMemcpy(lids)");
        for (auto& p : pend) segs[p.seg].lids = static_cast<char*>(dev.lids) + p.off;
    }
    const slot_partition part = partition_slots(gf, gb);
    for (size_t g = 0; g < part.segs.size(); ++g)
    {
        std::vector<seg_u> gs;
        for (uint32_t k : part.segs[g])
        {
            seg_u x = segs[k];
            x.field_slot = uint16_t(part.lf[k]);
            x.buf_slot = uint16_t(part.lb[k]);
            gs.push_back(x);
        }
        std::vector<uint32_t> tiles = build_tiles(gs, direction);
        if (g == 0)
        {
            n_tiles = uint32_t(tiles.size() / 2);
            host_segs = gs;
            fmap = part.fmap[0];
            bmap = part.bmap[0];
            void* keep = dev.lids;
            dev.lids = nullptr;  // upload() releases; re-attach after (the groups share it)
            upload(dev, gs, tiles);
            dev.lids = keep;
            continue;
        }
        auto grp = std::make_unique<slot_group<seg_u>>();
        grp->fmap = part.fmap[g];
        grp->bmap = part.bmap[g];
        grp->n_tiles = uint32_t(tiles.size() / 2);
        grp->host_segs = gs;
        upload(grp->dev, gs, tiles);
        more.push_back(std::move(grp));
    }
}

uint32_t uplan::total_tiles() const
{
    uint32_t t = n_tiles;
    for (const auto& g : more) t += g->n_tiles;
    return t;
}

int uplan::execute(void* const* fptr, int nf, void* const* bptr, int nb, void* stream) const
{
    if (total_tiles() == 0) return GHX_OK;
    if (nf <= max_field_slot || nb <= max_buf_slot) throw invalid("pointer arrays do not cover the plan's slots");
    auto run = [&](const device_tables& dt, uint32_t nt, const std::vector<int32_t>& fm,
                   const std::vector<int32_t>& bm, const std::vector<seg_u>& hs) {
        if (nt == 0) return int(GHX_OK);
        if (!dt.segs) throw hip_error("plan has no device tables (no HIP device at creation)");
        kargs a{};
        a.segs = dt.segs;
        a.tile_seg = dt.tiles;
        a.tile_recs = dt.recs;
        a.n_tiles = nt;
        fill_slots(a.field_ptr, fptr, fm, max_field_slot + 1, "field");
        fill_slots(a.buf_ptr, bptr, bm, max_buf_slot + 1, "buffer");
        parity.apply(a, bm, max_buf_slot + 1);
        // the run-path kernel when every segment qualifies with these pointers: flagged by the
        // planner, whole 16-B chunks per tile, 16-B aligned buffer ranges (both copies of a
        // double-buffered one), field base aligned to L
        bool runs = !hs.empty();
        for (const seg_u& s : hs)
            runs = runs && s.runs && s.tile_bytes % 16 == 0 &&
                   (a.buf_ptr[s.buf_slot] + s.buf_off) % 16 == 0 && a.dbl_off[s.buf_slot] % 16 == 0 &&
                   a.field_ptr[s.field_slot] % s.row_bytes == 0;
        return launch_unstructured(a, direction, stream, grid_for_tiles(nt), runs);
    };
    int rc = run(dev, n_tiles, fmap, bmap, host_segs);
    for (size_t g = 0; rc == GHX_OK && g < more.size(); ++g)
        rc = run(more[g]->dev, more[g]->n_tiles, more[g]->fmap, more[g]->bmap, more[g]->host_segs);
    return rc;
}

}  // namespace ghx
