// ghx_plan.hpp — host planner objects behind the opaque C handles.
#pragma once

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ghx_internal.hpp"

namespace ghx
{
struct invalid : std::runtime_error
{
    using std::runtime_error::runtime_error;
};
struct hip_error : std::runtime_error
{
    using std::runtime_error::runtime_error;
};

struct device_tables
{
    void* segs = nullptr;
    uint32_t* tiles = nullptr;
    void* recs = nullptr;  // tile records (g_tune.tile_records): per tile a copy of its segment
    void* lids = nullptr;
    void release();
    device_tables() = default;
    device_tables(const device_tables&) = delete;
    device_tables& operator=(const device_tables&) = delete;
    ~device_tables() { release(); }
};

void validate_field(const ghx_field_desc& f);
// segment table alone to device memory (a no-op without a HIP device)
void upload_segments(device_tables& dt, const std::vector<seg_s>& segs);
// Pair records of a fused launch (k_self, k_put; g_tune.tile_records): per tile of the primary
// plan, in its dispatch order, the primary segment (with the tile's index in first_tile) and
// the companion segment of the same index, side by side (dt.recs; a no-op without a device or
// with tile_records off)
void upload_pair_records(device_tables& dt, const std::vector<seg_s>& primary,
                         const std::vector<seg_s>& companion, const std::vector<uint32_t>& tiles);
uint64_t add_box_segments(std::vector<seg_s>& out, const ghx_field_desc& f, const ghx_box& box,
                          uint16_t field_slot, uint16_t buf_slot, uint64_t buf_off);

// Launch groups. A launch carries at most GHX_MAX_SLOTS field and buffer pointers (kargs is
// passed by value); a plan whose entries use more slots than that (many fields in one exchange,
// or many domain-pair buffers: a rank holding many domains) is cut into groups of segments in
// entry order, each with its own slot maps (local slot -> the caller's slot) and tables, and
// executes as one launch per group on the same stream. The reference has no such limit
// (include/ghex/communication_object.hpp:1003-1067 allocates any number of buffers).
template<typename Seg>
struct slot_group
{
    std::vector<int32_t> fmap, bmap;  // local slot -> caller slot; empty: identity
    uint32_t n_tiles = 0;
    std::vector<Seg> host_segs;
    device_tables dev;
};

// structured fused plan
struct splan
{
    int direction = 0;
    uint64_t bytes = 0;
    int32_t n_segments = 0;
    uint32_t n_tiles = 0;      // the first launch group's (the whole plan's when not grouped)
    uint32_t tile_bytes = kTileBytes;
    int max_field_slot = -1, max_buf_slot = -1;  // caller slots
    std::vector<seg_s> host_segs;                // the first group's, local slots
    std::vector<uint32_t> host_tiles;            // the first group's tile table (pair records)
    device_tables dev;
    std::vector<int32_t> fmap, bmap;             // the first group's slot maps (empty: identity)
    std::vector<std::unique_ptr<slot_group<seg_s>>> more;  // further launch groups
    parity_cfg parity;                           // double-buffered buffers (direct exchange)
    bool grouped() const { return !fmap.empty() || !bmap.empty() || !more.empty(); }
    uint32_t total_tiles() const;
    splan(const ghx_pack_entry* entries, int n_entries, int direction);
    int execute(void* const* fptr, int nf, void* const* bptr, int nb, void* stream) const;
};

// unstructured fused plan
struct uplan
{
    int direction = 0;
    uint64_t bytes = 0;
    int32_t n_segments = 0;
    uint32_t n_tiles = 0;
    uint32_t tile_bytes = kTileBytes;
    int max_field_slot = -1, max_buf_slot = -1;
    device_tables dev;
    std::vector<seg_u> host_segs;  // for the launch-time choice of the run-path kernel
    std::vector<int32_t> fmap, bmap;
    std::vector<std::unique_ptr<slot_group<seg_u>>> more;
    parity_cfg parity;
    bool grouped() const { return !fmap.empty() || !bmap.empty() || !more.empty(); }
    uint32_t total_tiles() const;
    uplan(const ghx_upack_entry* entries, int n_entries, int direction);
    int execute(void* const* fptr, int nf, void* const* bptr, int nb, void* stream) const;
};
}  // namespace ghx

// opaque handles
struct ghx_plan : ghx::splan
{
    using ghx::splan::splan;
};
struct ghx_uplan : ghx::uplan
{
    using ghx::uplan::uplan;
};
