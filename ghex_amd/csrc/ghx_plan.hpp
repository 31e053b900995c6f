// ghx_plan.hpp — host planner objects behind the opaque C handles.
#pragma once

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
uint64_t add_box_segments(std::vector<seg_s>& out, const ghx_field_desc& f, const ghx_box& box,
                          uint16_t field_slot, uint16_t buf_slot, uint64_t buf_off);

// structured fused plan
struct splan
{
    int direction = 0;
    uint64_t bytes = 0;
    int32_t n_segments = 0;
    uint32_t n_tiles = 0;
    uint32_t tile_bytes = kTileBytes;
    int max_field_slot = -1, max_buf_slot = -1;
    std::vector<seg_s> host_segs;
    device_tables dev;
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
