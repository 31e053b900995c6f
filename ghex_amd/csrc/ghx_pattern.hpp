// ghx_pattern.hpp — host-side halo patterns (setup time): the producers of the pack inputs.
#pragma once

#include <cstdint>
#include <vector>

#include "ghx_internal.hpp"

namespace ghx
{
struct is_pair
{
    int32_t lf[3], ll[3], gf[3], gl[3];
    int64_t size(int dim) const
    {
        int64_t s = 1;
        for (int d = 0; d < dim; ++d) s *= int64_t(ll[d]) - lf[d] + 1;
        return s;
    }
};

struct halo_key
{
    int32_t remote_id;
    int32_t remote_rank;
    int32_t tag;
};

struct halo_entry
{
    halo_key key;
    std::vector<is_pair> boxes;   // structured
    std::vector<int64_t> lids;    // unstructured (its single iteration space)
};

struct domain_pattern
{
    int32_t id = 0;
    std::vector<halo_entry> send;  // std::map order
    std::vector<halo_entry> recv;
};

struct pattern_set
{
    int kind = 0;  // 0 structured, 1 unstructured
    int dim = 3;
    int32_t max_tag = 0;
    int32_t my_rank = -1;  // the rank the pattern was made for (self messages: remote_rank ==)
    std::vector<domain_pattern> doms;
};

// halo_generator::operator() + intersect (include/ghex/structured/regular/halo_generator.hpp)
std::vector<is_pair> regular_halo_boxes(int dim, const int32_t* gfirst, const int32_t* glast,
                                        const int32_t* halos, const int32_t* periodic,
                                        const int32_t* dfirst, const int32_t* dlast);

int regular_make_pattern(int dim, const ghx_regular_domain* doms, int n, const int32_t* gfirst,
                         const int32_t* glast, const int32_t* halos, const int32_t* periodic,
                         int my_rank, pattern_set& out);

// make_staged_pattern (include/ghex/structured/regular/make_pattern.hpp:47-250): dim patterns
void staged_make_pattern(int dim, const ghx_regular_domain* doms, int n, const int32_t* nbrs,
                         const int32_t* gfirst, const int32_t* glast, const int32_t* halos,
                         const int32_t* periodic, int my_rank, std::vector<pattern_set>& out);

}  // namespace ghx

// the opaque C-ABI pattern handle (include/ghx.h)
struct ghx_pattern : ghx::pattern_set
{
};
