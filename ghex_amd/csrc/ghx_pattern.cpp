// ghx_pattern.cpp — structured and unstructured halo patterns, computed on the host.
//
// The pattern fixes the packed byte layout (its iteration-space order is the buffer order), so
// these follow the reference's ordering rules exactly. Setup collectives are replaced by taking
// every rank's domains as input (the caller all-gathers them once, e.g. with torch.distributed),
// after which each rank derives its own maps locally with no further communication.
#include "ghx_pattern.hpp"

#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>

namespace ghx
{
// ---------------------------------------------------------------------------------------------
// structured, regular
// ---------------------------------------------------------------------------------------------
std::vector<is_pair> regular_halo_boxes(int dim, const int32_t* gfirst, const int32_t* glast,
                                        const int32_t* halos, const int32_t* periodic,
                                        const int32_t* dfirst, const int32_t* dlast)
{
    // the three 1-D spaces {left, middle, right} per dimension (halo_generator.hpp:95-118)
    int32_t sp[3][3][4];  // [space][dim][lf, ll, gf, gl]
    for (int d = 0; d < dim; ++d)
    {
        const int32_t lf = -halos[2 * d];
        sp[0][d][0] = lf;
        sp[0][d][1] = -1;
        sp[0][d][2] = lf + dfirst[d];
        sp[0][d][3] = dfirst[d] - 1;
        sp[1][d][0] = 0;
        sp[1][d][1] = dlast[d] - dfirst[d];
        sp[1][d][2] = dfirst[d];
        sp[1][d][3] = dlast[d];
        sp[2][d][0] = sp[1][d][1] + 1;
        sp[2][d][1] = sp[1][d][1] + halos[2 * d + 1];
        sp[2][d][2] = dlast[d] + 1;
        sp[2][d][3] = dlast[d] + halos[2 * d + 1];
    }
    // compute_spaces (:163-197): dimension 0 is the outermost recursion level, i.e. the most
    // significant base-3 digit; the centre (3^D/2) and empty boxes are dropped (:124-131).
    int n3 = 1;
    for (int d = 0; d < dim; ++d) n3 *= 3;
    std::vector<is_pair> out;
    for (int j = 0; j < n3; ++j)
    {
        if (j == n3 / 2) continue;
        is_pair b{};
        int r = j;
        int digit[3] = {0, 0, 0};
        for (int d = dim - 1; d >= 0; --d)
        {
            digit[d] = r % 3;
            r /= 3;
        }
        bool empty = false;
        for (int d = 0; d < dim; ++d)
        {
            const int32_t* s = sp[digit[d]][d];
            b.lf[d] = s[0];
            b.ll[d] = s[1];
            b.gf[d] = s[2];
            b.gl[d] = s[3];
            if (b.ll[d] < b.lf[d]) empty = true;
        }
        if (!empty) out.push_back(b);
    }
    // periodic wrap of the global coordinates (:133-145)
    for (auto& b : out)
        for (int d = 0; d < dim; ++d)
        {
            if (!periodic[d]) continue;
            const int32_t ext_h = b.gl[d] - b.gf[d];
            const int32_t ext = glast[d] + 1 - gfirst[d];
            const int32_t off = b.gf[d] - gfirst[d];
            b.gf[d] = (off + ext) % ext + gfirst[d];
            b.gl[d] = b.gf[d] + ext_h;
        }
    return out;
}

int regular_make_pattern(int dim, const ghx_regular_domain* doms, int n, const int32_t* gfirst,
                         const int32_t* glast, const int32_t* halos, const int32_t* periodic,
                         int my_rank, pattern_set& out)
{
    if (dim < 1 || dim > 3 || n < 1) throw std::runtime_error("regular pattern: bad dim / count");
    // ranks in ascending order, each rank's domains in their given order (pattern.hpp:302-308)
    int world = 0;
    for (int i = 0; i < n; ++i) world = std::max(world, doms[i].rank + 1);
    std::vector<std::vector<int>> by_rank(world);
    for (int i = 0; i < n; ++i)
    {
        if (doms[i].rank < 0) throw std::runtime_error("regular pattern: negative rank");
        by_rank[doms[i].rank].push_back(i);
    }
    // recv halos of every domain (all ranks: the receivers assign the tags that the senders'
    // keys carry): boxes x ranks x domains, keyed by the remote domain id (pattern.hpp:290-329)
    struct recv_map
    {
        std::map<int32_t, std::pair<int32_t, std::vector<is_pair>>> by_id;  // id -> (rank, IS)
        std::vector<halo_entry> entries;                                    // with tags
    };
    std::vector<recv_map> recv(n);
    for (int a = 0; a < n; ++a)
    {
        const auto& d = doms[a];
        auto boxes = regular_halo_boxes(dim, gfirst, glast, halos, periodic, d.first, d.last);
        for (const auto& b : boxes)
            for (int j = 0; j < world; ++j)
                for (int k : by_rank[j])
                {
                    const auto& o = doms[k];
                    is_pair x{};
                    bool ok = true;
                    for (int c = 0; c < dim; ++c)
                    {
                        x.gf[c] = std::max(b.gf[c], o.first[c]);
                        x.gl[c] = std::min(b.gl[c], o.last[c]);
                        x.lf[c] = b.lf[c] + (x.gf[c] - b.gf[c]);
                        x.ll[c] = b.lf[c] + (x.gl[c] - b.gf[c]);
                        if (x.gf[c] > x.gl[c]) ok = false;
                    }
                    if (!ok) continue;
                    auto it = recv[a].by_id.find(o.id);
                    if (it == recv[a].by_id.end())
                        it = recv[a].by_id.emplace(o.id, std::make_pair(o.rank, std::vector<is_pair>{})).first;
                    it->second.second.push_back(x);
                }
    }
    // tags: per receiving rank, per remote rank 0,1,2,... over its patterns in order, each
    // pattern's map in key order (pattern.hpp:331-367)
    int32_t max_tag = 0;
    for (int r = 0; r < world; ++r)
    {
        std::map<int32_t, int32_t> tag_map;
        for (int a : by_rank[r])
            for (auto& kv : recv[a].by_id)
            {
                const int32_t rr = kv.second.first;
                int32_t tag;
                auto it = tag_map.find(rr);
                if (it == tag_map.end())
                {
                    tag_map[rr] = 0;
                    tag = 0;
                }
                else
                {
                    tag = ++it->second;
                    max_tag = std::max(max_tag, tag);
                }
                halo_entry e;
                e.key = {kv.first, rr, tag};
                e.boxes = kv.second.second;
                recv[a].entries.push_back(std::move(e));
            }
    }
    // my patterns: recv maps as computed; send maps = the receivers' lists translated into my
    // local coordinates, keyed (receiver id, tag) (pattern.hpp:369-437, 536-561)
    out = pattern_set{};
    out.kind = 0;
    out.dim = dim;
    out.max_tag = max_tag;
    out.my_rank = my_rank;
    if (my_rank < 0 || my_rank >= world) return GHX_OK;
    for (int a : by_rank[my_rank])
    {
        domain_pattern p;
        p.id = doms[a].id;
        p.recv = recv[a].entries;  // already in (id, tag) order: ids unique per map
        std::map<std::pair<int32_t, int32_t>, halo_entry> send;
        for (int b = 0; b < n; ++b)
            for (const auto& e : recv[b].entries)
            {
                if (e.key.remote_id != doms[a].id || e.key.remote_rank != my_rank) continue;
                halo_entry s;
                s.key = {doms[b].id, doms[b].rank, e.key.tag};
                for (auto x : e.boxes)
                {
                    for (int c = 0; c < dim; ++c)
                    {
                        x.lf[c] = x.gf[c] - doms[a].first[c];
                        x.ll[c] = x.gl[c] - doms[a].first[c];
                    }
                    s.boxes.push_back(x);
                }
                send.emplace(std::make_pair(s.key.remote_id, s.key.tag), std::move(s));
            }
        for (auto& kv : send) p.send.push_back(std::move(kv.second));
        out.doms.push_back(std::move(p));
    }
    return GHX_OK;
}

// ---------------------------------------------------------------------------------------------
// staged (dimension-by-dimension) patterns
// ---------------------------------------------------------------------------------------------
// make_staged_pattern (include/ghex/structured/regular/make_pattern.hpp:47-250): one pattern per
// dimension. Stage i exchanges the two halo slabs of dimension i only, over the domain box
// already extended by the halos of the stages before it, so that running the stages in order
// fills edges and corners without diagonal messages. Keys hold the neighbour the user's domain
// lookup names (nbrs: per domain and dimension the left and right neighbour's id); tags are
// assigned by the receivers per remote rank over their patterns in order (make_pattern.hpp:
// 199-243), max_tag is the receiving rank's own maximum (make_pattern.hpp:201, 227).
void staged_make_pattern(int dim, const ghx_regular_domain* doms, int n, const int32_t* nbrs,
                         const int32_t* gfirst, const int32_t* glast, const int32_t* halos,
                         const int32_t* periodic, int my_rank, std::vector<pattern_set>& out)
{
    if (dim < 1 || dim > 3 || n < 1) throw std::runtime_error("staged pattern: bad dim / count");
    std::map<int32_t, int> index_of;
    int world = 0;
    for (int a = 0; a < n; ++a)
    {
        if (doms[a].rank < 0) throw std::runtime_error("staged pattern: negative rank");
        if (!index_of.emplace(doms[a].id, a).second)
            throw std::runtime_error("staged pattern: domain ids must be unique");
        world = std::max(world, doms[a].rank + 1);
    }
    auto neighbour = [&](int a, int i, int side) -> int {
        const int32_t id = nbrs[(a * dim + i) * 2 + side];
        auto it = index_of.find(id);
        if (it == index_of.end())
            throw std::runtime_error("staged pattern: the domain lookup names an unknown neighbour");
        return it->second;
    };
    using keyed = std::map<int32_t, std::vector<is_pair>>;  // remote id -> spaces (map order)
    std::vector<std::vector<keyed>> recv(dim, std::vector<keyed>(n)), send(dim, std::vector<keyed>(n));
    for (int a = 0; a < n; ++a)
    {
        is_pair ext{};
        for (int c = 0; c < dim; ++c)
        {
            ext.lf[c] = 0;
            ext.ll[c] = doms[a].last[c] - doms[a].first[c];
            ext.gf[c] = doms[a].first[c];
            ext.gl[c] = doms[a].last[c];
        }
        for (int i = 0; i < dim; ++i)
        {
            const int hl = halos[2 * i], hr = halos[2 * i + 1];
            const bool has_left = hl > 0 && (periodic[i] || ext.gf[i] - hl >= gfirst[i]);
            const bool has_right = hr > 0 && (periodic[i] || ext.gl[i] + hr <= glast[i]);
            const int32_t left = has_left ? doms[neighbour(a, i, 0)].id : -1;
            const int32_t right = has_right ? doms[neighbour(a, i, 1)].id : -1;
            if (has_left)
            {
                is_pair x = ext;  // recv_left
                x.ll[i] = x.lf[i] - 1;
                x.lf[i] -= hl;
                x.gl[i] = x.gf[i] - 1;
                x.gf[i] -= hl;
                recv[i][a][left].push_back(x);
            }
            if (has_right)
            {
                is_pair x = ext;  // send_right: my last hl cells go to the right neighbour
                x.lf[i] = x.ll[i] + 1 - hl;
                x.gf[i] = x.gl[i] + 1 - hl;
                // hl = 0: an empty box that the right neighbour (no left halo) never receives;
                // the reference still keys it and its tag hand-off (make_pattern.hpp:219-243)
                // then waits for a tag message that no rank sends — dropped here
                if (hl > 0) send[i][a][right].push_back(x);
                is_pair y = ext;  // recv_right
                y.lf[i] = y.ll[i] + 1;
                y.gf[i] = y.gl[i] + 1;
                y.ll[i] += hr;
                y.gl[i] += hr;
                recv[i][a][right].push_back(y);
            }
            if (has_left)
            {
                is_pair x = ext;  // send_left: my first hr cells go to the left neighbour
                x.ll[i] = x.lf[i] - 1 + hr;
                x.gl[i] = x.gf[i] - 1 + hr;
                if (hr > 0) send[i][a][left].push_back(x);  // (hr = 0: as send_right above)
            }
            if (has_left)
            {
                ext.lf[i] -= hl;
                ext.gf[i] -= hl;
            }
            if (has_right)
            {
                ext.ll[i] += hr;
                ext.gl[i] += hr;
            }
        }
    }
    std::vector<std::vector<int>> by_rank(world);
    for (int a = 0; a < n; ++a) by_rank[doms[a].rank].push_back(a);
    out.assign(dim, pattern_set{});
    for (int i = 0; i < dim; ++i)
    {
        // receivers' tags: (sender id, receiver id) -> tag
        std::map<std::pair<int32_t, int32_t>, int32_t> tag_of;
        int32_t my_max_tag = 0;
        for (int r = 0; r < world; ++r)
        {
            std::map<int32_t, int32_t> last_tag;  // remote rank -> last tag handed out
            for (int a : by_rank[r])
                for (auto& kv : recv[i][a])
                {
                    const int32_t rr = doms[index_of[kv.first]].rank;
                    auto it = last_tag.find(rr);
                    const int32_t tag = it == last_tag.end() ? 0 : it->second + 1;
                    last_tag[rr] = tag;
                    tag_of[{kv.first, doms[a].id}] = tag;
                    if (r == my_rank) my_max_tag = std::max(my_max_tag, tag);
                }
        }
        auto& ps = out[i];
        ps.kind = 0;
        ps.dim = dim;
        ps.max_tag = my_max_tag;
        ps.my_rank = my_rank;
        if (my_rank < 0 || my_rank >= world) continue;
        for (int a : by_rank[my_rank])
        {
            domain_pattern p;
            p.id = doms[a].id;
            for (auto& kv : recv[i][a])
            {
                halo_entry e;
                e.key = {kv.first, doms[index_of[kv.first]].rank, tag_of.at({kv.first, p.id})};
                e.boxes = kv.second;
                p.recv.push_back(std::move(e));
            }
            for (auto& kv : send[i][a])
            {
                auto t = tag_of.find({p.id, kv.first});
                if (t == tag_of.end())
                    throw std::runtime_error("staged pattern: inconsistent domain lookup (a "
                                             "neighbour does not name this domain back)");
                halo_entry e;
                e.key = {kv.first, doms[index_of[kv.first]].rank, t->second};
                e.boxes = kv.second;
                p.send.push_back(std::move(e));
            }
            ps.doms.push_back(std::move(p));
        }
    }
}
}  // namespace ghx
