// ghx_upattern.cpp — make_pattern<unstructured::grid> as the reference runs it: every rank
// passes only ITS OWN domains; what travels between ranks is each domain's reduced halo (its halo
// gids) and, back to each halo's owner, the subset of those gids another rank holds as inner
// cells (include/ghex/unstructured/pattern.hpp:187-370). No rank ever sees another rank's full
// gid list, so setup memory and time per rank are O(own cells + all ranks' halos), not
// O(all ranks' cells).
//
// The caller moves the bytes (torch.distributed, a C++ transport, threads of one process); this
// file is the per-rank arithmetic of the three steps:
//   1. tags from the global max domain id and max domains per rank (pattern.hpp:218-233);
//   2. for every rank's reduced halos (its distributed_for_each ring, :284-330): the local ids of
//      the halo gids that are inner cells of each of my domains, in the halo's order -> my send
//      halos, plus the gid list to ship to the halo's owner;
//   3. for every gid list received (:337-365): make_outer_lids on the receiving domain -> my
//      receive halos.
// The gid -> lid maps are flat open-addressing tables (int64 keys, linear probing) instead of
// std::unordered_map/multimap: a 10.5M-cell domain takes ~270 MB and one probe per lookup.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "ghx_guard.hpp"
#include "ghx_pattern.hpp"

namespace ghx
{
namespace
{
// gid -> int64 table. The key INT64_MIN marks an empty slot (such a gid is refused).
class gid_table
{
    static constexpr int64_t kEmpty = INT64_MIN;
    std::vector<int64_t> m_keys, m_vals;
    uint64_t m_mask = 0;
    size_t m_n = 0;

    static uint64_t hash(int64_t k)
    {
        uint64_t x = uint64_t(k) + 0x9e3779b97f4a7c15ull;  // splitmix64 finaliser
        x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
        x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
        return x ^ (x >> 31);
    }

  public:
    void reserve(size_t items)
    {
        size_t cap = 16;
        while (cap * 7 < items * 10) cap <<= 1;  // load factor <= 0.7
        m_keys.assign(cap, kEmpty);
        m_vals.assign(cap, 0);
        m_mask = cap - 1;
        m_n = 0;
    }
    size_t size() const { return m_n; }
    size_t capacity() const { return m_keys.size(); }

    const int64_t* find(int64_t k) const
    {
        if (m_keys.empty()) return nullptr;
        for (uint64_t s = hash(k) & m_mask;; s = (s + 1) & m_mask)
        {
            if (m_keys[s] == k) return &m_vals[s];
            if (m_keys[s] == kEmpty) return nullptr;
        }
    }
    // (value slot, inserted)
    std::pair<int64_t*, bool> insert(int64_t k, int64_t v)
    {
        if (k == kEmpty) throw std::runtime_error("global index INT64_MIN is not supported");
        if ((m_n + 1) * 10 > capacity() * 7) grow();
        for (uint64_t s = hash(k) & m_mask;; s = (s + 1) & m_mask)
        {
            if (m_keys[s] == k) return {&m_vals[s], false};
            if (m_keys[s] == kEmpty)
            {
                m_keys[s] = k;
                m_vals[s] = v;
                ++m_n;
                return {&m_vals[s], true};
            }
        }
    }
    template<typename F>
    void for_each(F&& f) const
    {
        for (size_t s = 0; s < m_keys.size(); ++s)
            if (m_keys[s] != kEmpty) f(m_keys[s], m_vals[s]);
    }

  private:
    void grow()
    {
        std::vector<int64_t> k, v;
        k.swap(m_keys);
        v.swap(m_vals);
        reserve(std::max<size_t>(16, (m_n + 1) * 2));
        for (size_t s = 0; s < k.size(); ++s)
            if (k[s] != kEmpty) insert(k[s], v[s]);
    }
};

unsigned num_bits(unsigned n) { return n ? 1u + num_bits(n >> 1) : 1u; }
}  // namespace
}  // namespace ghx

// unstructured::domain_descriptor (include/ghex/unstructured/user_concepts.hpp:37-176)
struct ghx_udomain
{
    int32_t id = 0;
    int64_t size = 0;
    ghx::gid_table inner;  // gid -> lid (inner cells)
    // outer cells as an unordered_multimap: entries in storage order, each gid's chain starts at
    // its LAST entry and runs backwards, which is libstdc++'s equal_range order for repeated keys
    // (an equal key is linked in front of its range, _M_insert_multi_node)
    ghx::gid_table outer_head;  // gid -> index of its chain's first entry
    std::vector<int64_t> o_lid, o_gid, o_next;

    ghx_udomain(int32_t id_, const int64_t* gids, int64_t n, const int64_t* outer_lids,
                int64_t n_outer)
    : id{id_}
    , size{n}
    {
        // domain_descriptor ctor (user_concepts.hpp:145-174)
        std::vector<uint8_t> is_outer(size_t(n), 0);
        for (int64_t k = 0; k < n_outer; ++k)
        {
            const int64_t l = outer_lids[k];
            if (l < 0 || l >= n)
                throw ghx::invalid("outer local index " + std::to_string(l) + " outside the domain");
            if (is_outer[size_t(l)]) throw std::runtime_error("repeated outer (local) index");
            is_outer[size_t(l)] = 1;
        }
        inner.reserve(size_t(n - n_outer));
        outer_head.reserve(size_t(n_outer));
        o_lid.reserve(size_t(n_outer));
        for (int64_t lid = 0; lid < n; ++lid)
        {
            const int64_t gid = gids[lid];
            if (is_outer[size_t(lid)])
            {
                const int64_t e = int64_t(o_lid.size());
                auto ins = outer_head.insert(gid, e);
                o_next.push_back(ins.second ? -1 : *ins.first);
                if (!ins.second) *ins.first = e;
                o_lid.push_back(lid);
                o_gid.push_back(gid);
            }
            else if (!inner.insert(gid, lid).second)
                throw std::runtime_error("repeated inner (global) index");
        }
    }

    // domain_descriptor::make_outer_lids (user_concepts.hpp:88-113). Appends the lids, and the
    // gids that had one, in the order of `g` (gids that are not outer cells are skipped).
    void make_outer_lids(const int64_t* g, int64_t n, std::vector<int64_t>* lids,
                         std::vector<int64_t>* kept) const
    {
        ghx::gid_table count;
        count.reserve(size_t(std::min<int64_t>(n, int64_t(o_lid.size())) + 1));
        for (int64_t k = 0; k < n; ++k)
        {
            const int64_t gid = g[k];
            const int64_t* head = outer_head.find(gid);
            if (!head) continue;
            auto c = count.insert(gid, 0);
            int64_t e = *head;
            if (!c.second)
            {
                const int64_t steps = ++*c.first;
                for (int64_t s = 0; s < steps && e >= 0; ++s) e = o_next[size_t(e)];
                if (e < 0)
                    throw std::runtime_error("halo gid does not have an associated lid in the domain");
            }
            if (lids) lids->push_back(o_lid[size_t(e)]);
            if (kept) kept->push_back(gid);
        }
        count.for_each([&](int64_t gid, int64_t c) {
            int64_t len = 0;
            for (int64_t e = *outer_head.find(gid); e >= 0; e = o_next[size_t(e)]) ++len;
            if (c + 1 != len) throw std::runtime_error("halo gid occurs not often enough");
        });
    }
};

// The per-rank state of one make_pattern<unstructured::grid> call.
struct ghx_upattern
{
    struct send_record  // the reference's recv_halo_data + send_indices (pattern.hpp:267-326)
    {
        int32_t src_id, dst_id, dst_rank, tag;
        std::vector<int64_t> gids;
    };
    std::vector<const ghx_udomain*> doms;
    int32_t my_rank = 0;
    unsigned shift = 1;
    int32_t max_tag = 0;
    std::vector<std::map<std::pair<int32_t, int32_t>, ghx::halo_entry>> send, recv;
    std::vector<send_record> records;
    bool finished = false;

    int32_t make_tag(unsigned src_local, int32_t tgt) const
    {
        return int32_t((src_local << shift) | unsigned(tgt));
    }

    // Two halos of one local domain with one peer rank under the same tag: the reference's tag
    // layout (src_local << num_bits(max_num_domains)) | dst_id (unstructured/pattern.hpp:
    // 230-232) cannot tell them apart once a domain id needs more than `shift` bits and a rank
    // holds several domains. The reference's map insert keeps the first and drops the other
    // (its exchange then hangs or moves wrong data); here setup fails on the rank that sees it.
    std::string collision(int32_t local_id, int32_t peer, int32_t tag) const
    {
        return "unstructured make_pattern: two halos of domain " + std::to_string(local_id) +
               " with rank " + std::to_string(peer) + " share tag " + std::to_string(tag) +
               " (tag = source index << " + std::to_string(shift) +
               " | target domain id: with several domains per rank, domain ids must be below " +
               std::to_string(1u << shift) + ")";
    }
};

namespace
{
int need(const void* p, const char* what)
{
    if (!p) throw ghx::invalid(std::string("null argument: ") + what);
    return 0;
}
void need_open(const ghx_upattern* b)
{
    need(b, "builder");
    if (b->finished) throw ghx::invalid("make_pattern builder already finished");
}
}  // namespace

extern "C" {

int ghx_udomain_create(int32_t id, const int64_t* gids, int64_t n_gids, const int64_t* outer_lids,
                       int64_t n_outer, ghx_udomain** out)
{
    return ghx::guarded([&] {
        need(out, "out");
        if (n_gids < 0 || n_outer < 0 || n_outer > n_gids) throw ghx::invalid("bad domain sizes");
        if (n_gids) need(gids, "gids");
        if (n_outer) need(outer_lids, "outer_lids");
        if (id < 0) throw ghx::invalid("domain ids must be >= 0 (they are packed into tags)");
        *out = new ghx_udomain(id, gids, n_gids, outer_lids, n_outer);
        return GHX_OK;
    });
}

int ghx_udomain_destroy(ghx_udomain* d)
{
    delete d;
    return GHX_OK;
}

int ghx_udomain_info(const ghx_udomain* d, int32_t* id, int64_t* size, int64_t* inner_size,
                     int64_t* n_outer)
{
    return ghx::guarded([&] {
        need(d, "domain");
        if (id) *id = d->id;
        if (size) *size = d->size;
        if (inner_size) *inner_size = int64_t(d->inner.size());
        if (n_outer) *n_outer = int64_t(d->o_lid.size());
        return GHX_OK;
    });
}

int ghx_udomain_halo(const ghx_udomain* d, const int64_t* gen_gids, int64_t n_gen,
                     int64_t* halo_gids, int64_t cap, int64_t* n_halo)
{
    return ghx::guarded([&] {
        need(d, "domain");
        need(n_halo, "n_halo");
        const bool all = n_gen < 0;
        if (!all && n_gen > 0) need(gen_gids, "gen_gids");
        std::vector<int64_t> kept;
        // halo_generator::operator() (user_concepts.hpp:251-255)
        if (all) d->make_outer_lids(d->o_gid.data(), int64_t(d->o_gid.size()), nullptr, &kept);
        else d->make_outer_lids(gen_gids, n_gen, nullptr, &kept);
        *n_halo = int64_t(kept.size());
        if (int64_t(kept.size()) > cap) throw ghx::invalid("halo_gids: capacity too small");
        if (!kept.empty())
        {
            need(halo_gids, "halo_gids");
            std::memcpy(halo_gids, kept.data(), kept.size() * sizeof(int64_t));
        }
        return GHX_OK;
    });
}

int ghx_upattern_create(const ghx_udomain* const* domains, int32_t n_domains, int32_t my_rank,
                        int32_t max_num_domains, int32_t max_domain_id, ghx_upattern** out)
{
    return ghx::guarded([&] {
        need(out, "out");
        if (n_domains < 1) throw ghx::invalid("need at least one local domain");
        need(domains, "domains");
        if (max_num_domains < n_domains || max_domain_id < 0)
            throw ghx::invalid("max_num_domains / max_domain_id are global maxima over all ranks");
        auto b = std::make_unique<ghx_upattern>();
        for (int32_t i = 0; i < n_domains; ++i)
        {
            need(domains[i], "domain");
            if (domains[i]->id > max_domain_id) throw ghx::invalid("domain id above max_domain_id");
            b->doms.push_back(domains[i]);
        }
        b->my_rank = my_rank;
        b->shift = ghx::num_bits(unsigned(max_num_domains));
        b->max_tag = b->make_tag(unsigned(max_num_domains), max_domain_id);
        b->send.resize(size_t(n_domains));
        b->recv.resize(size_t(n_domains));
        *out = b.release();
        return GHX_OK;
    });
}

int ghx_upattern_add_halos(ghx_upattern* b, int32_t rank, int32_t n_domains,
                           const int32_t* domain_ids, const int64_t* halo_sizes,
                           const int64_t* halo_gids, int64_t* n_records)
{
    return ghx::guarded([&] {
        need_open(b);
        if (n_domains < 0 || rank < 0) throw ghx::invalid("bad rank / domain count");
        if (n_domains) {
            need(domain_ids, "domain_ids");
            need(halo_sizes, "halo_sizes");
        }
        int64_t off = 0;
        for (int32_t k = 0; k < n_domains; ++k)
        {
            if (halo_sizes[k] < 0) throw ghx::invalid("negative halo size");
            if (halo_sizes[k]) need(halo_gids, "halo_gids");
            const int64_t* first = halo_gids + off;
            for (size_t i = 0; i < b->doms.size(); ++i)
            {
                const ghx_udomain& d = *b->doms[i];
                const int32_t tag = b->make_tag(unsigned(i), domain_ids[k]);
                ghx::halo_entry e;
                std::vector<int64_t> g;
                for (int64_t j = 0; j < halo_sizes[k]; ++j)
                    if (const int64_t* lid = d.inner.find(first[j]))
                    {
                        e.lids.push_back(*lid);
                        g.push_back(first[j]);
                    }
                if (e.lids.empty()) continue;
                e.key = {domain_ids[k], rank, tag};
                if (!b->send[i].emplace(std::make_pair(rank, tag), std::move(e)).second)
                    throw std::runtime_error(b->collision(d.id, rank, tag));
                b->records.push_back({d.id, domain_ids[k], rank, tag, std::move(g)});
            }
            off += halo_sizes[k];
        }
        if (n_records) *n_records = int64_t(b->records.size());
        return GHX_OK;
    });
}

int ghx_upattern_record(const ghx_upattern* b, int64_t k, int32_t* src_id, int32_t* dst_id,
                        int32_t* dst_rank, int32_t* tag, int64_t* n_gids, const int64_t** gids)
{
    return ghx::guarded([&] {
        need(b, "builder");
        if (k < 0 || k >= int64_t(b->records.size())) throw ghx::invalid("record index out of range");
        const auto& r = b->records[size_t(k)];
        if (src_id) *src_id = r.src_id;
        if (dst_id) *dst_id = r.dst_id;
        if (dst_rank) *dst_rank = r.dst_rank;
        if (tag) *tag = r.tag;
        if (n_gids) *n_gids = int64_t(r.gids.size());
        if (gids) *gids = r.gids.data();
        return GHX_OK;
    });
}

int ghx_upattern_add_recv(ghx_upattern* b, int32_t src_rank, int32_t src_id, int32_t dst_id,
                          int32_t tag, const int64_t* gids, int64_t n_gids)
{
    return ghx::guarded([&] {
        need_open(b);
        if (n_gids < 0) throw ghx::invalid("negative gid count");
        if (n_gids) need(gids, "gids");
        for (size_t i = 0; i < b->doms.size(); ++i)
        {
            if (b->doms[i]->id != dst_id) continue;
            ghx::halo_entry e;
            b->doms[i]->make_outer_lids(gids, n_gids, &e.lids, nullptr);
            if (int64_t(e.lids.size()) != n_gids)
                throw std::runtime_error("received halo gids that are not outer cells of domain " +
                                         std::to_string(dst_id));
            e.key = {src_id, src_rank, tag};
            if (!b->recv[i].emplace(std::make_pair(src_rank, tag), std::move(e)).second)
                throw std::runtime_error(b->collision(dst_id, src_rank, tag));
            return GHX_OK;
        }
        throw ghx::invalid("no local domain with id " + std::to_string(dst_id));
    });
}

int ghx_upattern_finish(ghx_upattern* b, ghx_pattern** out)
{
    return ghx::guarded([&] {
        need_open(b);
        need(out, "out");
        auto p = std::make_unique<ghx_pattern>();
        p->kind = 1;
        p->dim = 1;
        p->max_tag = b->max_tag;
        p->my_rank = b->my_rank;
        for (size_t i = 0; i < b->doms.size(); ++i)
        {
            ghx::domain_pattern dp;
            dp.id = b->doms[i]->id;
            for (auto& kv : b->send[i]) dp.send.push_back(std::move(kv.second));
            for (auto& kv : b->recv[i]) dp.recv.push_back(std::move(kv.second));
            p->doms.push_back(std::move(dp));
        }
        b->finished = true;
        b->send.clear();
        b->recv.clear();
        *out = p.release();
        return GHX_OK;
    });
}

int ghx_upattern_destroy(ghx_upattern* b)
{
    delete b;
    return GHX_OK;
}

}  // extern "C"
