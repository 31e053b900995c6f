// ghex_amd/data_descriptor.hpp — header-only C++ adaptor: GHEX's unstructured data-descriptor
// concept on top of the C ABI of libghx.so (include/ghx.h).
//
// Replaces ghex::unstructured::data_descriptor<ghex::gpu, DomainId, Idx, T>
// (include/ghex/unstructured/user_concepts.hpp:526-667): same constructor arguments, same
// queries (domain_id(), domain_size(), num_components(), levels_first(), data(),
// device_id()), and the concept's
//     pack(T* buffer, const IndexContainer& c, void* stream_ptr)
//     unpack(const T* buffer, const IndexContainer& c, void* stream_ptr)
// where IndexContainer is a range of iteration spaces with `.local_indices()` (a host-readable
// contiguous vector of 4- or 8-byte integer local ids, ghex's
// unstructured::pattern::iteration_space, include/ghex/unstructured/pattern.hpp:53-90). As in
// the reference, the buffer is NOT advanced between iteration spaces (there is exactly one per
// neighbour, unstructured/pattern.hpp:324-325). Each list becomes one fused libghx launch with
// the indices resident in device memory (the reference reads them from managed memory).
//
// Plans: the first pack/unpack of an index list uploads it once (ghx_uplan_create); later calls
// with the same list find the plan by the list's address, length and index width, and confirm
// the list is unchanged by comparing it with a host copy kept with the plan (a memcmp: exact, so
// a list rebuilt at a freed list's address, e.g. by a new pattern, always gets a new plan; about
// 30 us per 500k-entry list, tools/udata_cost.hip). A caller that keeps the reference's contract —
// the pattern's index containers are immutable and outlive every exchange that uses them
// (include/ghex/pattern_container.hpp:84-87) — may call assume_immutable_index_lists(true):
// then 16 sampled entries are compared instead (O(1) host work per call), and a list changed in
// place, or rebuilt at the same address, needs forget_plans(). At most max_plans() plans are
// kept (least recently used dropped first; each holds a device copy of its list), so rebuilding
// patterns does not grow device memory without bound. Copies of a descriptor share its plans
// (guarded by a mutex). (The plain C entry points ghx_unstructured_pack/unpack compare the whole
// list on every call too.)
//
// Depends only on <ghx.h> and the standard library; link with -lghx.
#pragma once

#include <ghx.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

namespace ghex_amd
{
namespace unstructured
{
inline void check_u(int rc, const char* what)
{
    if (rc != GHX_OK)
        throw std::runtime_error(std::string(what) + " failed: " + ghx_last_error());
}

template<typename DomainId, typename T>
class data_descriptor
{
  public:  // member types (user_concepts.hpp:529-533)
    using value_type = T;
    using domain_id_type = DomainId;
    using device_id_type = int;

  private:
    domain_id_type m_domain_id;
    std::size_t m_domain_size;
    int m_levels;
    bool m_levels_first;
    std::size_t m_index_stride;
    std::size_t m_level_stride;
    value_type* m_values;
    device_id_type m_device_id;
    ghx_udata_desc m_desc{};
    // (list address, length, index bytes, direction) -> plan; shared by copies of the descriptor
    using plan_key = std::tuple<const void*, std::size_t, int32_t, int32_t>;
    static constexpr int kSamples = 16;
    struct cached
    {
        std::shared_ptr<ghx_uplan> plan;
        std::vector<char> content;  // the list's bytes (exact check), empty in sampled mode
        int64_t sample[kSamples];   // entries at i * (n - 1) / (kSamples - 1)
        uint64_t used = 0;          // LRU stamp
    };
    struct plan_cache
    {
        std::mutex mtx;
        std::map<plan_key, cached> map;
        uint64_t clock = 0;
        std::size_t max_plans = 64;
        bool trust = false;  // assume_immutable_index_lists
    };
    std::shared_ptr<plan_cache> m_plans = std::make_shared<plan_cache>();

  public:
    /** values: device pointer to domain_size * levels elements (plus padding when
     * outer_stride is given); levels_first: levels of one index are contiguous; outer_stride:
     * distance between consecutive indices (levels_first) or levels (levels last), 0 = dense.
     * (user_concepts.hpp:547-566) */
    template<typename Domain>
    data_descriptor(const Domain& domain, value_type* values, int levels = 1,
                    bool levels_first = true, std::size_t outer_stride = 0, device_id_type device_id = 0)
    : data_descriptor(domain.domain_id(), domain.size(), values, levels, levels_first,
                      outer_stride, device_id)
    {
    }

    data_descriptor(domain_id_type domain_id, std::size_t domain_size, value_type* values,
                    int levels = 1, bool levels_first = true, std::size_t outer_stride = 0,
                    device_id_type device_id = 0)
    : m_domain_id{domain_id}
    , m_domain_size{domain_size}
    , m_levels{levels}
    , m_levels_first{levels_first}
    , m_index_stride{levels_first ? (outer_stride ? outer_stride : std::size_t(levels)) : 1u}
    , m_level_stride{levels_first ? 1u : (outer_stride ? outer_stride : domain_size)}
    , m_values{values}
    , m_device_id{device_id}
    {
        if (levels < 1) throw std::runtime_error("levels must be >= 1");
        m_desc.elem_size = int32_t(sizeof(T));
        m_desc.levels = levels;
        m_desc.levels_first = levels_first ? 1 : 0;
        m_desc.index_stride = int64_t(m_index_stride);
        m_desc.level_stride = int64_t(m_level_stride);
    }

    domain_id_type domain_id() const noexcept { return m_domain_id; }
    std::size_t domain_size() const noexcept { return m_domain_size; }
    int num_components() const noexcept { return m_levels; }
    bool levels_first() const noexcept { return m_levels_first; }
    value_type* data() const noexcept { return m_values; }
    device_id_type device_id() const noexcept { return m_device_id; }
    const ghx_udata_desc& desc() const noexcept { return m_desc; }

    template<typename IndexContainer>
    void pack(value_type* buffer, const IndexContainer& c, void* stream_ptr)
    {
        for (const auto& is : c) run(is.local_indices(), 0, buffer, stream_ptr);
    }

    template<typename IndexContainer>
    void unpack(const value_type* buffer, const IndexContainer& c, void* stream_ptr)
    {
        for (const auto& is : c)
            run(is.local_indices(), 1, const_cast<value_type*>(buffer), stream_ptr);
    }

    // drop the cached plans (after an index list was changed in place, in sampled mode)
    void forget_plans()
    {
        std::lock_guard<std::mutex> g(m_plans->mtx);
        m_plans->map.clear();
    }

    // true: trust the reference's contract that index lists are immutable while cached and
    // check 16 sampled entries per call instead of the whole list (see the header comment)
    void assume_immutable_index_lists(bool on)
    {
        std::lock_guard<std::mutex> g(m_plans->mtx);
        if (on != m_plans->trust) m_plans->map.clear();  // entries carry the other mode's check
        m_plans->trust = on;
    }

    // plans kept at most (least recently used dropped first); >= 1
    void set_max_plans(std::size_t n)
    {
        std::lock_guard<std::mutex> g(m_plans->mtx);
        m_plans->max_plans = std::max<std::size_t>(1, n);
        evict();
    }
    std::size_t max_plans() const { return m_plans->max_plans; }
    std::size_t num_plans() const
    {
        std::lock_guard<std::mutex> g(m_plans->mtx);
        return m_plans->map.size();
    }

  private:
    // drop least recently used plans beyond the bound (caller holds the mutex); a plan still
    // referenced by a running call stays alive through its shared_ptr
    void evict()
    {
        auto& m = m_plans->map;
        while (m.size() > m_plans->max_plans)
            m.erase(std::min_element(m.begin(), m.end(), [](const auto& a, const auto& b) {
                return a.second.used < b.second.used;
            }));
    }

    template<typename V>
    void run(const V& l, int32_t dir, value_type* buffer, void* stream_ptr)
    {
        if (l.empty()) return;
        const plan_key key{static_cast<const void*>(l.data()), l.size(), lid_bytes(l), dir};
        const std::size_t nbytes = l.size() * std::size_t(lid_bytes(l));
        const char* raw = reinterpret_cast<const char*>(l.data());
        int64_t sample[kSamples];
        for (int i = 0; i < kSamples; ++i)
            sample[i] = int64_t(l[(l.size() - 1) * std::size_t(i) / (kSamples - 1)]);
        std::shared_ptr<ghx_uplan> plan;  // held: a concurrent forget_plans() cannot free it
        {
            std::lock_guard<std::mutex> g(m_plans->mtx);
            const bool trust = m_plans->trust;
            auto it = m_plans->map.find(key);
            if (it != m_plans->map.end())
            {
                const cached& c = it->second;
                const bool same = trust ? std::equal(sample, sample + kSamples, c.sample)
                                        : c.content.size() == nbytes &&
                                              std::memcmp(c.content.data(), raw, nbytes) == 0;
                if (!same)
                {
                    m_plans->map.erase(it);  // a different list at the same address
                    it = m_plans->map.end();
                }
            }
            if (it == m_plans->map.end())
            {
                std::vector<int64_t> wide(l.begin(), l.end());
                ghx_upack_entry e{};
                e.data = m_desc;
                e.field_slot = 0;
                e.buffer_slot = 0;
                e.buffer_offset = 0;
                e.lids = wide.data();
                e.n_lids = int64_t(wide.size());
                ghx_uplan* p = nullptr;
                check_u(ghx_uplan_create(&e, 1, dir, &p), "ghx_uplan_create");
                cached c;
                c.plan.reset(p, ghx_uplan_destroy);
                if (!trust) c.content.assign(raw, raw + nbytes);
                std::copy(sample, sample + kSamples, c.sample);
                it = m_plans->map.emplace(key, std::move(c)).first;
            }
            it->second.used = ++m_plans->clock;
            plan = it->second.plan;
            evict();
        }
        void* f[1] = {m_values};
        void* b[1] = {buffer};
        check_u(ghx_uplan_execute(plan.get(), f, 1, b, 1, stream_of(stream_ptr)),
                dir ? "unpack: ghx_uplan_execute" : "pack: ghx_uplan_execute");
    }

    template<typename V>
    static int32_t lid_bytes(const V&)
    {
        using I = std::decay_t<decltype(*std::declval<const V&>().data())>;
        static_assert(std::is_integral<I>::value && (sizeof(I) == 4 || sizeof(I) == 8),
                      "local indices must be 4- or 8-byte integers");
        return int32_t(sizeof(I));
    }

    static ghx_stream stream_of(void* arg) { return arg ? *static_cast<ghx_stream*>(arg) : nullptr; }
};
}  // namespace unstructured
}  // namespace ghex_amd
