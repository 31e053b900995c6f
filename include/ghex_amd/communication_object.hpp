// ghex_amd/communication_object.hpp — the reference's host-side exchange API in C++ over the C
// ABI of libghx.so: context, domain descriptors, halo generators, make_pattern, pattern(field)
// -> buffer_info, make_communication_object, exchange(...) -> handle.wait().
//
// Mirrors (paths relative to the GHEX v0.8.0 tree):
//   ghex::context                                    include/ghex/context.hpp
//   structured::regular::{domain_descriptor, halo_generator}
//                                                    include/ghex/structured/regular/{domain_descriptor,halo_generator}.hpp
//   unstructured::{domain_descriptor, halo_generator} include/ghex/unstructured/user_concepts.hpp:37-256
//   make_pattern<grid>(ctx, halo_gen, domains)       include/ghex/pattern_container.hpp:112-120
//   pattern_container::operator()(field) -> buffer_info   pattern_container.hpp:88-95, buffer_info.hpp
//   communication_object::exchange / schedule_exchange, communication_handle::wait / is_ready /
//   schedule_wait                                    include/ghex/communication_object.hpp:78-130, 271-330, 801-968
//
// What an exchange does (the reference's stream-aware branch, communication_object.hpp:703-767):
//   plan once per set of fields (ghx_exchange_create = communication_object::allocate: one buffer
//   per domain pair, fields in argument order with alignof padding, tags = pattern tag + a
//   per-container offset); then per exchange, on the object's stream:
//     all messages self messages -> ONE fused pack+unpack launch (ghx_exchange_self);
//     otherwise -> ONE pack launch for every send buffer (ghx_exchange_pack), one transport group
//     of the peer messages (rccl_transport: ncclSend/ncclRecv over xGMI), ONE unpack launch for
//     every receive buffer (ghx_exchange_unpack). Self messages never leave the device: their
//     receive buffer IS the send buffer.
// The host never blocks inside exchange(); handle.wait() synchronises with the stream.
// Errors throw std::runtime_error (the reference's convention). Link with -lghx (+ -lrccl for
// rccl_transport).
#pragma once

#include <ghx.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "transport.hpp"

namespace ghex_amd
{
inline void check_ghx(int rc, const char* what)
{
    if (rc != GHX_OK) throw std::runtime_error(std::string(what) + " failed: " + ghx_last_error());
}

// ghx_epochs_status codes as text (the zero-copy exchanges' failures)
inline std::string epochs_error_text(std::int32_t err)
{
    switch (err)
    {
        case 1: return "a wait of the open phase timed out (a target never opened its memory)";
        case 2: return "a wait of the close phase timed out (a source never completed its writes)";
        case 3: return "the close kernel did not reach every XCD in time (fence placement)";
        default: break;
    }
    if ((err & 0xff) == 4)
        return "node-local rank " + std::to_string(err >> 8) +
               " failed an epoch wait: its later writes may have overlapped this rank's reads";
    return "epoch error code " + std::to_string(err);
}

// ghex::context (include/ghex/context.hpp): the process group the patterns and exchanges span.
class context
{
    transport* m_transport;

  public:
    explicit context(transport& t)
    : m_transport{&t}
    {
    }
    int rank() const { return m_transport->rank(); }
    int size() const { return m_transport->size(); }
    transport& get_transport() const { return *m_transport; }
};

namespace detail
{
template<typename T>
void put(std::vector<char>& out, const T& v)
{
    const char* p = reinterpret_cast<const char*>(&v);
    out.insert(out.end(), p, p + sizeof(T));
}
template<typename T>
T get(const std::vector<char>& in, std::size_t& pos)
{
    if (pos + sizeof(T) > in.size()) throw std::runtime_error("malformed all_gather payload");
    T v;
    std::memcpy(&v, in.data() + pos, sizeof(T));
    pos += sizeof(T);
    return v;
}
}  // namespace detail

// A pattern container: the halo maps of this rank's domains (one pattern per local domain), owned
// by libghx (ghx_pattern). pattern(field) selects the pattern of the field's domain.
class pattern_container;

template<typename Field>
struct buffer_info
{
    const pattern_container* pattern;
    int local_index;
    Field* field;
};

class pattern_container
{
    std::shared_ptr<ghx_pattern> m_p;
    std::vector<int> m_ids;
    int m_max_tag = 0;

  public:
    explicit pattern_container(ghx_pattern* p)
    : m_p{p, [](ghx_pattern* q) { ghx_pattern_destroy(q); }}
    {
        int32_t n = 0;
        check_ghx(ghx_pattern_num_domains(p, &n), "ghx_pattern_num_domains");
        for (int32_t i = 0; i < n; ++i)
        {
            int32_t id = 0;
            check_ghx(ghx_pattern_domain_id(p, i, &id), "ghx_pattern_domain_id");
            m_ids.push_back(id);
        }
        int32_t mt = 0;
        check_ghx(ghx_pattern_max_tag(p, &mt), "ghx_pattern_max_tag");
        m_max_tag = mt;
    }
    const ghx_pattern* handle() const { return m_p.get(); }
    int max_tag() const { return m_max_tag; }  // pattern_container::max_tag (:78-83)
    std::size_t size() const { return m_ids.size(); }

    // pattern_container::operator()(field) (pattern_container.hpp:88-95)
    template<typename Field>
    buffer_info<Field> operator()(Field& field) const
    {
        for (std::size_t i = 0; i < m_ids.size(); ++i)
            if (m_ids[i] == int(field.domain_id())) return {this, int(i), &field};
        throw std::runtime_error("field's domain id is not a local domain of this pattern");
    }
};

namespace structured
{
namespace regular
{
// structured::regular::domain_descriptor (3-D, int ids), inclusive first/last global coords.
class domain_descriptor
{
    int m_id;
    std::array<int, 3> m_first, m_last;

  public:
    domain_descriptor(int id, const std::array<int, 3>& first, const std::array<int, 3>& last)
    : m_id{id}
    , m_first{first}
    , m_last{last}
    {
    }
    int domain_id() const { return m_id; }
    const std::array<int, 3>& first() const { return m_first; }
    const std::array<int, 3>& last() const { return m_last; }
};

// structured::regular::halo_generator (halo_generator.hpp:61-90): global box, halos
// (dim0-, dim0+, dim1-, dim1+, dim2-, dim2+), periodicity.
struct halo_generator
{
    std::array<int, 3> global_first, global_last;
    std::array<int, 6> halos;
    std::array<bool, 3> periodic;
};

// make_pattern<structured::grid> (include/ghex/structured/pattern.hpp:214-571): the domains of
// all ranks are all-gathered through the context's transport, libghx intersects.
inline pattern_container make_pattern(context& ctx, const halo_generator& hg,
                                      const std::vector<domain_descriptor>& domains)
{
    std::vector<char> mine;
    detail::put(mine, std::int32_t(domains.size()));
    for (const auto& d : domains)
    {
        detail::put(mine, std::int32_t(d.domain_id()));
        for (int k = 0; k < 3; ++k) detail::put(mine, std::int32_t(d.first()[k]));
        for (int k = 0; k < 3; ++k) detail::put(mine, std::int32_t(d.last()[k]));
    }
    const auto all = ctx.get_transport().all_gather(mine);
    std::vector<ghx_regular_domain> doms;
    for (std::size_t r = 0; r < all.size(); ++r)
    {
        std::size_t pos = 0;
        const auto n = detail::get<std::int32_t>(all[r], pos);
        for (std::int32_t i = 0; i < n; ++i)
        {
            ghx_regular_domain g{};
            g.id = detail::get<std::int32_t>(all[r], pos);
            g.rank = std::int32_t(r);
            for (int k = 0; k < 3; ++k) g.first[k] = detail::get<std::int32_t>(all[r], pos);
            for (int k = 0; k < 3; ++k) g.last[k] = detail::get<std::int32_t>(all[r], pos);
            doms.push_back(g);
        }
    }
    std::int32_t per[3];
    for (int k = 0; k < 3; ++k) per[k] = hg.periodic[std::size_t(k)] ? 1 : 0;
    ghx_pattern* p = nullptr;
    check_ghx(ghx_regular_pattern_create(3, doms.data(), std::int32_t(doms.size()),
                                         hg.global_first.data(), hg.global_last.data(),
                                         hg.halos.data(), per, ctx.rank(), &p),
              "ghx_regular_pattern_create");
    return pattern_container(p);
}
}  // namespace regular
}  // namespace structured

namespace unstructured
{
// unstructured::domain_descriptor (user_concepts.hpp:143-175): all global ids in storage order
// and the local ids of the outer (halo) cells; the gid -> lid maps are built once in libghx
// (ghx_udomain_create).
class domain_descriptor
{
    int m_id;
    std::vector<std::int64_t> m_gids, m_outer;
    std::shared_ptr<ghx_udomain> m_h;

  public:
    domain_descriptor(int id, std::vector<std::int64_t> gids, std::vector<std::int64_t> outer_lids)
    : m_id{id}
    , m_gids(std::move(gids))
    , m_outer(std::move(outer_lids))
    {
        ghx_udomain* h = nullptr;
        check_ghx(ghx_udomain_create(id, m_gids.data(), std::int64_t(m_gids.size()), m_outer.data(),
                                     std::int64_t(m_outer.size()), &h),
                  "ghx_udomain_create");
        m_h.reset(h, [](ghx_udomain* q) { ghx_udomain_destroy(q); });
    }
    int domain_id() const { return m_id; }
    std::size_t size() const { return m_gids.size(); }
    const std::vector<std::int64_t>& gids() const { return m_gids; }
    const std::vector<std::int64_t>& outer_lids() const { return m_outer; }
    const ghx_udomain* handle() const { return m_h.get(); }
};

// unstructured::halo_generator (user_concepts.hpp:234-253): every outer gid (default) or an
// explicit list of halo gids.
struct halo_generator
{
    bool all_outer = true;
    std::vector<std::int64_t> gids;
};

// make_pattern<unstructured::grid> (include/ghex/unstructured/pattern.hpp:187-370): the
// reference's reduced-halo algorithm through the context's all_gather. Only halo gids travel:
// (1) max domain id / count, (2) every rank's reduced halos, (3) the gid lists of the send
// halos found in (2), which their receivers turn into outer lids.
inline pattern_container make_pattern(context& ctx, const halo_generator& hg,
                                      const std::vector<domain_descriptor>& domains)
{
    if (domains.empty()) throw std::runtime_error("make_pattern needs at least one local domain");
    auto& tr = ctx.get_transport();
    const int me = ctx.rank();
    std::int32_t max_id = 0;
    for (const auto& d : domains) max_id = std::max<std::int32_t>(max_id, d.domain_id());
    std::vector<char> meta;
    detail::put(meta, max_id);
    detail::put(meta, std::int32_t(domains.size()));
    std::int32_t g_max_id = 0, g_max_n = 0;
    for (const auto& m : tr.all_gather(meta))
    {
        std::size_t pos = 0;
        g_max_id = std::max(g_max_id, detail::get<std::int32_t>(m, pos));
        g_max_n = std::max(g_max_n, detail::get<std::int32_t>(m, pos));
    }
    std::vector<const ghx_udomain*> hs;
    for (const auto& d : domains) hs.push_back(d.handle());
    ghx_upattern* b = nullptr;
    check_ghx(ghx_upattern_create(hs.data(), std::int32_t(hs.size()), me, g_max_n, g_max_id, &b),
              "ghx_upattern_create");
    std::unique_ptr<ghx_upattern, int (*)(ghx_upattern*)> guard(b, ghx_upattern_destroy);
    // (2) reduced halos: [n][ids][sizes][gids...]
    std::vector<char> mine;
    detail::put(mine, std::int32_t(domains.size()));
    std::vector<std::vector<std::int64_t>> halos;
    for (const auto& d : domains)
    {
        const std::int64_t cap = hg.all_outer ? std::int64_t(d.outer_lids().size())
                                              : std::int64_t(hg.gids.size());
        std::vector<std::int64_t> h(std::size_t(std::max<std::int64_t>(cap, 1)));
        std::int64_t n = 0;
        check_ghx(ghx_udomain_halo(d.handle(), hg.all_outer ? nullptr : hg.gids.data(),
                                   hg.all_outer ? -1 : std::int64_t(hg.gids.size()), h.data(), cap,
                                   &n),
                  "ghx_udomain_halo");
        h.resize(std::size_t(n));
        detail::put(mine, std::int32_t(d.domain_id()));
        detail::put(mine, n);
        halos.push_back(std::move(h));
    }
    for (const auto& h : halos)
    {
        const char* p = reinterpret_cast<const char*>(h.data());
        mine.insert(mine.end(), p, p + h.size() * sizeof(std::int64_t));
    }
    const auto all = tr.all_gather(mine);
    std::int64_t n_rec = 0;
    for (std::size_t r = 0; r < all.size(); ++r)
    {
        std::size_t pos = 0;
        const auto n = detail::get<std::int32_t>(all[r], pos);
        std::vector<std::int32_t> ids;
        std::vector<std::int64_t> sizes, gids;
        for (std::int32_t i = 0; i < n; ++i)
        {
            ids.push_back(detail::get<std::int32_t>(all[r], pos));
            sizes.push_back(detail::get<std::int64_t>(all[r], pos));
        }
        for (auto s : sizes)
            for (std::int64_t k = 0; k < s; ++k) gids.push_back(detail::get<std::int64_t>(all[r], pos));
        check_ghx(ghx_upattern_add_halos(b, std::int32_t(r), n, ids.data(), sizes.data(),
                                         gids.data(), &n_rec),
                  "ghx_upattern_add_halos");
    }
    // (3) the send halos' gid lists to their receivers
    std::vector<char> recs;
    detail::put(recs, n_rec);
    for (std::int64_t k = 0; k < n_rec; ++k)
    {
        std::int32_t src_id, dst_id, dst_rank, tag;
        std::int64_t n = 0;
        const std::int64_t* g = nullptr;
        check_ghx(ghx_upattern_record(b, k, &src_id, &dst_id, &dst_rank, &tag, &n, &g),
                  "ghx_upattern_record");
        for (auto v : {src_id, dst_id, dst_rank, tag}) detail::put(recs, v);
        detail::put(recs, n);
        const char* p = reinterpret_cast<const char*>(g);
        recs.insert(recs.end(), p, p + std::size_t(n) * sizeof(std::int64_t));
    }
    const auto every = tr.all_gather(recs);
    for (std::size_t r = 0; r < every.size(); ++r)
    {
        std::size_t pos = 0;
        const auto n = detail::get<std::int64_t>(every[r], pos);
        for (std::int64_t k = 0; k < n; ++k)
        {
            const auto src_id = detail::get<std::int32_t>(every[r], pos);
            const auto dst_id = detail::get<std::int32_t>(every[r], pos);
            const auto dst_rank = detail::get<std::int32_t>(every[r], pos);
            const auto tag = detail::get<std::int32_t>(every[r], pos);
            const auto cnt = detail::get<std::int64_t>(every[r], pos);
            if (pos + std::size_t(cnt) * sizeof(std::int64_t) > every[r].size())
                throw std::runtime_error("malformed all_gather payload");
            if (dst_rank == me)
            {
                std::vector<std::int64_t> g(static_cast<std::size_t>(cnt));
                std::memcpy(g.data(), every[r].data() + pos, g.size() * sizeof(std::int64_t));
                check_ghx(ghx_upattern_add_recv(b, std::int32_t(r), src_id, dst_id, tag, g.data(),
                                                cnt),
                          "ghx_upattern_add_recv");
            }
            pos += std::size_t(cnt) * sizeof(std::int64_t);
        }
    }
    ghx_pattern* p = nullptr;
    check_ghx(ghx_upattern_finish(b, &p), "ghx_upattern_finish");
    return pattern_container(p);
}
}  // namespace unstructured

class communication_object;

// communication_handle (communication_object.hpp:78-130)
class communication_handle
{
    communication_object* m_co = nullptr;
    hipEvent_t m_done = nullptr;

  public:
    communication_handle() = default;
    communication_handle(communication_object* co, hipEvent_t done)
    : m_co{co}
    , m_done{done}
    {
    }
    inline void wait();
    inline bool is_ready();
    void progress() { (void)is_ready(); }
    // make `stream` wait for the exchange without blocking the host (:832-856, 918-945)
    void schedule_wait(hipStream_t stream)
    {
        if (m_done) check_hip(hipStreamWaitEvent(stream, m_done, 0), "hipStreamWaitEvent");
    }
};

struct communication_options
{
    bool fuse_self = true;                // all-self exchanges as one launch
    bool self_through_transport = false;  // route self messages through the transport too
                                          // (transport testing; oomph also sends to self)
    // per-peer pipeline (the reference's per-buffer streams + send as packed,
    // device/cuda/stream.hpp:25-73, communication_object.hpp:568-637, 703-767): each peer's
    // buffers packed on one of `max_streams` lanes, its group posted there
    // (transport::exchange_peer), its buffers unpacked there; peers in the global round order
    bool pipelined = false;
    int max_streams = 4;
    // direct (one process per rank, node-local peers, device buffers): the pack launch writes
    // each peer message straight into the receiver's buffer (IPC mapping; xGMI between GPUs),
    // device epochs (ghx_epochs_*: one close launch per exchange, the receive buffers double-
    // buffered by epoch parity) order it, the receiver unpacks locally — no transport step.
    // Setup at a plan's first exchange: receive buffers exported and imported over the
    // transport's all_gather (collective). The Python CommunicationObject(direct=True).
    bool direct = false;
    double epoch_timeout = 30.0;  // seconds an epoch wait may take before wait() throws
};

// communication_object<grid, domain_id> (make_communication_object, :1105-1112)
class communication_object
{
  public:
    using options = communication_options;

  private:
    struct buf
    {
        std::int32_t first_id, second_id, rank, tag;
        std::uint64_t size;
        void* data = nullptr;
        bool owned = true;
    };
    struct plan
    {
        ghx_exchange* ex = nullptr;
        std::vector<buf> send, recv;
        bool fused = false;
        bool mixed = false;  // self AND peer messages: ghx_exchange_pack_self / _unpack_peers
        std::vector<void*> sptr, rptr;
        std::vector<void*> dsptr;     // direct: peer-message entries = the receivers' buffers
        ghx_epochs* ep = nullptr;     // direct: this plan's flag block
        std::vector<void*> imports;   // direct: IPC bases to close
        ~plan()
        {
            for (auto b : imports) ghx_ipc_close(b);
            if (ep) ghx_epochs_destroy(ep);
            for (auto* v : {&send, &recv})
                for (auto& b : *v)
                    if (b.owned && b.data) (void)hipFree(b.data);
            if (ex) ghx_exchange_destroy(ex);
        }
    };

    context* m_ctx;
    options m_opt;
    hipStream_t m_stream = nullptr;
    bool m_capturing = false;  // the exchange being started is enqueued into a stream capture
    hipEvent_t m_done = nullptr, m_start = nullptr;
    std::vector<hipStream_t> m_lanes;     // pipelined: the peer streams
    std::vector<hipEvent_t> m_lane_done;
    hipEvent_t m_fork = nullptr;
    bool m_valid = false;
    std::map<std::string, std::unique_ptr<plan>> m_plans;

  public:
    explicit communication_object(context& ctx, options opt = {})
    : m_ctx{&ctx}
    , m_opt{opt}
    {
        if (m_opt.direct && (m_opt.pipelined || m_opt.self_through_transport))
            throw std::runtime_error("direct packs into the peers' buffers: no pipeline, no self_through_transport");
        // a non-blocking stream of the greatest priority, like the reference's device::stream
        // (include/ghex/device/cuda/stream.hpp:30-37)
        int lo = 0, hi = 0;
        check_hip(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
        check_hip(hipStreamCreateWithPriority(&m_stream, hipStreamNonBlocking, hi), "hipStreamCreate");
        check_hip(hipEventCreateWithFlags(&m_done, hipEventDisableTiming), "hipEventCreate");
        check_hip(hipEventCreateWithFlags(&m_start, hipEventDisableTiming), "hipEventCreate");
        if (m_opt.pipelined)
        {
            if (m_opt.max_streams < 1) throw std::runtime_error("max_streams must be >= 1");
            check_hip(hipEventCreateWithFlags(&m_fork, hipEventDisableTiming), "hipEventCreate");
            for (int l = 0; l < m_opt.max_streams; ++l)
            {
                hipStream_t st;
                hipEvent_t ev;
                check_hip(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, hi), "hipStreamCreate");
                check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                m_lanes.push_back(st);
                m_lane_done.push_back(ev);
            }
        }
    }
    communication_object(const communication_object&) = delete;
    communication_object& operator=(const communication_object&) = delete;
    ~communication_object()
    {
        if (m_stream) (void)hipStreamSynchronize(m_stream);
        for (auto l : m_lanes) (void)hipStreamSynchronize(l);
        m_plans.clear();
        if (m_done) (void)hipEventDestroy(m_done);
        if (m_start) (void)hipEventDestroy(m_start);
        if (m_fork) (void)hipEventDestroy(m_fork);
        for (auto e : m_lane_done) (void)hipEventDestroy(e);
        for (auto l : m_lanes) (void)hipStreamDestroy(l);
        if (m_stream) (void)hipStreamDestroy(m_stream);
    }

    hipStream_t stream() const { return m_stream; }

    // exchange(pattern(f1), pattern(f2), ...) (:271-285)
    template<typename... Fields>
    communication_handle exchange(buffer_info<Fields>... bis)
    {
        return start(nullptr, {item_of(bis)...}, {ptr_of(bis)...});
    }
    // exchange(first, last) over buffer_infos of one field type (:349-355)
    template<typename Iterator>
    communication_handle exchange(Iterator first, Iterator last)
    {
        std::vector<ghx_exchange_item> items;
        std::vector<void*> ptrs;
        for (auto it = first; it != last; ++it)
        {
            items.push_back(item_of(*it));
            ptrs.push_back(ptr_of(*it));
        }
        return start(nullptr, std::move(items), std::move(ptrs));
    }
    // schedule_exchange(stream, ...) (:287-330): starts after the work already on `stream`,
    // never blocks the host; pair with handle.schedule_wait(stream).
    template<typename... Fields>
    communication_handle schedule_exchange(hipStream_t stream, buffer_info<Fields>... bis)
    {
        return start(stream, {item_of(bis)...}, {ptr_of(bis)...});
    }

    // plan facts (tests / benchmarks)
    std::size_t num_plans() const { return m_plans.size(); }

  private:
    friend class communication_handle;
    friend class bulk_communication_object;  // starts the remote part of a bulk exchange
    void finish()
    {
        check_hip(hipEventSynchronize(m_done), "hipEventSynchronize");
        m_valid = false;
        check_epochs();
    }
    bool ready()
    {
        const hipError_t e = hipEventQuery(m_done);
        if (e == hipErrorNotReady) return false;
        check_hip(e, "hipEventQuery");
        m_valid = false;
        check_epochs();
        return true;
    }
    void check_epochs() const
    {
        for (const auto& kv : m_plans)
        {
            if (!kv.second->ep) continue;
            std::int32_t err = 0;
            check_ghx(ghx_epochs_status(kv.second->ep, &err, nullptr), "ghx_epochs_status");
            if (err) throw std::runtime_error("direct exchange failed: " + epochs_error_text(err));
        }
    }

    // direct: export this rank's peer receive buffers, import the ones its messages go to, and
    // attach the plan's epoch flag block (collective over the transport, at plan creation)
    void setup_direct(plan& p)
    {
        if (m_capturing)
            throw std::runtime_error("direct exchange: a plan's first exchange sets up IPC handles and flag "
                                     "blocks collectively and cannot run inside a stream capture; run one "
                                     "exchange of these fields before capturing");
        auto& t = m_ctx->get_transport();
        const int me = m_ctx->rank(), world = m_ctx->size();
        char hn[256] = {0};
        if (gethostname(hn, sizeof(hn) - 1) != 0) hn[0] = '?';
        const std::string host(hn);
        std::vector<char> mine;
        detail::put(mine, std::int32_t(host.size()));
        mine.insert(mine.end(), host.begin(), host.end());
        detail::put(mine, std::int64_t(getpid()));
        std::int32_t n = 0;
        for (auto& b : p.recv) n += b.rank != me;
        detail::put(mine, n);
        for (auto& b : p.recv)
        {
            if (b.rank == me) continue;
            unsigned char h[64];
            std::uint64_t off = 0;
            check_ghx(ghx_ipc_export(b.data, h, &off), "ghx_ipc_export");
            detail::put(mine, b.rank);
            detail::put(mine, b.tag);
            detail::put(mine, b.size);
            mine.insert(mine.end(), reinterpret_cast<char*>(h), reinterpret_cast<char*>(h) + 64);
            detail::put(mine, off);
            detail::put(mine, dbl_of(b.size));  // the odd-parity copy's offset
        }
        const auto all = t.all_gather(mine);
        struct entry
        {
            std::int32_t src, tag;
            std::uint64_t size, off, dbl;
            unsigned char h[64];
        };
        std::vector<std::string> hosts(static_cast<std::size_t>(world));
        std::vector<std::int64_t> pids(static_cast<std::size_t>(world));
        std::vector<std::vector<entry>> recv_of(static_cast<std::size_t>(world));
        for (int r = 0; r < world; ++r)
        {
            const auto& in = all[std::size_t(r)];
            std::size_t pos = 0;
            const auto hl = detail::get<std::int32_t>(in, pos);
            if (hl < 0 || pos + std::size_t(hl) > in.size()) throw std::runtime_error("malformed direct payload");
            hosts[std::size_t(r)].assign(in.data() + pos, std::size_t(hl));
            pos += std::size_t(hl);
            pids[std::size_t(r)] = detail::get<std::int64_t>(in, pos);
            const auto k = detail::get<std::int32_t>(in, pos);
            for (std::int32_t i = 0; i < k; ++i)
            {
                entry e{};
                e.src = detail::get<std::int32_t>(in, pos);
                e.tag = detail::get<std::int32_t>(in, pos);
                e.size = detail::get<std::uint64_t>(in, pos);
                if (pos + 64 > in.size()) throw std::runtime_error("malformed direct payload");
                std::memcpy(e.h, in.data() + pos, 64);
                pos += 64;
                e.off = detail::get<std::uint64_t>(in, pos);
                e.dbl = detail::get<std::uint64_t>(in, pos);
                recv_of[std::size_t(r)].push_back(e);
            }
        }
        // every rank checks every pair (the receivers' entries name their senders), so all
        // throw together and none is left waiting in a collective
        for (int r = 0; r < world; ++r)
            for (const auto& e : recv_of[std::size_t(r)])
                if (e.src >= 0 && e.src < world && hosts[std::size_t(e.src)] != hosts[std::size_t(r)])
                    throw std::runtime_error("direct exchange needs node-local peers: rank " + std::to_string(e.src) +
                                             " (host " + hosts[std::size_t(e.src)] + ") sends to rank " +
                                             std::to_string(r) + " (host " + hosts[std::size_t(r)] + ")");
        p.dsptr = p.sptr;
        std::vector<std::int64_t> send_dbl(p.send.size(), 0);
        std::map<int, std::vector<std::size_t>> by_peer;
        for (std::size_t i = 0; i < p.send.size(); ++i)
            if (p.send[i].rank != me) by_peer[p.send[i].rank].push_back(i);
        for (auto& [q, idx] : by_peer)
        {
            if (hosts[std::size_t(q)] != host || pids[std::size_t(q)] == pids[std::size_t(me)])
                throw std::runtime_error("direct exchange: rank " + std::to_string(q) +
                                         " is not another process of this host (direct needs one "
                                         "process per rank, node-local)");
            // the k-th message of the pair in tag order on both sides (stable: plan order)
            std::vector<entry> theirs;
            for (const auto& e : recv_of[std::size_t(q)])
                if (e.src == me) theirs.push_back(e);
            std::stable_sort(theirs.begin(), theirs.end(), [](const entry& a, const entry& b) { return a.tag < b.tag; });
            std::stable_sort(idx.begin(), idx.end(),
                             [&](std::size_t a, std::size_t b) { return p.send[a].tag < p.send[b].tag; });
            if (theirs.size() != idx.size())
                throw std::runtime_error("direct exchange: rank " + std::to_string(q) + " expects " +
                                         std::to_string(theirs.size()) + " messages, this rank sends " +
                                         std::to_string(idx.size()));
            for (std::size_t k = 0; k < idx.size(); ++k)
            {
                const auto& b = p.send[idx[k]];
                const auto& e = theirs[k];
                if (e.tag != b.tag || e.size != b.size)
                    throw std::runtime_error("direct exchange: message mismatch with rank " + std::to_string(q));
                void *base = nullptr, *ptr = nullptr;
                check_ghx(ghx_ipc_import(e.h, e.off, &base, &ptr), "ghx_ipc_import");
                p.imports.push_back(base);
                p.dsptr[idx[k]] = ptr;
                send_dbl[idx[k]] = std::int64_t(e.dbl);
            }
        }
        if (world > 1)
        {
            // one flag block per plan and host, indexed by node-local position: the host's
            // lowest rank creates it, the host's other ranks attach
            std::vector<std::int32_t> pos(std::size_t(world), -1);
            int leader = -1, nlocal = 0;
            for (int r = 0; r < world; ++r)
                if (hosts[std::size_t(r)] == host)
                {
                    if (leader < 0) leader = r;
                    pos[std::size_t(r)] = nlocal++;
                }
            std::string name;
            if (me == leader && nlocal > 1)  // created (and sized) before anyone learns its name
            {
                name = "/ghx_dx_" + std::to_string(getpid()) + "_" +
                       std::to_string(reinterpret_cast<std::uintptr_t>(&p) & 0xffffffu);
                check_ghx(ghx_epochs_create(name.c_str(), 1, nlocal, pos[std::size_t(me)], m_opt.epoch_timeout,
                                            &p.ep),
                          "ghx_epochs_create");
            }
            const auto names = t.all_gather(std::vector<char>(name.begin(), name.end()));
            if (me != leader && nlocal > 1)
                check_ghx(ghx_epochs_create(std::string(names[std::size_t(leader)].begin(),
                                                        names[std::size_t(leader)].end()).c_str(),
                                            0, nlocal, pos[std::size_t(me)], m_opt.epoch_timeout, &p.ep),
                          "ghx_epochs_create");
            (void)t.all_gather({});  // every rank has attached
            if (me == leader && nlocal > 1) (void)ghx_epochs_unlink(name.c_str());
            std::vector<std::int32_t> srcs, tgts;
            for (auto& b : p.recv)
                if (b.rank != me && std::find(srcs.begin(), srcs.end(), pos[std::size_t(b.rank)]) == srcs.end())
                    srcs.push_back(pos[std::size_t(b.rank)]);
            for (auto& kv : by_peer) tgts.push_back(pos[std::size_t(kv.first)]);
            std::sort(srcs.begin(), srcs.end());
            std::sort(tgts.begin(), tgts.end());
            if (p.ep)
            {
                check_ghx(ghx_epochs_peers(p.ep, srcs.data(), std::int32_t(srcs.size()), tgts.data(),
                                           std::int32_t(tgts.size())),
                          "ghx_epochs_peers");
                // one epoch launch per exchange: the peers' receive buffers are double-buffered
                // by epoch parity, chosen on the device from the epoch counter
                const std::uint64_t* word = nullptr;
                check_ghx(ghx_epochs_counter(p.ep, &word), "ghx_epochs_counter");
                std::vector<std::int64_t> recv_dbl;
                for (auto& b : p.recv) recv_dbl.push_back(b.rank != me ? std::int64_t(dbl_of(b.size)) : 0);
                check_ghx(ghx_exchange_set_parity(p.ex, 0, word, 1, send_dbl.data(), std::int32_t(send_dbl.size())),
                          "ghx_exchange_set_parity");
                check_ghx(ghx_exchange_set_parity(p.ex, 1, word, 0, recv_dbl.data(), std::int32_t(recv_dbl.size())),
                          "ghx_exchange_set_parity");
            }
        }
    }

    // the odd-parity copy of a double-buffered (direct) receive buffer starts this far in
    static std::uint64_t dbl_of(std::uint64_t size) { return std::max<std::uint64_t>(256, (size + 255) / 256 * 256); }

    // tag offsets per distinct pattern container in argument order (:540-549) are assigned in
    // start(); here only the per-field description
    template<typename Field>
    static ghx_exchange_item item_of(const buffer_info<Field>& bi)
    {
        ghx_exchange_item it;
        std::memset(&it, 0, sizeof(it));
        it.pattern = bi.pattern->handle();
        it.local_index = bi.local_index;
        describe(it, bi.field->desc());
        it.align = std::int32_t(alignof(typename Field::value_type));
        it.tag_offset = 0;
        return it;
    }
    static void describe(ghx_exchange_item& it, const ghx_field_desc& d)
    {
        it.kind = 0;
        it.field = d;
    }
    static void describe(ghx_exchange_item& it, const ghx_udata_desc& d)
    {
        it.kind = 1;
        it.udata = d;
    }
    template<typename Field>
    static void* ptr_of(const buffer_info<Field>& bi)
    {
        return const_cast<void*>(static_cast<const void*>(bi.field->data()));
    }

    // plan cache key: every member of every item (no padding bytes)
    static std::string key_of(const std::vector<ghx_exchange_item>& items)
    {
        std::vector<char> k;
        for (const auto& it : items)
        {
            detail::put(k, it.pattern);
            detail::put(k, it.local_index);
            detail::put(k, it.kind);
            detail::put(k, it.align);
            detail::put(k, it.tag_offset);
            if (it.kind == 0)
            {
                const auto& f = it.field;
                detail::put(k, f.dim);
                detail::put(k, f.elem_size);
                detail::put(k, f.num_components);
                detail::put(k, f.has_components);
                for (int d = 0; d < GHX_MAX_DIM; ++d)
                {
                    detail::put(k, f.layout[d]);
                    detail::put(k, f.byte_strides[d]);
                    detail::put(k, f.offsets[d]);
                    detail::put(k, f.extents[d]);
                }
            }
            else
            {
                const auto& u = it.udata;
                detail::put(k, u.elem_size);
                detail::put(k, u.levels);
                detail::put(k, u.levels_first);
                detail::put(k, u.index_stride);
                detail::put(k, u.level_stride);
            }
        }
        return std::string(k.begin(), k.end());
    }

    plan& plan_for(std::vector<ghx_exchange_item>& items)
    {
        std::map<const ghx_pattern*, std::int32_t> offsets;
        std::int32_t acc = 0;
        for (auto& it : items)
        {
            auto f = offsets.find(it.pattern);
            if (f == offsets.end())
            {
                std::int32_t mt = 0;
                check_ghx(ghx_pattern_max_tag(it.pattern, &mt), "ghx_pattern_max_tag");
                f = offsets.emplace(it.pattern, acc).first;
                acc += mt + 1;
            }
            it.tag_offset = f->second;
        }
        const std::string key = key_of(items);
        auto found = m_plans.find(key);
        if (found != m_plans.end()) return *found->second;
        auto p = std::make_unique<plan>();
        check_ghx(ghx_exchange_create(items.data(), std::int32_t(items.size()), &p->ex), "ghx_exchange_create");
        const int me = m_ctx->rank();
        for (int dir = 0; dir < 2; ++dir)
        {
            std::int32_t n = 0;
            check_ghx(ghx_exchange_num_buffers(p->ex, dir, &n), "ghx_exchange_num_buffers");
            auto& v = dir == 0 ? p->send : p->recv;
            for (std::int32_t i = 0; i < n; ++i)
            {
                buf b{};
                check_ghx(ghx_exchange_buffer(p->ex, dir, i, &b.first_id, &b.second_id, &b.rank, &b.tag, &b.size),
                          "ghx_exchange_buffer");
                v.push_back(b);
            }
        }
        for (auto& b : p->send)
            check_hip(hipMalloc(&b.data, std::max<std::uint64_t>(1, b.size)), "hipMalloc(send buffer)");
        for (auto& b : p->recv)
        {
            if (b.rank == me && !m_opt.self_through_transport)
            {
                // self message: unpack straight from the matching send buffer
                for (auto& s : p->send)
                    if (s.first_id == b.first_id && s.second_id == b.second_id && s.rank == me)
                    {
                        b.data = s.data;
                        b.owned = false;
                    }
            }
            // direct: a peer's receive buffer exists twice (one-launch epochs, setup_direct)
            const std::uint64_t bytes = m_opt.direct && b.rank != me ? 2 * dbl_of(b.size) : std::max<std::uint64_t>(1, b.size);
            if (!b.data) check_hip(hipMalloc(&b.data, bytes), "hipMalloc(recv buffer)");
        }
        bool all_self = !m_opt.self_through_transport;
        for (auto* v : {&p->send, &p->recv})
            for (auto& b : *v) all_self = all_self && b.rank == me;
        std::int32_t fusable = 0;
        check_ghx(ghx_exchange_self_fusable(p->ex, &fusable), "ghx_exchange_self_fusable");
        p->fused = m_opt.fuse_self && all_self && fusable;
        std::int32_t mixed = 0;
        check_ghx(ghx_exchange_mixed(p->ex, &mixed), "ghx_exchange_mixed");
        p->mixed = m_opt.fuse_self && !m_opt.self_through_transport && !p->fused && mixed;
        for (auto& b : p->send) p->sptr.push_back(b.data);
        for (auto& b : p->recv) p->rptr.push_back(b.data);
        if (m_opt.pipelined)
        {
            check_ghx(ghx_exchange_split(p->ex), "ghx_exchange_split");
            p->fused = false;
            p->mixed = false;
        }
        if (m_opt.direct) setup_direct(*p);  // every rank, at this plan's first exchange
        auto& ref = *p;
        m_plans.emplace(std::move(key), std::move(p));
        return ref;
    }

    // peers in the global round order, dealt over the lanes; self messages on the object's
    // stream (unless routed through the transport); the object's stream joins every lane
    void run_pipelined(plan& p, std::vector<void*>& fptrs, std::int32_t nf, std::int32_t ns,
                       std::int32_t nr)
    {
        const int me = m_ctx->rank(), world = m_ctx->size();
        const bool self_tr = m_opt.self_through_transport;
        std::vector<int> peers;
        for (auto* v : {&p.send, &p.recv})
            for (auto& b : *v)
                if ((b.rank != me || self_tr) &&
                    std::find(peers.begin(), peers.end(), b.rank) == peers.end())
                    peers.push_back(b.rank);
        std::sort(peers.begin(), peers.end(), [&](int a, int b) {
            const int ra = round_of(me, a, world), rb = round_of(me, b, world);
            return ra != rb ? ra < rb : a < b;
        });
        check_hip(hipEventRecord(m_fork, m_stream), "hipEventRecord");
        for (auto l : m_lanes) check_hip(hipStreamWaitEvent(l, m_fork, 0), "hipStreamWaitEvent");
        for (std::size_t k = 0; k < peers.size(); ++k)
        {
            const int q = peers[k];
            hipStream_t lane = m_lanes[k % m_lanes.size()];
            std::vector<message> sends, recvs;
            for (std::size_t i = 0; i < p.send.size(); ++i)
                if (p.send[i].rank == q)
                {
                    check_ghx(ghx_exchange_pack_buffer(p.ex, std::int32_t(i), fptrs.data(), nf,
                                                       p.sptr.data(), ns, lane),
                              "ghx_exchange_pack_buffer");
                    sends.push_back({p.send[i].data, p.send[i].size, q, p.send[i].tag});
                }
            for (auto& b : p.recv)
                if (b.rank == q) recvs.push_back({b.data, b.size, q, b.tag});
            m_ctx->get_transport().exchange_peer(q, sends, recvs, lane);
            for (std::size_t j = 0; j < p.recv.size(); ++j)
                if (p.recv[j].rank == q)
                    check_ghx(ghx_exchange_unpack_buffer(p.ex, std::int32_t(j), fptrs.data(), nf,
                                                         p.rptr.data(), nr, lane),
                              "ghx_exchange_unpack_buffer");
        }
        if (!self_tr)
        {
            for (std::size_t i = 0; i < p.send.size(); ++i)
                if (p.send[i].rank == me)
                    check_ghx(ghx_exchange_pack_buffer(p.ex, std::int32_t(i), fptrs.data(), nf,
                                                       p.sptr.data(), ns, m_stream),
                              "ghx_exchange_pack_buffer");
            for (std::size_t j = 0; j < p.recv.size(); ++j)  // recv aliases the send buffer
                if (p.recv[j].rank == me)
                    check_ghx(ghx_exchange_unpack_buffer(p.ex, std::int32_t(j), fptrs.data(), nf,
                                                         p.rptr.data(), nr, m_stream),
                              "ghx_exchange_unpack_buffer");
        }
        for (std::size_t l = 0; l < m_lanes.size(); ++l)
        {
            check_hip(hipEventRecord(m_lane_done[l], m_lanes[l]), "hipEventRecord");
            check_hip(hipStreamWaitEvent(m_stream, m_lane_done[l], 0), "hipStreamWaitEvent");
        }
    }

    communication_handle start(hipStream_t after, std::vector<ghx_exchange_item> items,
                               std::vector<void*> fptrs)
    {
        if (m_valid) throw std::runtime_error("earlier exchange operation was not finished");
        if (items.empty()) return {};
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        m_capturing = after && hipStreamIsCapturing(after, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
        plan& p = plan_for(items);
        if (after)
        {
            check_hip(hipEventRecord(m_start, after), "hipEventRecord");
            check_hip(hipStreamWaitEvent(m_stream, m_start, 0), "hipStreamWaitEvent");
        }
        const auto nf = std::int32_t(fptrs.size());
        const auto ns = std::int32_t(p.sptr.size()), nr = std::int32_t(p.rptr.size());
        if (m_opt.pipelined)
            run_pipelined(p, fptrs, nf, ns, nr);
        else if (p.fused)
            check_ghx(ghx_exchange_self(p.ex, fptrs.data(), nf, p.sptr.data(), ns, m_stream), "ghx_exchange_self");
        else if (m_opt.direct)
        {
            // pack into copy e&1 of the receivers' buffers -> one-launch close (every sender's
            // pack landed, every receiver done with the copy of e+1) -> unpack copy e&1
            if (p.mixed)
                check_ghx(ghx_exchange_pack_self(p.ex, fptrs.data(), nf, p.dsptr.data(), ns, m_stream),
                          "ghx_exchange_pack_self");
            else
                check_ghx(ghx_exchange_pack(p.ex, fptrs.data(), nf, p.dsptr.data(), ns, m_stream), "ghx_exchange_pack");
            if (p.ep) check_ghx(ghx_epochs_enqueue(p.ep, 2, m_stream), "ghx_epochs_enqueue(close)");
            if (p.mixed)
                check_ghx(ghx_exchange_unpack_peers(p.ex, fptrs.data(), nf, p.rptr.data(), nr, m_stream),
                          "ghx_exchange_unpack_peers");
            else
                check_ghx(ghx_exchange_unpack(p.ex, fptrs.data(), nf, p.rptr.data(), nr, m_stream),
                          "ghx_exchange_unpack");
        }
        else
        {
            if (p.mixed)  // the pack launch also completes the self messages
                check_ghx(ghx_exchange_pack_self(p.ex, fptrs.data(), nf, p.sptr.data(), ns, m_stream),
                          "ghx_exchange_pack_self");
            else
                check_ghx(ghx_exchange_pack(p.ex, fptrs.data(), nf, p.sptr.data(), ns, m_stream),
                          "ghx_exchange_pack");
            const int me = m_ctx->rank();
            std::vector<message> sends, recvs;
            for (auto& b : p.send)
                if (b.rank != me || m_opt.self_through_transport) sends.push_back({b.data, b.size, b.rank, b.tag});
            for (auto& b : p.recv)
                if (b.rank != me || m_opt.self_through_transport) recvs.push_back({b.data, b.size, b.rank, b.tag});
            if (!sends.empty() || !recvs.empty()) m_ctx->get_transport().exchange(sends, recvs, m_stream);
            if (p.mixed)
                check_ghx(ghx_exchange_unpack_peers(p.ex, fptrs.data(), nf, p.rptr.data(), nr, m_stream),
                          "ghx_exchange_unpack_peers");
            else
                check_ghx(ghx_exchange_unpack(p.ex, fptrs.data(), nf, p.rptr.data(), nr, m_stream),
                          "ghx_exchange_unpack");
        }
        check_hip(hipEventRecord(m_done, m_stream), "hipEventRecord");
        m_valid = true;
        return {this, m_done};
    }
};

inline void communication_handle::wait()
{
    if (m_co) m_co->finish();
    m_co = nullptr;
}

inline bool communication_handle::is_ready()
{
    if (!m_co) return true;
    if (!m_co->ready()) return false;
    m_co = nullptr;
    return true;
}

inline communication_object make_communication_object(context& ctx)
{
    return communication_object(ctx);
}
}  // namespace ghex_amd
