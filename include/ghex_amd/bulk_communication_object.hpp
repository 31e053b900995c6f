// ghex_amd/bulk_communication_object.hpp — the reference's zero-copy exchange for node-local
// GPUs in C++ over the C ABI: bulk_communication_object (include/ghex/bulk_communication_object.hpp
// :206-704), its structured put (include/ghex/structured/rma_put.hpp:204-245) and the CUDA IPC
// handles (include/ghex/rma/cuda/handle.hpp:20-96), in the same shape as ghex_amd.
// BulkCommunicationObject (ghex_amd/bulk_communication_object.py):
//
//   bulk_communication_object bco(ctx);
//   bco.add_field(pattern(field_a)); bco.add_field(pattern(field_b));   // same order on every rank
//   bco.init();                                                         // collective
//   bco.exchange().wait();                                              // collective
//
// Instead of pack -> transport -> unpack, every rank copies its send regions straight into the
// receiving rank's halo cells: libghx put plans (ghx_put_*: the sender's send halo and the
// receiver's recv halo of one key describe the same virtual message bytes; one launch per group
// of up to 64 messages) on the object's stream. Peer fields are mapped once in init(): through
// IPC handles (ghx_ipc_export/import) for ranks in other processes of this host, directly for
// ranks that are threads of this process (loopback transport). Halos from and to ranks on other
// hosts go through a communication_object over the pattern's remote part (ghx_pattern_filter),
// started by the same exchange() and awaited by the same wait() — the reference's split into
// local (RMA) and remote pattern maps (bulk_communication_object.hpp:330-383).
//
// Epochs (the reference's access guards, include/ghex/rma/access_guard.hpp:35-140, and its
// open / put-when-writable / wait sequence, bulk_communication_object.hpp:621-694). Ranks in
// separate processes (one per GPU): stream-ordered device epochs (ghx_epochs_*): the object's
// stream waits for the caller's stream, k_epoch(open) opens this rank's halos to its sources and
// waits until its targets have opened theirs, the puts run, k_epoch(close) signals its targets
// and waits for its sources; the caller's stream then waits for the object's stream. No host
// synchronisation, no barrier; wait() reports a peer that never arrived. Ranks that are threads
// of one process (loopback transport) share hardware queues, where one rank's waiting kernel
// could hold back another rank's signalling kernel: they keep the host form — drain, barrier
// (every target open), puts, drain, barrier (every halo written; barriers are transport
// all_gathers of nothing).
// Structured fields only (the reference's bulk object serves structured fields through
// rma_range_generator; unstructured exchanges use communication_object).
#pragma once

#include <ghx.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "communication_object.hpp"

namespace ghex_amd
{
class bulk_handle
{
    hipEvent_t m_done = nullptr;       // the object's completion event (device epochs)
    const ghx_epochs* m_ep = nullptr;
    communication_handle m_remote;     // the halos exchanged with other hosts' ranks

    void check() const
    {
        if (!m_ep) return;
        std::int32_t err = 0;
        check_ghx(ghx_epochs_status(m_ep, &err, nullptr), "ghx_epochs_status");
        if (err) throw std::runtime_error("bulk exchange failed: " + epochs_error_text(err));
    }

  public:
    bulk_handle() = default;
    bulk_handle(hipEvent_t done, const ghx_epochs* ep, communication_handle remote = {})
    : m_done{done}
    , m_ep{ep}
    , m_remote{remote}
    {
    }
    void wait()
    {
        if (m_done) check_hip(hipEventSynchronize(m_done), "hipEventSynchronize");
        check();
        m_remote.wait();
    }
    bool is_ready()
    {
        if (m_done && hipEventQuery(m_done) != hipSuccess) return false;
        check();
        return m_remote.is_ready();
    }
    void progress() { (void)is_ready(); }
};

class bulk_communication_object
{
    struct local_field
    {
        const pattern_container* pattern;
        int local_index;
        ghx_field_desc desc;
        void* data;
        int domain;
        int j;  // the j-th field registered for this domain on this rank
        int align;  // alignof(value_type): the buffer layout of the remote part
    };
    struct remote_space_key
    {
        int remote_id, tag;
        std::vector<ghx_box> boxes;
    };
    struct remote_field
    {
        int domain, j;
        ghx_field_desc desc;
        unsigned char ipc[64];
        std::uint64_t offset, raw;
        std::vector<remote_space_key> recv;
    };
    struct remote_rank
    {
        std::string host;
        long pid;
        std::string epochs;  // rank 0: name of the epochs flag block
        std::vector<remote_field> fields;
    };
    struct put
    {
        ghx_put* h = nullptr;
        std::vector<void*> src, dst;  // the plan's source / target field slots
    };

    context* m_ctx;
    hipStream_t m_stream = nullptr;
    std::vector<local_field> m_fields;
    std::vector<put> m_puts;
    std::vector<void*> m_imports;
    bool m_init = false;
    ghx_epochs* m_ep = nullptr;        // device epochs (this host's ranks all separate processes)
    hipEvent_t m_after = nullptr, m_done = nullptr;
    std::string m_host;                // set_host_name(): tests emulate several hosts
    // the remote part: halos exchanged with ranks on other hosts, buffered
    std::vector<std::unique_ptr<pattern_container>> m_rpcs;
    std::vector<ghx_exchange_item> m_ritems;
    std::vector<void*> m_rptrs;
    std::unique_ptr<communication_object> m_remote;

    std::string hostname() const
    {
        if (!m_host.empty()) return m_host;
        char buf[256] = {0};
        if (gethostname(buf, sizeof(buf) - 1) != 0) return "?";
        return buf;
    }
    void barrier() { (void)m_ctx->get_transport().all_gather({}); }

    // halos of a local domain: [(remote id, remote rank, tag, local boxes)]
    static std::vector<std::tuple<int, int, int, std::vector<ghx_box>>> halos(const pattern_container& pc,
                                                                             int li, int dir)
    {
        std::int32_t n = 0;
        check_ghx(ghx_pattern_num_keys(pc.handle(), li, dir, &n), "ghx_pattern_num_keys");
        std::vector<std::tuple<int, int, int, std::vector<ghx_box>>> out;
        for (std::int32_t k = 0; k < n; ++k)
        {
            std::int32_t rid = 0, rr = 0, tag = 0, ns = 0;
            std::int64_t ne = 0;
            check_ghx(ghx_pattern_key(pc.handle(), li, dir, k, &rid, &rr, &tag, &ns, &ne), "ghx_pattern_key");
            std::vector<ghx_box> loc(std::size_t(std::max(1, ns))), glo(loc.size());
            check_ghx(ghx_pattern_key_boxes(pc.handle(), li, dir, k, loc.data(), glo.data(), ns),
                      "ghx_pattern_key_boxes");
            loc.resize(std::size_t(ns));
            out.emplace_back(rid, rr, tag, std::move(loc));
        }
        return out;
    }

    std::vector<char> serialize_mine() const
    {
        std::vector<char> out;
        const std::string host = hostname();
        detail::put(out, std::int32_t(host.size()));
        out.insert(out.end(), host.begin(), host.end());
        detail::put(out, std::int64_t(getpid()));
        detail::put(out, std::int32_t(0));  // (the epochs name travels in init()'s second round)
        detail::put(out, std::int32_t(m_fields.size()));
        for (const auto& f : m_fields)
        {
            detail::put(out, std::int32_t(f.domain));
            detail::put(out, std::int32_t(f.j));
            detail::put(out, f.desc);
            unsigned char h[64];
            std::uint64_t off = 0;
            check_ghx(ghx_ipc_export(f.data, h, &off), "ghx_ipc_export");
            out.insert(out.end(), reinterpret_cast<char*>(h), reinterpret_cast<char*>(h) + 64);
            detail::put(out, off);
            detail::put(out, std::uint64_t(reinterpret_cast<std::uintptr_t>(f.data)));
            const auto recv = halos(*f.pattern, f.local_index, 1);
            detail::put(out, std::int32_t(recv.size()));
            for (const auto& [rid, rr, tag, boxes] : recv)
            {
                (void)rr;
                detail::put(out, std::int32_t(rid));
                detail::put(out, std::int32_t(tag));
                detail::put(out, std::int32_t(boxes.size()));
                for (const auto& b : boxes) detail::put(out, b);
            }
        }
        return out;
    }

    static remote_rank deserialize(const std::vector<char>& in)
    {
        remote_rank r;
        std::size_t pos = 0;
        const auto hl = detail::get<std::int32_t>(in, pos);
        if (hl < 0 || pos + std::size_t(hl) > in.size()) throw std::runtime_error("malformed bulk payload");
        r.host.assign(in.data() + pos, std::size_t(hl));
        pos += std::size_t(hl);
        r.pid = long(detail::get<std::int64_t>(in, pos));
        const auto nl = detail::get<std::int32_t>(in, pos);
        if (nl < 0 || pos + std::size_t(nl) > in.size()) throw std::runtime_error("malformed bulk payload");
        r.epochs.assign(in.data() + pos, std::size_t(nl));
        pos += std::size_t(nl);
        const auto nf = detail::get<std::int32_t>(in, pos);
        for (std::int32_t i = 0; i < nf; ++i)
        {
            remote_field f;
            f.domain = detail::get<std::int32_t>(in, pos);
            f.j = detail::get<std::int32_t>(in, pos);
            f.desc = detail::get<ghx_field_desc>(in, pos);
            if (pos + 64 > in.size()) throw std::runtime_error("malformed bulk payload");
            std::memcpy(f.ipc, in.data() + pos, 64);
            pos += 64;
            f.offset = detail::get<std::uint64_t>(in, pos);
            f.raw = detail::get<std::uint64_t>(in, pos);
            const auto nk = detail::get<std::int32_t>(in, pos);
            for (std::int32_t k = 0; k < nk; ++k)
            {
                remote_space_key key;
                key.remote_id = detail::get<std::int32_t>(in, pos);
                key.tag = detail::get<std::int32_t>(in, pos);
                const auto nb = detail::get<std::int32_t>(in, pos);
                for (std::int32_t b = 0; b < nb; ++b) key.boxes.push_back(detail::get<ghx_box>(in, pos));
                f.recv.push_back(std::move(key));
            }
            r.fields.push_back(std::move(f));
        }
        return r;
    }

    struct msg
    {
        int src;                     // index into m_fields
        std::vector<ghx_box> sboxes;  // sender's local coordinates
        std::pair<int, int> target;  // (rank, index in that rank's field list)
        const std::vector<ghx_box>* tboxes;
    };

    void make_put(const std::vector<msg>& chunk, const std::vector<int>& srcs,
                  const std::vector<std::pair<int, int>>& dsts, const std::vector<remote_rank>& all,
                  const std::map<std::pair<int, int>, void*>& ptr_of)
    {
        const auto n = chunk.size();
        std::vector<ghx_pack_entry> src(n), dst(n);
        for (std::size_t b = 0; b < n; ++b)
        {
            const auto& m = chunk[b];
            std::memset(&src[b], 0, sizeof(ghx_pack_entry));
            std::memset(&dst[b], 0, sizeof(ghx_pack_entry));
            src[b].field = m_fields[std::size_t(m.src)].desc;
            src[b].field_slot = std::int32_t(std::find(srcs.begin(), srcs.end(), m.src) - srcs.begin());
            src[b].buffer_slot = std::int32_t(b);
            src[b].boxes = m.sboxes.data();
            src[b].n_boxes = std::int32_t(m.sboxes.size());
            dst[b].field = all[std::size_t(m.target.first)].fields[std::size_t(m.target.second)].desc;
            dst[b].field_slot =
                std::int32_t(std::find(dsts.begin(), dsts.end(), m.target) - dsts.begin());
            dst[b].buffer_slot = std::int32_t(b);
            dst[b].boxes = m.tboxes->data();
            dst[b].n_boxes = std::int32_t(m.tboxes->size());
        }
        put p;
        check_ghx(ghx_put_create(src.data(), std::int32_t(n), dst.data(), std::int32_t(n), &p.h), "ghx_put_create");
        for (int k : srcs) p.src.push_back(m_fields[std::size_t(k)].data);
        for (const auto& t : dsts) p.dst.push_back(ptr_of.at(t));
        m_puts.push_back(std::move(p));
    }

  public:
    explicit bulk_communication_object(context& ctx)
    : m_ctx{&ctx}
    {
        int lo = 0, hi = 0;
        check_hip(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
        check_hip(hipStreamCreateWithPriority(&m_stream, hipStreamNonBlocking, hi), "hipStreamCreate");
    }
    bulk_communication_object(const bulk_communication_object&) = delete;
    bulk_communication_object& operator=(const bulk_communication_object&) = delete;
    ~bulk_communication_object()
    {
        if (m_stream) (void)hipStreamSynchronize(m_stream);
        for (auto& p : m_puts) ghx_put_destroy(p.h);
        for (auto b : m_imports) ghx_ipc_close(b);
        if (m_ep) ghx_epochs_destroy(m_ep);
        if (m_after) (void)hipEventDestroy(m_after);
        if (m_done) (void)hipEventDestroy(m_done);
        if (m_stream) (void)hipStreamDestroy(m_stream);
    }

    // seconds an epoch wait may take before wait() throws (device epochs)
    double epoch_timeout = 30.0;
    bool device_epochs() const { return m_ep != nullptr; }

    hipStream_t stream() const { return m_stream; }
    bool initialized() const { return m_init; }

    // add_field(pattern(field)) (bulk_communication_object.hpp:430-470)
    template<typename Field>
    void add_field(buffer_info<Field> bi)
    {
        static_assert(std::is_same_v<std::decay_t<decltype(bi.field->desc())>, ghx_field_desc>,
                      "bulk (zero-copy) exchange is implemented for structured fields");
        if (m_init) throw std::runtime_error("this bulk communication object has been initialized already");
        local_field f{bi.pattern, bi.local_index, bi.field->desc(),
                      const_cast<void*>(static_cast<const void*>(bi.field->data())), int(bi.field->domain_id()), 0,
                      int(alignof(typename Field::value_type))};
        for (const auto& g : m_fields) f.j += g.domain == f.domain;
        m_fields.push_back(f);
    }

    // init() (bulk_communication_object.hpp:472-560): collective
    void init()
    {
        if (m_init) return;
        const int me = m_ctx->rank();
        const int world = m_ctx->size();
        const auto gathered = m_ctx->get_transport().all_gather(serialize_mine());
        std::vector<remote_rank> all;
        for (const auto& g : gathered) all.push_back(deserialize(g));
        const auto& mine = all[std::size_t(me)];
        // this host's ranks get puts; the others' halos go through the remote part
        std::vector<char> local(std::size_t(world), 0);
        std::vector<std::int32_t> remote_ranks;
        int leader = -1, nlocal = 0;
        bool distinct = true;  // every rank of this host its own process: device epochs
        for (int r = 0; r < world; ++r)
        {
            local[std::size_t(r)] = all[std::size_t(r)].host == mine.host;
            if (!local[std::size_t(r)])
            {
                remote_ranks.push_back(r);
                continue;
            }
            if (leader < 0) leader = r;
            ++nlocal;
            for (int q = 0; q < r; ++q)
                if (local[std::size_t(q)] && all[std::size_t(q)].pid == all[std::size_t(r)].pid) distinct = false;
        }
        distinct = distinct && nlocal > 1;
        // the flag block is indexed by node-local position (its size follows the ranks per
        // host, not the world size)
        std::vector<std::int32_t> pos(std::size_t(world), -1);
        for (int r = 0, k = 0; r < world; ++r)
            if (local[std::size_t(r)]) pos[std::size_t(r)] = k++;
        // one flag block per host: its lowest rank creates it, publishes the name in a second
        // round, the others attach, the creator unlinks it once all have
        std::string name;
        if (distinct && me == leader)
        {
            name = "/ghx_ep_" + std::to_string(getpid()) + "_" +
                   std::to_string(reinterpret_cast<std::uintptr_t>(this) & 0xffffffu);
            check_ghx(ghx_epochs_create(name.c_str(), 1, nlocal, pos[std::size_t(me)], epoch_timeout, &m_ep),
                      "ghx_epochs_create");
        }
        if (world > 1)
        {
            const auto names = m_ctx->get_transport().all_gather(std::vector<char>(name.begin(), name.end()));
            if (distinct && me != leader)
            {
                const auto& ln = names[std::size_t(leader)];
                check_ghx(ghx_epochs_create(std::string(ln.begin(), ln.end()).c_str(), 0, nlocal,
                                            pos[std::size_t(me)], epoch_timeout, &m_ep),
                          "ghx_epochs_create");
            }
            barrier();  // every rank attached
            if (distinct && me == leader) (void)ghx_epochs_unlink(name.c_str());
        }
        if (m_ep)
        {
            std::vector<std::int32_t> srcs, tgts;
            for (const auto& f : m_fields)
                for (int dir = 0; dir < 2; ++dir)
                    for (const auto& h : halos(*f.pattern, f.local_index, dir))
                    {
                        const int rr = std::get<1>(h);
                        auto& v = dir == 0 ? tgts : srcs;
                        const std::int32_t lr = pos[std::size_t(rr)];  // node-local index
                        if (rr != me && local[std::size_t(rr)] && std::find(v.begin(), v.end(), lr) == v.end())
                            v.push_back(lr);
                    }
            std::sort(srcs.begin(), srcs.end());
            std::sort(tgts.begin(), tgts.end());
            check_ghx(ghx_epochs_peers(m_ep, srcs.data(), std::int32_t(srcs.size()), tgts.data(),
                                       std::int32_t(tgts.size())),
                      "ghx_epochs_peers");
            check_hip(hipEventCreateWithFlags(&m_after, hipEventDisableTiming), "hipEventCreate");
            check_hip(hipEventCreateWithFlags(&m_done, hipEventDisableTiming), "hipEventCreate");
        }
        if (!remote_ranks.empty())
        {
            // the remote part: each pattern container filtered to the other hosts' ranks, every
            // field registered with it, exchanged by a communication_object
            std::map<const pattern_container*, std::size_t> filtered;
            for (const auto& f : m_fields)
            {
                if (!filtered.count(f.pattern))
                {
                    ghx_pattern* out = nullptr;
                    check_ghx(ghx_pattern_filter(f.pattern->handle(), remote_ranks.data(),
                                                 std::int32_t(remote_ranks.size()), 1, &out),
                              "ghx_pattern_filter");
                    m_rpcs.push_back(std::make_unique<pattern_container>(out));
                    filtered[f.pattern] = m_rpcs.size() - 1;
                }
                ghx_exchange_item it;
                std::memset(&it, 0, sizeof(it));
                it.pattern = m_rpcs[filtered[f.pattern]]->handle();
                it.local_index = f.local_index;
                it.kind = 0;
                it.field = f.desc;
                it.align = f.align;
                m_ritems.push_back(it);
                m_rptrs.push_back(f.data);
            }
            m_remote = std::make_unique<communication_object>(*m_ctx);
        }
        std::map<std::tuple<int, int, int>, std::pair<int, int>> target;  // (rank, domain, j)
        for (std::size_t r = 0; r < all.size(); ++r)
            for (std::size_t i = 0; i < all[r].fields.size(); ++i)
                target[{int(r), all[r].fields[i].domain, all[r].fields[i].j}] = {int(r), int(i)};
        std::vector<msg> msgs;
        for (std::size_t k = 0; k < m_fields.size(); ++k)
        {
            const auto& f = m_fields[k];
            for (auto& [rid, rr, tag, boxes] : halos(*f.pattern, f.local_index, 0))
            {
                if (!local[std::size_t(rr)]) continue;  // the remote part's
                const auto t = target.find({rr, rid, f.j});
                if (t == target.end())
                    throw std::runtime_error("rank " + std::to_string(rr) + " registered no field #" +
                                             std::to_string(f.j) + " for domain " + std::to_string(rid));
                const auto& tf = all[std::size_t(t->second.first)].fields[std::size_t(t->second.second)];
                const std::vector<ghx_box>* tb = nullptr;
                for (const auto& key : tf.recv)
                    if (key.remote_id == f.domain && key.tag == tag) tb = &key.boxes;
                if (!tb)
                    throw std::runtime_error("no receive halo on rank " + std::to_string(rr) + " for domain " +
                                             std::to_string(f.domain) + ", tag " + std::to_string(tag));
                msgs.push_back({int(k), std::move(boxes), t->second, tb});
            }
        }
        // map every target field once: own fields and fields of ranks in this process directly,
        // the others through their IPC handles
        std::map<std::pair<int, int>, void*> ptr_of;
        for (const auto& m : msgs)
        {
            if (ptr_of.count(m.target)) continue;
            const auto& owner = all[std::size_t(m.target.first)];
            const auto& tf = owner.fields[std::size_t(m.target.second)];
            if (owner.pid == mine.pid)
                ptr_of[m.target] = reinterpret_cast<void*>(std::uintptr_t(tf.raw));
            else
            {
                void *base = nullptr, *ptr = nullptr;
                check_ghx(ghx_ipc_import(tf.ipc, tf.offset, &base, &ptr), "ghx_ipc_import");
                m_imports.push_back(base);
                ptr_of[m.target] = ptr;
            }
        }
        // put plans (one launch each) of <= 64 messages, <= 64 source and <= 64 target fields
        std::vector<msg> chunk;
        std::vector<int> srcs;
        std::vector<std::pair<int, int>> dsts;
        for (std::size_t i = 0; i <= msgs.size(); ++i)
        {
            const bool end = i == msgs.size();
            const bool full =
                !end && (chunk.size() == GHX_MAX_SLOTS ||
                         (std::find(srcs.begin(), srcs.end(), msgs[i].src) == srcs.end() &&
                          srcs.size() == GHX_MAX_SLOTS) ||
                         (std::find(dsts.begin(), dsts.end(), msgs[i].target) == dsts.end() &&
                          dsts.size() == GHX_MAX_SLOTS));
            if ((end || full) && !chunk.empty())
            {
                make_put(chunk, srcs, dsts, all, ptr_of);
                chunk.clear();
                srcs.clear();
                dsts.clear();
            }
            if (end) break;
            if (std::find(srcs.begin(), srcs.end(), msgs[i].src) == srcs.end()) srcs.push_back(msgs[i].src);
            if (std::find(dsts.begin(), dsts.end(), msgs[i].target) == dsts.end()) dsts.push_back(msgs[i].target);
            chunk.push_back(std::move(msgs[i]));
        }
        m_init = true;
    }

    // exchange() (bulk_communication_object.hpp:600-704): collective. `after`: the stream this
    // rank's kernels that read or write the fields run on (null: the whole device is drained).
    bulk_handle exchange(hipStream_t after = nullptr)
    {
        if (!m_init) init();
        communication_handle rh;
        if (m_ep)
        {
            // stream-ordered: the object's stream follows `after` (or the device), the epochs
            // and puts run on it, and `after` follows it again
            if (after)
            {
                check_hip(hipEventRecord(m_after, after), "hipEventRecord");
                check_hip(hipStreamWaitEvent(m_stream, m_after, 0), "hipStreamWaitEvent");
            }
            else check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
            if (m_remote) rh = m_remote->start(after, m_ritems, m_rptrs);  // other hosts' halos
            check_ghx(ghx_epochs_enqueue(m_ep, 0, m_stream), "ghx_epochs_enqueue(open)");
            for (auto& p : m_puts)
                check_ghx(ghx_put_execute(p.h, p.src.data(), std::int32_t(p.src.size()), p.dst.data(),
                                          std::int32_t(p.dst.size()), m_stream),
                          "ghx_put_execute");
            check_ghx(ghx_epochs_enqueue(m_ep, 1, m_stream), "ghx_epochs_enqueue(close)");
            check_hip(hipEventRecord(m_done, m_stream), "hipEventRecord");
            if (after)
            {
                check_hip(hipStreamWaitEvent(after, m_done, 0), "hipStreamWaitEvent");
                rh.schedule_wait(after);
            }
            return {m_done, m_ep, rh};
        }
        if (after) check_hip(hipStreamSynchronize(after), "hipStreamSynchronize");
        else check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
        if (m_remote) rh = m_remote->start(nullptr, m_ritems, m_rptrs);
        barrier();  // every target open
        for (auto& p : m_puts)
            check_ghx(ghx_put_execute(p.h, p.src.data(), std::int32_t(p.src.size()), p.dst.data(),
                                      std::int32_t(p.dst.size()), m_stream),
                      "ghx_put_execute");
        check_hip(hipStreamSynchronize(m_stream), "hipStreamSynchronize");
        barrier();  // every halo of every rank written
        if (after) rh.schedule_wait(after);
        return {nullptr, nullptr, rh};
    }

    // tests: the host name this rank reports (several hosts emulated in one process)
    void set_host_name(std::string host)
    {
        if (m_init) throw std::runtime_error("set_host_name before init()");
        m_host = std::move(host);
    }
    bool has_remote_part() const { return m_remote != nullptr; }

    // bytes moved per exchange by this rank's puts
    std::uint64_t bytes_per_exchange() const
    {
        std::uint64_t tot = 0;
        for (const auto& p : m_puts)
        {
            std::uint64_t b = 0;
            check_ghx(ghx_put_info(p.h, &b, nullptr), "ghx_put_info");
            tot += b;
        }
        return tot;
    }
    std::size_t num_puts() const { return m_puts.size(); }
};

inline bulk_communication_object make_bulk_communication_object(context& ctx)
{
    return bulk_communication_object(ctx);
}
}  // namespace ghex_amd
