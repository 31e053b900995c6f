// ghex_amd/transport.hpp — the transport a ghex_amd::communication_object moves its messages
// through, in place of the reference's oomph communicator (ext/oomph; used at
// include/ghex/communication_object.hpp:278-281, 633-660, 705-729).
//
// The reference's stream-aware branch (communication_object.hpp:703-714, 751-765) is the model:
// the pack is enqueued on a stream, the messages are posted as ONE group whose transfers start
// after the pack and complete before anything enqueued later on the same stream, and the unpack
// is enqueued behind them; the host never blocks inside an exchange. Two implementations:
//   * ghex_amd::rccl_transport (rccl_transport.hpp): one rank per GPU, ncclSend/ncclRecv in an
//     ncclGroupStart/End group over xGMI (RCCL);
//   * ghex_amd::loopback_transport (this file): several ranks as threads of one process sharing a
//     device (tests, and multi-domain runs on one GPU), device-to-device copies.
// Setup (pattern construction) needs one collective, all_gather of host bytes — the reference's
// ghex::mpi::communicator::all_gather (include/ghex/mpi/communicator.hpp:63-345).
#pragma once

#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

namespace ghex_amd
{
inline void check_hip(hipError_t e, const char* what)
{
    if (e != hipSuccess)
        throw std::runtime_error(std::string(what) + " failed: " + hipGetErrorString(e));
}

// One message of an exchange: a device buffer, its size, the peer rank and the tag (pattern tag
// + the communication object's per-container tag offset, communication_object.hpp:1049).
struct message
{
    void* data;
    std::size_t bytes;
    int peer;
    int tag;
};

class transport
{
  public:
    virtual ~transport() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // Setup-time collective: every rank contributes `mine`; returns all contributions in rank
    // order (sizes may differ per rank).
    virtual std::vector<std::vector<char>> all_gather(const std::vector<char>& mine) = 0;
    // One group of messages, ordered on `stream` (see above). Messages between one pair of
    // ranks are matched by tag; a (peer, tag) pair occurs at most once per direction.
    virtual void exchange(const std::vector<message>& sends, const std::vector<message>& recvs,
                          hipStream_t stream) = 0;
    // The messages with ONE peer, ordered on `stream` (a pipelined exchange posts one such group
    // per peer, each on its own stream, as soon as that peer's buffers are packed). A transport
    // whose groups are independent per peer may specialise it; by default it is one exchange().
    virtual void exchange_peer(int /*peer*/, const std::vector<message>& sends,
                               const std::vector<message>& recvs, hipStream_t stream)
    {
        exchange(sends, recvs, stream);
    }
};

// Round of the pair (a, b) in a round-robin tournament over `world` ranks (circle method):
// every rank meets every other exactly once, at most once per round. Every rank issues its
// per-peer groups in this one global order, so with streams that run in issue order (shared
// hardware queues, a communicator's own serialisation) every wait between ranks points to the
// same or an earlier round and no cycle can form.
inline int round_of(int a, int b, int world)
{
    const int m = world + (world % 2), q = m - 1;
    if (a > b) std::swap(a, b);
    if (q <= 0) return 0;
    if (b == q) return a;
    return ((a + b) * (m / 2)) % q;
}

// ---------------------------------------------------------------------------------------------
// loopback: ranks = threads of one process on one device
// ---------------------------------------------------------------------------------------------
class loopback_hub
{
  public:
    explicit loopback_hub(int n_ranks)
    : m_n{n_ranks}
    , m_slots(std::size_t(n_ranks))
    {
        if (n_ranks < 1) throw std::runtime_error("loopback_hub: need at least one rank");
    }
    int size() const { return m_n; }

  private:
    friend class loopback_transport;
    struct posted
    {
        const void* data;
        std::size_t bytes;
        hipEvent_t ready;  // recorded on the sender's stream after its pack
    };
    using key = std::tuple<int, int, int>;  // (src, dst, tag)

    int m_n;
    std::mutex m_mtx;
    std::condition_variable m_cv;
    // all_gather: generation-counted rendezvous
    std::vector<std::vector<char>> m_slots;
    std::vector<std::vector<char>> m_result;
    int m_arrived = 0;
    int m_departed = 0;
    std::uint64_t m_gen = 0;
    // data path: sends waiting for their receive, and receive-done events waiting for the sender
    std::map<key, std::deque<posted>> m_sends;
    std::map<key, std::deque<hipEvent_t>> m_done;
};

class loopback_transport : public transport
{
    loopback_hub* m_hub;
    int m_rank;

  public:
    loopback_transport(loopback_hub& hub, int rank)
    : m_hub{&hub}
    , m_rank{rank}
    {
        if (rank < 0 || rank >= hub.size()) throw std::runtime_error("loopback_transport: bad rank");
    }
    int rank() const override { return m_rank; }
    int size() const override { return m_hub->size(); }

    std::vector<std::vector<char>> all_gather(const std::vector<char>& mine) override
    {
        auto& h = *m_hub;
        std::unique_lock<std::mutex> lk(h.m_mtx);
        h.m_cv.wait(lk, [&] { return h.m_departed == 0; });  // previous round fully drained
        const std::uint64_t gen = h.m_gen;
        h.m_slots[std::size_t(m_rank)] = mine;
        if (++h.m_arrived == h.m_n)
        {
            h.m_result = h.m_slots;
            h.m_arrived = 0;
            h.m_departed = h.m_n;
            ++h.m_gen;
            h.m_cv.notify_all();
        }
        else
            h.m_cv.wait(lk, [&] { return h.m_gen != gen; });
        auto out = h.m_result;
        if (--h.m_departed == 0) h.m_cv.notify_all();
        return out;
    }

    // Sends are published with an event recorded after the pack on the sender's stream; each
    // receive makes the receiver's stream wait for that event, copies device to device, and
    // hands a completion event back, which the sender's stream waits for before anything it
    // enqueues later (its next pack may then overwrite the send buffer safely).
    void exchange(const std::vector<message>& sends, const std::vector<message>& recvs,
                  hipStream_t stream) override
    {
        auto& h = *m_hub;
        {
            std::lock_guard<std::mutex> lk(h.m_mtx);
            for (const auto& s : sends)
            {
                hipEvent_t ev;
                check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
                check_hip(hipEventRecord(ev, stream), "hipEventRecord");
                h.m_sends[{m_rank, s.peer, s.tag}].push_back({s.data, s.bytes, ev});
            }
        }
        h.m_cv.notify_all();
        for (const auto& r : recvs)
        {
            loopback_hub::posted p;
            {
                std::unique_lock<std::mutex> lk(h.m_mtx);
                const loopback_hub::key k{r.peer, m_rank, r.tag};
                h.m_cv.wait(lk, [&] {
                    auto it = h.m_sends.find(k);
                    return it != h.m_sends.end() && !it->second.empty();
                });
                auto& q = h.m_sends[k];
                p = q.front();
                q.pop_front();
            }
            if (p.bytes != r.bytes)
                throw std::runtime_error("loopback_transport: message size mismatch (peer " +
                                         std::to_string(r.peer) + ", tag " + std::to_string(r.tag) + ")");
            check_hip(hipStreamWaitEvent(stream, p.ready, 0), "hipStreamWaitEvent");
            check_hip(hipEventDestroy(p.ready), "hipEventDestroy");
            if (r.bytes)
                check_hip(hipMemcpyAsync(r.data, p.data, r.bytes, hipMemcpyDeviceToDevice, stream),
                          "hipMemcpyAsync");
            hipEvent_t done;
            check_hip(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate");
            check_hip(hipEventRecord(done, stream), "hipEventRecord");
            {
                std::lock_guard<std::mutex> lk(h.m_mtx);
                h.m_done[{r.peer, m_rank, r.tag}].push_back(done);
            }
            h.m_cv.notify_all();
        }
        for (const auto& s : sends)
        {
            hipEvent_t done;
            {
                std::unique_lock<std::mutex> lk(h.m_mtx);
                const loopback_hub::key k{m_rank, s.peer, s.tag};
                h.m_cv.wait(lk, [&] {
                    auto it = h.m_done.find(k);
                    return it != h.m_done.end() && !it->second.empty();
                });
                auto& q = h.m_done[k];
                done = q.front();
                q.pop_front();
            }
            check_hip(hipStreamWaitEvent(stream, done, 0), "hipStreamWaitEvent");
            check_hip(hipEventDestroy(done), "hipEventDestroy");
        }
    }
};
}  // namespace ghex_amd
