// tests/cpp/shm_transport.hpp — TEST INFRASTRUCTURE, not product (transports are out of scope,
// SURVEY §2 row 9): ranks as separate PROCESSES of one host, meeting in a named POSIX
// shared-memory segment: the setup all_gather and a host-staged exchange (device buffer -> the
// segment's pages -> device buffer). In the reference's terms: the MPI communicator's all_gather
// of the setup (include/ghex/mpi/communicator.hpp:63-345) and oomph's host-buffer message path
// (include/ghex/arch_traits.hpp:51-75, communication_object.hpp:611-637) on one node.
//
// It needs neither RCCL nor MPI, so any number of processes may share one GPU: this is what lets
// the process-per-rank forms of the C++ objects — the bulk object's device epochs above all —
// run on a one-GPU box, where RCCL refuses two ranks per device (`Duplicate GPU detected`).
// Between GPUs in production the RCCL transport (rccl_transport.hpp) is the one to use.
//
//   shm_transport t("/myjob_ghx", rank, world);   // every rank the same name and sizes
//   ghex_amd::context ctx(t);
//
// Rank 0 creates the segment (O_EXCL: a leftover of a killed job is an error, not reused), the
// others attach, and rank 0 unlinks the name once every rank has attached — nothing is left in
// /dev/shm after the constructors return, whatever happens later. The segment is sparse: only
// the pages a rank writes are allocated.
//
// Layout: a header (barrier counter + generation), one all_gather slot per rank, and one channel
// per ordered rank pair (src, dst) holding ONE posted message group at a time (a sequence pair
// posted/consumed). exchange(): the stream is drained (the pack is done), every send group is
// posted (all messages to one peer in tag order, D2H into the channel), then every receive group
// is taken (H2D from the channel, in tag order, checked against the expected sizes). A channel is
// reused once its consumer has taken the previous group, so ranks that run the same sequence of
// exchanges never wait on each other in a cycle; per-peer groups (exchange_peer, the pipelined
// form) post and take one pair's group, in the global round order the caller uses.
// Every wait is bounded (`timeout_s`): a peer that died or never arrives becomes an exception.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <map>
#include <thread>

#include <ghex_amd/transport.hpp>

namespace ghex_amd
{
class shm_transport : public transport
{
    static constexpr std::uint64_t kMagic = 0x67687873686d7631ull;  // "ghxshmv1"
    static constexpr std::size_t kPage = 4096;

    struct header
    {
        std::atomic<std::uint64_t> ready;  // kMagic once rank 0 has laid the segment out
        std::atomic<std::uint64_t> count;  // barrier arrivals
        std::atomic<std::uint64_t> gen;    // barrier generation
        std::uint64_t world, slot_bytes, channel_bytes;
    };
    struct slot
    {
        std::uint64_t bytes;  // the data follows the 64-B slot header
    };
    struct channel
    {
        std::atomic<std::uint64_t> posted;    // groups posted by src
        std::atomic<std::uint64_t> consumed;  // groups taken by dst
        std::uint64_t bytes;                  // size of the posted group
    };
    static_assert(sizeof(header) <= kPage && sizeof(channel) <= 64 && sizeof(slot) <= 64, "layout");
    static_assert(std::atomic<std::uint64_t>::is_always_lock_free, "process-shared atomics");

    std::string m_name;
    int m_rank, m_size;
    std::size_t m_slot_bytes, m_channel_bytes, m_slot_stride, m_channel_stride, m_total;
    char* m_base = nullptr;
    bool m_unlinked = false;
    double m_timeout;

    static std::size_t round_up(std::size_t v, std::size_t a) { return (v + a - 1) / a * a; }
    header& hdr() const { return *reinterpret_cast<header*>(m_base); }
    char* slot_at(int r) const { return m_base + kPage + std::size_t(r) * m_slot_stride; }
    char* channel_at(int src, int dst) const
    {
        return m_base + kPage + std::size_t(m_size) * m_slot_stride +
               (std::size_t(src) * std::size_t(m_size) + std::size_t(dst)) * m_channel_stride;
    }
    channel& chan(int src, int dst) const { return *reinterpret_cast<channel*>(channel_at(src, dst)); }

    template<typename Pred>
    void wait_until(Pred pred, const char* what, int peer = -1) const
    {
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned spin = 0; !pred(); ++spin)
        {
            if (spin < 1024)
                std::this_thread::yield();
            else
            {
                std::this_thread::sleep_for(std::chrono::microseconds(20));
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > m_timeout)
                    throw std::runtime_error("shm_transport: rank " + std::to_string(m_rank) + " waited " +
                                             std::to_string(int(m_timeout)) + " s in " + what +
                                             (peer >= 0 ? " for rank " + std::to_string(peer) : std::string()));
            }
        }
    }

    void unlink_name()
    {
        if (m_rank == 0 && !m_unlinked)
        {
            (void)shm_unlink(m_name.c_str());
            m_unlinked = true;
        }
    }

  public:
    // `name`: a POSIX shm name ("/..."), the same on every rank of the job and not in use.
    // `slot_bytes`: the largest all_gather contribution; `channel_bytes`: the largest message
    // group one rank sends another in one exchange (tag/size headers included, 16 B per message
    // + 8 B). Both only reserve address space.
    shm_transport(std::string name, int rank, int size, std::size_t slot_bytes = std::size_t(16) << 20,
                  std::size_t channel_bytes = std::size_t(64) << 20, double timeout_s = 60.0)
    : m_name{std::move(name)}
    , m_rank{rank}
    , m_size{size}
    , m_slot_bytes{slot_bytes}
    , m_channel_bytes{channel_bytes}
    , m_timeout{timeout_s}
    {
        if (size < 1 || rank < 0 || rank >= size) throw std::runtime_error("shm_transport: bad rank/size");
        if (m_name.size() < 2 || m_name[0] != '/' || m_name.find('/', 1) != std::string::npos)
            throw std::runtime_error("shm_transport: the name must look like \"/name\"");
        m_slot_stride = round_up(64 + slot_bytes, kPage);
        m_channel_stride = round_up(64 + channel_bytes, kPage);
        m_total = kPage + std::size_t(size) * m_slot_stride + std::size_t(size) * std::size_t(size) * m_channel_stride;
        int fd = -1;
        if (rank == 0)
        {
            fd = shm_open(m_name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
            if (fd < 0)
                throw std::runtime_error("shm_transport: cannot create " + m_name + ": " + std::strerror(errno) +
                                         (errno == EEXIST ? " (a segment of that name exists: choose another name, "
                                                            "or shm_unlink a leftover)"
                                                          : ""));
            if (ftruncate(fd, off_t(m_total)) != 0)
            {
                const int e = errno;
                close(fd);
                (void)shm_unlink(m_name.c_str());
                throw std::runtime_error(std::string("shm_transport: ftruncate failed: ") + std::strerror(e));
            }
        }
        else
        {
            // the creator may not have got there yet: retry until the name exists at full size
            try
            {
                wait_until(
                    [&] {
                        if (fd < 0) fd = shm_open(m_name.c_str(), O_RDWR, 0600);
                        struct stat st;
                        return fd >= 0 && fstat(fd, &st) == 0 && std::size_t(st.st_size) == m_total;
                    },
                    "attach (is rank 0 running, with the same name and sizes?)", 0);
            }
            catch (...)
            {
                if (fd >= 0) close(fd);
                throw;
            }
        }
        void* p = mmap(nullptr, m_total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED)
        {
            if (rank == 0) (void)shm_unlink(m_name.c_str());
            throw std::runtime_error(std::string("shm_transport: mmap failed: ") + std::strerror(errno));
        }
        m_base = static_cast<char*>(p);
        auto& h = hdr();
        if (rank == 0)
        {
            // fresh pages are zero: counters at 0; publish the geometry last
            h.world = std::uint64_t(size);
            h.slot_bytes = slot_bytes;
            h.channel_bytes = channel_bytes;
            h.ready.store(kMagic, std::memory_order_release);
        }
        else
        {
            wait_until([&] { return h.ready.load(std::memory_order_acquire) == kMagic; }, "attach", 0);
            if (h.world != std::uint64_t(size) || h.slot_bytes != slot_bytes || h.channel_bytes != channel_bytes)
                throw std::runtime_error("shm_transport: rank " + std::to_string(rank) +
                                         " was given other sizes than rank 0");
        }
        try
        {
            barrier();  // every rank has attached
        }
        catch (...)
        {
            // no destructor runs for a half-built object: leave nothing behind
            unlink_name();
            munmap(m_base, m_total);
            m_base = nullptr;
            throw;
        }
        unlink_name();  // nothing left in /dev/shm from here on
    }
    shm_transport(const shm_transport&) = delete;
    shm_transport& operator=(const shm_transport&) = delete;
    ~shm_transport() override
    {
        unlink_name();
        if (m_base) munmap(m_base, m_total);
    }

    int rank() const override { return m_rank; }
    int size() const override { return m_size; }

    // sense-free counting barrier: the last arriver resets the count before it opens the next
    // generation, so nobody can arrive at the next barrier before the reset
    void barrier()
    {
        auto& h = hdr();
        const std::uint64_t g = h.gen.load(std::memory_order_acquire);
        if (h.count.fetch_add(1, std::memory_order_acq_rel) + 1 == std::uint64_t(m_size))
        {
            h.count.store(0, std::memory_order_relaxed);
            h.gen.store(g + 1, std::memory_order_release);
        }
        else
            wait_until([&] { return h.gen.load(std::memory_order_acquire) != g; }, "barrier");
    }

    std::vector<std::vector<char>> all_gather(const std::vector<char>& mine) override
    {
        if (mine.size() > m_slot_bytes)
            throw std::runtime_error("shm_transport: all_gather contribution of " + std::to_string(mine.size()) +
                                     " B exceeds slot_bytes " + std::to_string(m_slot_bytes));
        barrier();  // everyone has read the previous round's slots
        char* s = slot_at(m_rank);
        reinterpret_cast<slot*>(s)->bytes = mine.size();
        if (!mine.empty()) std::memcpy(s + 64, mine.data(), mine.size());
        barrier();
        std::vector<std::vector<char>> out(static_cast<std::size_t>(m_size));
        for (int r = 0; r < m_size; ++r)
        {
            const char* q = slot_at(r);
            const std::size_t n = reinterpret_cast<const slot*>(q)->bytes;
            out[std::size_t(r)].assign(q + 64, q + 64 + n);
        }
        return out;
    }

    void exchange(const std::vector<message>& sends, const std::vector<message>& recvs,
                  hipStream_t stream) override
    {
        auto by_tag = [](const message& a, const message& b) { return a.tag < b.tag; };
        std::map<int, std::vector<message>> out, in;
        for (const auto& m : sends) out[m.peer].push_back(m);
        for (const auto& m : recvs) in[m.peer].push_back(m);
        for (auto* g : {&out, &in})
            for (auto& [peer, ms] : *g)
            {
                if (peer < 0 || peer >= m_size) throw std::runtime_error("shm_transport: bad peer rank");
                std::sort(ms.begin(), ms.end(), by_tag);
            }
        check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");  // the packs are done
        for (const auto& [peer, ms] : out) post(peer, ms);
        for (const auto& [peer, ms] : in) take(peer, ms, stream);
    }

  private:
    void post(int peer, const std::vector<message>& ms)
    {
        std::size_t need = 8;
        for (const auto& m : ms) need += 16 + round_up(m.bytes, 8);
        if (need > m_channel_bytes)
            throw std::runtime_error("shm_transport: " + std::to_string(need) + " B to rank " + std::to_string(peer) +
                                     " exceed channel_bytes " + std::to_string(m_channel_bytes));
        channel& c = chan(m_rank, peer);
        const std::uint64_t seq = c.posted.load(std::memory_order_relaxed);
        wait_until([&] { return c.consumed.load(std::memory_order_acquire) == seq; }, "send", peer);
        char* d = channel_at(m_rank, peer) + 64;
        const std::uint64_t n = ms.size();
        std::memcpy(d, &n, 8);
        std::size_t off = 8;
        for (const auto& m : ms)
        {
            const std::int64_t tag = m.tag;
            const std::uint64_t bytes = m.bytes;
            std::memcpy(d + off, &tag, 8);
            std::memcpy(d + off + 8, &bytes, 8);
            off += 16;
            if (bytes) check_hip(hipMemcpy(d + off, m.data, bytes, hipMemcpyDeviceToHost), "hipMemcpy(D2H)");
            off += round_up(bytes, 8);
        }
        c.bytes = off;
        c.posted.store(seq + 1, std::memory_order_release);
    }

    void take(int peer, const std::vector<message>& ms, hipStream_t stream)
    {
        channel& c = chan(peer, m_rank);
        const std::uint64_t seq = c.consumed.load(std::memory_order_relaxed);
        wait_until([&] { return c.posted.load(std::memory_order_acquire) > seq; }, "receive", peer);
        const char* d = channel_at(peer, m_rank) + 64;
        std::uint64_t n = 0;
        std::memcpy(&n, d, 8);
        if (n != ms.size())
            throw std::runtime_error("shm_transport: rank " + std::to_string(peer) + " sent " + std::to_string(n) +
                                     " messages, rank " + std::to_string(m_rank) + " expects " +
                                     std::to_string(ms.size()));
        std::size_t off = 8;
        for (const auto& m : ms)  // both sides in tag order
        {
            std::int64_t tag = 0;
            std::uint64_t bytes = 0;
            std::memcpy(&tag, d + off, 8);
            std::memcpy(&bytes, d + off + 8, 8);
            off += 16;
            if (tag != m.tag || bytes != m.bytes)
                throw std::runtime_error("shm_transport: message mismatch from rank " + std::to_string(peer) +
                                         " (tag " + std::to_string(tag) + ", " + std::to_string(bytes) +
                                         " B; expected tag " + std::to_string(m.tag) + ", " +
                                         std::to_string(m.bytes) + " B)");
            if (bytes)
                check_hip(hipMemcpyAsync(m.data, d + off, bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync(H2D)");
            off += round_up(bytes, 8);
        }
        // the channel's pages are reused by the sender's next group only after these copies
        check_hip(hipStreamSynchronize(stream), "hipStreamSynchronize");
        c.consumed.store(seq + 1, std::memory_order_release);
    }
};
}  // namespace ghex_amd
