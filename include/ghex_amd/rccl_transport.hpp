// ghex_amd/rccl_transport.hpp — RCCL (NCCL API on ROCm, over xGMI inside a node) as the
// transport of a ghex_amd::communication_object: one rank per GPU, the messages of an exchange
// posted as one ncclGroupStart/ncclGroupEnd group of ncclRecv/ncclSend on the exchange stream —
// the reference's NCCL backend of oomph with its start_group/end_group bracketing
// (include/ghex/communication_object.hpp:278-281). NCCL has no tags: messages between one pair
// of ranks are matched in issue order, so both sides issue them sorted by (peer, tag); the tag of
// a send buffer equals the tag of the matching receive buffer by construction of the pattern.
// Link with -lrccl.
#pragma once

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>

#include "transport.hpp"

namespace ghex_amd
{
inline void check_nccl(ncclResult_t r, const char* what)
{
    if (r != ncclSuccess)
        throw std::runtime_error(std::string(what) + " failed: " + ncclGetErrorString(r));
}

class rccl_transport : public transport
{
    ncclComm_t m_comm;
    int m_rank = 0, m_size = 1;

  public:
    // `comm` is owned by the caller (created with ncclCommInitRank / ncclCommInitAll).
    explicit rccl_transport(ncclComm_t comm)
    : m_comm{comm}
    {
        check_nccl(ncclCommUserRank(comm, &m_rank), "ncclCommUserRank");
        check_nccl(ncclCommCount(comm, &m_size), "ncclCommCount");
    }
    int rank() const override { return m_rank; }
    int size() const override { return m_size; }

    // sizes, then the bytes padded to the largest contribution, through ncclAllGather on device
    // staging buffers (setup time: synchronous).
    std::vector<std::vector<char>> all_gather(const std::vector<char>& mine) override
    {
        hipStream_t s;
        check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
        const std::size_t n = std::size_t(m_size);
        std::int64_t* dsz = nullptr;
        check_hip(hipMalloc(&dsz, (n + 1) * sizeof(std::int64_t)), "hipMalloc");
        const std::int64_t my = std::int64_t(mine.size());
        check_hip(hipMemcpyAsync(dsz + n, &my, sizeof(my), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
        check_nccl(ncclAllGather(dsz + n, dsz, 1, ncclInt64, m_comm, s), "ncclAllGather");
        std::vector<std::int64_t> sizes(n);
        check_hip(hipMemcpyAsync(sizes.data(), dsz, n * sizeof(std::int64_t), hipMemcpyDeviceToHost, s),
                  "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        const std::size_t mx = std::size_t(std::max<std::int64_t>(1, *std::max_element(sizes.begin(), sizes.end())));
        char* dbuf = nullptr;
        check_hip(hipMalloc(&dbuf, mx * (n + 1)), "hipMalloc");
        std::vector<char> padded(mx, 0);
        std::memcpy(padded.data(), mine.data(), mine.size());
        check_hip(hipMemcpyAsync(dbuf + mx * n, padded.data(), mx, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
        check_nccl(ncclAllGather(dbuf + mx * n, dbuf, mx, ncclChar, m_comm, s), "ncclAllGather");
        std::vector<char> all(mx * n);
        check_hip(hipMemcpyAsync(all.data(), dbuf, mx * n, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
        check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        (void)hipFree(dbuf);
        (void)hipFree(dsz);
        (void)hipStreamDestroy(s);
        std::vector<std::vector<char>> out(n);
        for (std::size_t r = 0; r < n; ++r)
            out[r].assign(all.begin() + std::ptrdiff_t(r * mx), all.begin() + std::ptrdiff_t(r * mx + std::size_t(sizes[r])));
        return out;
    }

    void exchange(const std::vector<message>& sends, const std::vector<message>& recvs,
                  hipStream_t stream) override
    {
        auto by_peer_tag = [](const message& a, const message& b) {
            return a.peer != b.peer ? a.peer < b.peer : a.tag < b.tag;
        };
        std::vector<message> s(sends), r(recvs);
        std::sort(s.begin(), s.end(), by_peer_tag);
        std::sort(r.begin(), r.end(), by_peer_tag);
        check_nccl(ncclGroupStart(), "ncclGroupStart");
        for (const auto& m : r)
            check_nccl(ncclRecv(m.data, m.bytes, ncclChar, m.peer, m_comm, stream), "ncclRecv");
        for (const auto& m : s)
            check_nccl(ncclSend(m.data, m.bytes, ncclChar, m.peer, m_comm, stream), "ncclSend");
        check_nccl(ncclGroupEnd(), "ncclGroupEnd");
    }
};
}  // namespace ghex_amd
