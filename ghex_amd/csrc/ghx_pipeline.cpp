// ghx_pipeline.cpp — per-peer exchange pipeline over RCCL point-to-point (xGMI inside a node).
//
// The reference packs every buffer on its own non-blocking, greatest-priority stream
// (include/ghex/device/cuda/stream.hpp:25-73; communication_object.hpp:568-597), posts each send
// when that buffer's pack has completed (communication_object.hpp:611-637, packer.hpp:73-96) and,
// with a stream-aware transport such as NCCL, queues each unpack behind its receive on the
// buffer's stream (:703-714, 751-765). Here each PEER RANK rides one of a few streams (lanes):
// its send buffers are packed there (one launch per buffer), one RCCL group {ncclRecv...,
// ncclSend...} with that peer follows on the same stream, then its recv buffers are unpacked — so
// a face message leaves as soon as its own pack is done, while the packs of the other lanes'
// buffers still run, and each unpack starts as soon as its own message has landed. Self messages (periodic wrap onto the same
// rank) are packed and unpacked on the caller's stream, never through RCCL. The caller's stream
// then waits for every peer stream.
//
// Each peer pair uses its OWN 2-rank communicator: NCCL serialises the operations of one
// communicator, so per-peer groups on a single world communicator would run one link at a time.
// Deadlock freedom with more streams than hardware queues (operations of streams that share a
// queue run in issue order): every rank issues its peers in the same global round order (a
// round-robin tournament schedule, computed by the caller), so every wait chain across ranks
// follows increasing rounds.
//
// RCCL is resolved at run time (dlopen) from the library the caller names — the one the
// process's torch already loaded — so libghx has no link-time RCCL dependency and shares that
// RCCL instance.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ghx_exchange.hpp"
#include "ghx_guard.hpp"

namespace ghx
{
namespace
{
struct rccl_api
{
    void* handle = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
rccl_api g_rccl;
std::mutex g_rccl_mtx;

const rccl_api& rccl()
{
    if (!g_rccl.handle) throw invalid("RCCL not loaded (ghx_rccl_open)");
    return g_rccl;
}

void nccl_check(ncclResult_t r, const char* what)
{
    if (r != ncclSuccess)
        throw hip_error(std::string(what) + " failed: " +
                        (g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "RCCL error"));
}

void hip_check(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw hip_error(what);
}

template<typename F>
void sym(void* h, const char* name, F& f)
{
    f = reinterpret_cast<F>(dlsym(h, name));
    if (!f) throw invalid(std::string("RCCL library lacks ") + name);
}
}  // namespace

struct pipeline
{
    struct peer
    {
        int32_t rank = -1;
        ncclComm_t comm = nullptr;
        int32_t comm_peer = 0;     // the peer's rank inside `comm`
        int lane = 0;              // which of the pipeline's streams carries this peer
        std::vector<int> sends, recvs;  // buffer indices, in matching order on both sides
    };
    const exchange_plan* ex = nullptr;
    std::vector<peer> peers;                    // issue order (global rounds)
    std::vector<std::pair<int, int>> local;     // (send, recv) buffers of self messages
    // Peer k rides stream k mod S (S = max_streams): the device runs few hardware queues
    // (GPU_MAX_HW_QUEUES, 4 by default), and streams beyond them share queues in an order
    // nobody chooses; dealing the peers over S streams in round order keeps each stream's
    // sequence in the global round order (so the cross-rank argument above still holds) and
    // puts the first S peers — the order every rank agrees on — on distinct streams.
    std::vector<hipStream_t> lanes;
    std::vector<hipEvent_t> lane_done;
    hipEvent_t start = nullptr;

    ~pipeline()
    {
        for (auto e : lane_done)
            if (e) (void)hipEventDestroy(e);
        for (auto s : lanes)
            if (s) (void)hipStreamDestroy(s);
        if (start) (void)hipEventDestroy(start);
    }

    void run(void* const* fptr, int nf, void* const* sbuf, int ns, void* const* rbuf, int nr,
             hipStream_t stream) const
    {
        if (ns < int(ex->send.size()) || nr < int(ex->recv.size()))
            throw invalid("pointer arrays do not cover the exchange's buffers");
        hip_check(hipEventRecord(start, stream), "hipEventRecord");
        for (hipStream_t l : lanes) hip_check(hipStreamWaitEvent(l, start, 0), "hipStreamWaitEvent");
        for (const auto& p : peers)
        {
            hipStream_t ps = lanes[size_t(p.lane)];
            for (int i : p.sends)
                if (ex->execute_buffer(0, i, fptr, nf, sbuf, ns, ps) != GHX_OK)
                    throw hip_error(std::string("pack: ") + get_error());
            const auto& R = rccl();
            nccl_check(R.GroupStart(), "ncclGroupStart");
            for (int j : p.recvs)
                nccl_check(R.Recv(rbuf[j], size_t(ex->recv[size_t(j)].size), ncclInt8, p.comm_peer,
                                  p.comm, ps),
                           "ncclRecv");
            for (int i : p.sends)
                nccl_check(R.Send(sbuf[i], size_t(ex->send[size_t(i)].size), ncclInt8, p.comm_peer,
                                  p.comm, ps),
                           "ncclSend");
            nccl_check(R.GroupEnd(), "ncclGroupEnd");
            for (int j : p.recvs)
                if (ex->execute_buffer(1, j, fptr, nf, rbuf, nr, ps) != GHX_OK)
                    throw hip_error(std::string("unpack: ") + get_error());
        }
        for (size_t l = 0; l < lanes.size(); ++l)
            hip_check(hipEventRecord(lane_done[l], lanes[l]), "hipEventRecord");
        for (const auto& [i, j] : local)
        {
            if (ex->execute_buffer(0, i, fptr, nf, sbuf, ns, stream) != GHX_OK)
                throw hip_error(std::string("pack: ") + get_error());
            if (rbuf[j] != sbuf[i])
                hip_check(hipMemcpyAsync(rbuf[j], sbuf[i], size_t(ex->send[size_t(i)].size),
                                         hipMemcpyDeviceToDevice, stream),
                          "hipMemcpyAsync");
            if (ex->execute_buffer(1, j, fptr, nf, rbuf, nr, stream) != GHX_OK)
                throw hip_error(std::string("unpack: ") + get_error());
        }
        for (hipEvent_t e : lane_done) hip_check(hipStreamWaitEvent(stream, e, 0), "hipStreamWaitEvent");
    }
};
}  // namespace ghx

struct ghx_pipeline : ghx::pipeline
{
};

using namespace ghx;

extern "C" {

int ghx_rccl_open(const char* path)
{
    return guarded([&] {
        std::lock_guard<std::mutex> lk(g_rccl_mtx);
        if (g_rccl.handle) return int(GHX_OK);
        void* h = dlopen(path && *path ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) throw invalid(std::string("dlopen RCCL: ") + dlerror());
        rccl_api a;
        sym(h, "ncclGetUniqueId", a.GetUniqueId);
        sym(h, "ncclCommInitRank", a.CommInitRank);
        sym(h, "ncclCommDestroy", a.CommDestroy);
        sym(h, "ncclCommGetAsyncError", a.CommGetAsyncError);
        sym(h, "ncclGroupStart", a.GroupStart);
        sym(h, "ncclGroupEnd", a.GroupEnd);
        sym(h, "ncclSend", a.Send);
        sym(h, "ncclRecv", a.Recv);
        sym(h, "ncclGetErrorString", a.GetErrorString);
        a.handle = h;
        g_rccl = a;
        return int(GHX_OK);
    });
}

int ghx_rccl_unique_id(unsigned char id[128])
{
    return guarded([&] {
        if (!id) throw invalid("null id");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
        ncclUniqueId u;
        nccl_check(rccl().GetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, &u, sizeof(u));
        return int(GHX_OK);
    });
}

int ghx_rccl_comm_init(const unsigned char id[128], int32_t nranks, int32_t rank, void** comm)
{
    return guarded([&] {
        if (!id || !comm) throw invalid("null argument");
        if (nranks < 1 || rank < 0 || rank >= nranks) throw invalid("bad nranks / rank");
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        ncclComm_t c = nullptr;
        nccl_check(rccl().CommInitRank(&c, nranks, u, rank), "ncclCommInitRank");
        *comm = c;
        return int(GHX_OK);
    });
}

int ghx_rccl_comm_destroy(void* comm)
{
    return guarded([&] {
        if (comm) nccl_check(rccl().CommDestroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
        return int(GHX_OK);
    });
}

int ghx_rccl_comm_check(void* comm)
{
    return guarded([&] {
        if (!comm) throw invalid("null comm");
        ncclResult_t r = ncclSuccess;
        nccl_check(rccl().CommGetAsyncError(static_cast<ncclComm_t>(comm), &r), "ncclCommGetAsyncError");
        nccl_check(r, "communicator");
        return int(GHX_OK);
    });
}

int ghx_pipeline_create(ghx_exchange* ex, int32_t my_rank, int32_t n_peers,
                        const int32_t* peer_ranks, void* const* comms, const int32_t* comm_ranks,
                        int32_t max_streams, ghx_pipeline** out)
{
    return guarded([&] {
        if (!ex || !out) throw invalid("null argument");
        if (max_streams < 1) throw invalid("max_streams must be >= 1");
        if (n_peers < 0 || (n_peers > 0 && (!peer_ranks || !comms || !comm_ranks)))
            throw invalid("bad peer arrays");
        *out = nullptr;
        ex->make_split();
        auto pl = std::make_unique<ghx_pipeline>();
        pl->ex = ex;
        hip_check(hipEventCreateWithFlags(&pl->start, hipEventDisableTiming), "hipEventCreate");
        int least = 0, greatest = 0;
        hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
        // messages between one pair of ranks: matched in issue order, so both sides sort them by
        // (tag, domain pair); a send key (remote, mine) equals the receiver's recv key (its, mine)
        auto order = [](const std::vector<xbuffer>& v) {
            return [&v](int a, int b) {
                const auto& x = v[size_t(a)];
                const auto& y = v[size_t(b)];
                if (x.tag != y.tag) return x.tag < y.tag;
                if (x.first_id != y.first_id) return x.first_id < y.first_id;
                return x.second_id < y.second_id;
            };
        };
        std::vector<char> routed_s(ex->send.size(), 0), routed_r(ex->recv.size(), 0);
        for (int32_t k = 0; k < n_peers; ++k)
        {
            if (!comms[k]) throw invalid("null communicator");
            for (int32_t q = 0; q < k; ++q)
                if (peer_ranks[q] == peer_ranks[k]) throw invalid("peer listed twice");
            if (!g_rccl.handle) throw invalid("RCCL not loaded (ghx_rccl_open)");
            ghx::pipeline::peer p;
            p.rank = peer_ranks[k];
            p.comm = static_cast<ncclComm_t>(comms[k]);
            p.comm_peer = comm_ranks[k];
            for (size_t i = 0; i < ex->send.size(); ++i)
                if (ex->send[i].rank == p.rank) p.sends.push_back(int(i)), routed_s[i] = 1;
            for (size_t j = 0; j < ex->recv.size(); ++j)
                if (ex->recv[j].rank == p.rank) p.recvs.push_back(int(j)), routed_r[j] = 1;
            std::sort(p.sends.begin(), p.sends.end(), order(ex->send));
            std::sort(p.recvs.begin(), p.recvs.end(), order(ex->recv));
            p.lane = int(k % max_streams);
            pl->peers.push_back(p);
        }
        const int n_lanes = std::min<int>(max_streams, n_peers);
        pl->lanes.assign(size_t(n_lanes), nullptr);
        pl->lane_done.assign(size_t(n_lanes), nullptr);
        for (int l = 0; l < n_lanes; ++l)
        {
            hip_check(hipStreamCreateWithPriority(&pl->lanes[size_t(l)], hipStreamNonBlocking, greatest),
                      "hipStreamCreateWithPriority");
            hip_check(hipEventCreateWithFlags(&pl->lane_done[size_t(l)], hipEventDisableTiming),
                      "hipEventCreate");
        }
        // everything else must be a self message: recv j <- the send buffer of the same pair
        for (size_t j = 0; j < ex->recv.size(); ++j)
        {
            if (routed_r[j]) continue;
            const auto& r = ex->recv[j];
            if (r.rank != my_rank) throw invalid("a peer rank has no communicator");
            int found = -1;
            for (size_t i = 0; i < ex->send.size() && found < 0; ++i)
                if (!routed_s[i] && ex->send[i].rank == my_rank && ex->send[i].first_id == r.first_id &&
                    ex->send[i].second_id == r.second_id && ex->send[i].size == r.size)
                    found = int(i);
            if (found < 0) throw invalid("self message without its send buffer");
            routed_s[size_t(found)] = 1;
            pl->local.emplace_back(found, int(j));
        }
        for (size_t i = 0; i < ex->send.size(); ++i)
            if (!routed_s[i]) throw invalid("a send buffer has no receiver in the pipeline");
        *out = pl.release();
        return int(GHX_OK);
    });
}

int ghx_pipeline_run(const ghx_pipeline* pl, void* const* field_ptrs, int32_t n_fields,
                     void* const* send_buffers, int32_t n_send, void* const* recv_buffers,
                     int32_t n_recv, ghx_stream stream)
{
    return guarded([&] {
        if (!pl) throw invalid("null pipeline");
        pl->run(field_ptrs, n_fields, send_buffers, n_send, recv_buffers, n_recv,
                static_cast<hipStream_t>(stream));
        return int(GHX_OK);
    });
}

int ghx_pipeline_destroy(ghx_pipeline* pl)
{
    return guarded([&] {
        delete pl;
        return int(GHX_OK);
    });
}

}  // extern "C"
