// co_demo.cpp — drives the C++ communication object (include/ghex_amd/communication_object.hpp)
// the way a GHEX application drives ghex::communication_object, and checks every cell.
//
//   co_demo loopback PX PY PZ N H       PX*PY*PZ ranks as threads on device 0 (loopback
//                                        transport), one N^3 domain each of a periodic global
//                                        grid, two fields (double, float) in ONE exchange; every
//                                        cell of every rank vs the wrapped global index; twice
//                                        (the second exchange reuses the cached plan/buffers)
//   co_demo pipeloop PX PY PZ N H       the same with options.pipelined: per-peer lanes (pack,
//                                        transport::exchange_peer, unpack per peer, round order)
//   co_demo bulkloop PX PY PZ N H       the same two fields through the C++
//                                        bulk_communication_object (zero-copy puts between the
//                                        thread-ranks' fields, no buffers)
//   co_demo bulkhosts PX PY PZ N H K    bulkloop with the ranks spread over K emulated hosts
//                                        (rank r on host r % K): puts between ranks of one host,
//                                        the other halos through the bulk object's remote part
//   co_demo rma NRANKS                  test_local_rma.cpp's geometry (two domains per rank,
//                                        offset 3 > halo 2, double/float/int fields) through the
//                                        C++ bulk_communication_object
//   co_demo rccl N H SELF [PIPE]         one rank, RCCL communicator on device 0; SELF=1 sends the
//                                        self messages through ncclSend/ncclRecv (group), SELF=0
//                                        takes the fused self path; PIPE=1 the pipelined form
//   co_demo unstructured FILE LEVELS     ranks as threads, domains from FILE (per line:
//                                        "id n_gids gids... n_outer lids..."), one domain per rank;
//                                        value(lid, level) = dom*10000 + gid*100 + level
//                                        (test/unstructured/unstructured_test_case.hpp:345-388);
//                                        every halo value vs its owner's encoding
//   co_demo bench N H ITERS              one rank, host-inclusive microseconds per exchange
//                                        (exchange + wait) on the fused self path
//   co_demo shm NAME RANK PX PY PZ N H MODE [HOSTS]
//                                        ONE rank of a PX*PY*PZ job, this process (start one
//                                        process per rank; shm_transport NAME): MODE plain (one
//                                        group), pipe (per-peer lanes), direct (the pack writes
//                                        into the receivers' buffers over IPC, device epochs) or
//                                        bulk (zero-copy puts
//                                        over IPC with device epochs between the processes;
//                                        HOSTS > 0 spreads the ranks over emulated hosts, the
//                                        other hosts' halos through the bulk object's remote part)
//   co_demo shmgather NAME RANK WORLD ROUNDS [TIMEOUT_S]
//                                        the shm transport's all_gather alone (no GPU calls):
//                                        contributions of varying size, every byte checked
// Prints one JSON line per rank / result; exit status 0 iff every cell matched.
#include <ghex_amd/bulk_communication_object.hpp>
#include <ghex_amd/communication_object.hpp>
#include <ghex_amd/data_descriptor.hpp>
#include <ghex_amd/field_descriptor.hpp>
#include <ghex_amd/rccl_transport.hpp>
#include "shm_transport.hpp"  // test infrastructure: ranks as processes sharing the one test GPU

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <set>
#include <sstream>
#include <thread>

using namespace ghex_amd;
namespace R = ghex_amd::structured::regular;

namespace
{
struct cube
{
    int N, H, E;
    std::array<int, 3> parts, G, c;
    long idx(int x, int y, int z) const { return (long(z) * E + y) * E + x; }
    double expect(int x, int y, int z) const  // wrapped global linear index of local (x,y,z)
    {
        const int l[3] = {x, y, z};
        long g[3];
        for (int d = 0; d < 3; ++d) g[d] = ((long(c[d]) * N + l[d] - H) % G[d] + G[d]) % G[d];
        return double(g[0] + long(G[0]) * (g[1] + long(G[1]) * g[2]));
    }
    bool owned(int x, int y, int z) const
    {
        return x >= H && x < H + N && y >= H && y < H + N && z >= H && z < H + N;
    }
};

// one rank: its domain, two fields, exchange twice, count bad cells
long run_structured_rank(transport& t, const std::array<int, 3>& parts, int N, int H,
                         communication_object::options opt, int reps = 2, bool bulk = false,
                         int hosts = 0)
{
    check_hip(hipSetDevice(0), "hipSetDevice");
    context ctx(t);
    const int r = ctx.rank();
    cube cb{N, H, N + 2 * H, parts, {parts[0] * N, parts[1] * N, parts[2] * N},
            {r % parts[0], (r / parts[0]) % parts[1], r / (parts[0] * parts[1])}};
    R::domain_descriptor dom(r, {cb.c[0] * N, cb.c[1] * N, cb.c[2] * N},
                             {(cb.c[0] + 1) * N - 1, (cb.c[1] + 1) * N - 1, (cb.c[2] + 1) * N - 1});
    R::halo_generator hg{{0, 0, 0}, {cb.G[0] - 1, cb.G[1] - 1, cb.G[2] - 1}, {H, H, H, H, H, H},
                         {true, true, true}};
    auto pattern = R::make_pattern(ctx, hg, {dom});
    const long E3 = long(cb.E) * cb.E * cb.E;
    std::vector<double> hd(std::size_t(E3), -1.0);
    std::vector<float> hf(std::size_t(E3), -1.0f);
    for (int z = 0; z < cb.E; ++z)
        for (int y = 0; y < cb.E; ++y)
            for (int x = 0; x < cb.E; ++x)
                if (cb.owned(x, y, z))
                {
                    hd[std::size_t(cb.idx(x, y, z))] = cb.expect(x, y, z);
                    hf[std::size_t(cb.idx(x, y, z))] = float(cb.expect(x, y, z) + 1.0);
                }
    double* dd = nullptr;
    float* df = nullptr;
    check_hip(hipMalloc(&dd, std::size_t(E3) * 8), "hipMalloc");
    check_hip(hipMalloc(&df, std::size_t(E3) * 4), "hipMalloc");
    structured::field_descriptor<double, 3> fd(r, dd, {H, H, H}, {cb.E, cb.E, cb.E}, {2, 1, 0});
    structured::field_descriptor<float, 3> ff(r, df, {H, H, H}, {cb.E, cb.E, cb.E}, {2, 1, 0});
    communication_object co(ctx, opt);
    bulk_communication_object bco(ctx);
    if (bulk)
    {
        if (hosts > 0) bco.set_host_name("host" + std::to_string(r % hosts));  // emulated hosts
        bco.add_field(pattern(fd));
        bco.add_field(pattern(ff));
        bco.init();
    }
    long bad = 0;
    for (int rep = 0; rep < reps; ++rep)
    {
        check_hip(hipMemcpy(dd, hd.data(), std::size_t(E3) * 8, hipMemcpyHostToDevice), "hipMemcpy");
        check_hip(hipMemcpy(df, hf.data(), std::size_t(E3) * 4, hipMemcpyHostToDevice), "hipMemcpy");
        if (bulk)
            bco.exchange().wait();
        else
            co.exchange(pattern(fd), pattern(ff)).wait();
        std::vector<double> od(static_cast<std::size_t>(E3));
        std::vector<float> of(static_cast<std::size_t>(E3));
        check_hip(hipMemcpy(od.data(), dd, std::size_t(E3) * 8, hipMemcpyDeviceToHost), "hipMemcpy");
        check_hip(hipMemcpy(of.data(), df, std::size_t(E3) * 4, hipMemcpyDeviceToHost), "hipMemcpy");
        for (int z = 0; z < cb.E; ++z)
            for (int y = 0; y < cb.E; ++y)
                for (int x = 0; x < cb.E; ++x)
                {
                    const double e = cb.expect(x, y, z);
                    bad += od[std::size_t(cb.idx(x, y, z))] != e;
                    bad += of[std::size_t(cb.idx(x, y, z))] != float(e + 1.0);
                }
    }
    std::printf("{\"mode\":\"%s\",\"rank\":%d,\"plans\":%zu,\"puts\":%zu,\"remote\":%d,\"epochs\":%d,"
                "\"bad\":%ld}\n",
                bulk ? "bulk" : "structured", r, co.num_plans(), bco.num_puts(), bco.has_remote_part() ? 1 : 0,
                bco.device_epochs() ? 1 : 0, bad);
    (void)hipFree(dd);
    (void)hipFree(df);
    return bad;
}

int loopback(int px, int py, int pz, int N, int H, bool pipelined = false, bool bulk = false,
             int hosts = 0)
{
    const int n = px * py * pz;
    loopback_hub hub(n);
    std::vector<loopback_transport> ts;
    for (int r = 0; r < n; ++r) ts.emplace_back(hub, r);
    std::atomic<long> bad{0};
    std::atomic<int> errors{0};
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            try
            {
                communication_object::options opt;
                opt.pipelined = pipelined;
                bad += run_structured_rank(ts[std::size_t(r)], {px, py, pz}, N, H, opt, 2, bulk, hosts);
            }
            catch (const std::exception& e)
            {
                std::printf("{\"rank\":%d,\"error\":\"%s\"}\n", r, e.what());
                ++errors;
            }
        });
    for (auto& t : th) t.join();
    return (bad == 0 && errors == 0) ? 0 : 1;
}

int rccl(int N, int H, int self, int pipelined = 0)
{
    check_hip(hipSetDevice(0), "hipSetDevice");
    ncclComm_t comm;
    int dev = 0;
    check_nccl(ncclCommInitAll(&comm, 1, &dev), "ncclCommInitAll");
    long bad = 0;
    {
        rccl_transport t(comm);
        communication_object::options opt;
        opt.self_through_transport = self != 0;
        opt.pipelined = pipelined != 0;
        bad = run_structured_rank(t, {1, 1, 1}, N, H, opt);
    }
    check_nccl(ncclCommDestroy(comm), "ncclCommDestroy");
    return bad == 0 ? 0 : 1;
}

int unstructured_case(const char* file, int levels)
{
    struct dom
    {
        int id;
        std::vector<std::int64_t> gids, outer;
    };
    std::vector<dom> doms;
    std::ifstream in(file);
    std::string line;
    while (std::getline(in, line))
    {
        std::istringstream ss(line);
        dom d;
        long ng, no;
        if (!(ss >> d.id >> ng)) continue;
        d.gids.resize(std::size_t(ng));
        for (auto& g : d.gids) ss >> g;
        ss >> no;
        d.outer.resize(std::size_t(no));
        for (auto& l : d.outer) ss >> l;
        doms.push_back(d);
    }
    // owner of every gid: the domain where it is an inner cell
    std::map<std::int64_t, int> owner;
    for (const auto& d : doms)
    {
        std::set<std::int64_t> o(d.outer.begin(), d.outer.end());
        for (std::size_t l = 0; l < d.gids.size(); ++l)
            if (!o.count(std::int64_t(l))) owner[d.gids[l]] = d.id;
    }
    const int n = int(doms.size());
    loopback_hub hub(n);
    std::vector<loopback_transport> ts;
    for (int r = 0; r < n; ++r) ts.emplace_back(hub, r);
    std::atomic<long> bad{0};
    std::atomic<int> errors{0};
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            try
            {
                check_hip(hipSetDevice(0), "hipSetDevice");
                context ctx(ts[std::size_t(r)]);
                const auto& d = doms[std::size_t(r)];
                unstructured::domain_descriptor ud(d.id, d.gids, d.outer);
                auto pattern = unstructured::make_pattern(ctx, {}, {ud});
                const std::size_t ncell = d.gids.size();
                std::set<std::int64_t> o(d.outer.begin(), d.outer.end());
                std::vector<double> hv(ncell * std::size_t(levels), -1.0);
                for (std::size_t l = 0; l < ncell; ++l)
                    if (!o.count(std::int64_t(l)))
                        for (int k = 0; k < levels; ++k)
                            hv[l * std::size_t(levels) + std::size_t(k)] = d.id * 10000.0 + double(d.gids[l]) * 100 + k;
                double* dv = nullptr;
                check_hip(hipMalloc(&dv, hv.size() * 8), "hipMalloc");
                check_hip(hipMemcpy(dv, hv.data(), hv.size() * 8, hipMemcpyHostToDevice), "hipMemcpy");
                unstructured::data_descriptor<int, double> field(ud, dv, levels, true);
                communication_object co(ctx);
                co.exchange(pattern(field)).wait();
                std::vector<double> out(hv.size());
                check_hip(hipMemcpy(out.data(), dv, hv.size() * 8, hipMemcpyDeviceToHost), "hipMemcpy");
                long b = 0;
                for (std::size_t l = 0; l < ncell; ++l)
                    for (int k = 0; k < levels; ++k)
                    {
                        const int own = o.count(std::int64_t(l)) ? owner.at(d.gids[l]) : d.id;
                        b += out[l * std::size_t(levels) + std::size_t(k)] != own * 10000.0 + double(d.gids[l]) * 100 + k;
                    }
                std::printf("{\"mode\":\"unstructured\",\"rank\":%d,\"bad\":%ld}\n", r, b);
                bad += b;
                (void)hipFree(dv);
            }
            catch (const std::exception& e)
            {
                std::printf("{\"rank\":%d,\"error\":\"%s\"}\n", r, e.what());
                ++errors;
            }
        });
    for (auto& t : th) t.join();
    return (bad == 0 && errors == 0) ? 0 : 1;
}

// test/structured/regular/test_local_rma.cpp's simulation_1 geometry through the C++ bulk object:
// n ranks as threads, TWO domains per rank (ids 2r, 2r+1, local extent 4x3x2), fields allocated
// with offset 3 > halo 2 (extent 10x9x8), three value types per domain (double, float, int), one
// bulk object per rank with all six fields. Owned cell = wrapped global linear index + type
// number; after two exchanges every cell within the halo equals its wrapped value and every cell
// beyond it is untouched (-1).
template<typename T>
long rma_check(const std::vector<T>& h, const std::array<int, 3>& first, const std::array<int, 3>& G,
               int k)
{
    long bad = 0;
    for (int z = 0; z < 8; ++z)
        for (int y = 0; y < 9; ++y)
            for (int x = 0; x < 10; ++x)
            {
                const int l[3] = {x - 3, y - 3, z - 3};
                const int ext[3] = {4, 3, 2};
                bool in_halo = true;
                for (int d = 0; d < 3; ++d) in_halo = in_halo && l[d] >= -2 && l[d] < ext[d] + 2;
                long g[3];
                for (int d = 0; d < 3; ++d) g[d] = ((first[std::size_t(d)] + l[d]) % G[std::size_t(d)] + G[std::size_t(d)]) % G[std::size_t(d)];
                const T want = in_halo ? T(g[0] + long(G[0]) * (g[1] + long(G[1]) * g[2]) + k) : T(-1);
                bad += h[std::size_t((z * 9 + y) * 10 + x)] != want;
            }
    return bad;
}

int rma_case(int n)
{
    loopback_hub hub(n);
    std::vector<loopback_transport> ts;
    for (int r = 0; r < n; ++r) ts.emplace_back(hub, r);
    std::atomic<long> bad{0};
    std::atomic<int> errors{0};
    const std::array<int, 3> G{16, ((n - 1) / 2 + 1) * 3, 2};
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            try
            {
                check_hip(hipSetDevice(0), "hipSetDevice");
                context ctx(ts[std::size_t(r)]);
                std::vector<R::domain_descriptor> doms;
                for (int k = 0; k < 2; ++k)
                    doms.emplace_back(2 * r + k,
                                      std::array<int, 3>{((r % 2) * 2 + k) * 4, (r / 2) * 3, 0},
                                      std::array<int, 3>{((r % 2) * 2 + k + 1) * 4 - 1, (r / 2 + 1) * 3 - 1, 1});
                R::halo_generator hg{{0, 0, 0}, {G[0] - 1, G[1] - 1, G[2] - 1}, {2, 2, 2, 2, 2, 2},
                                     {true, true, true}};
                auto pattern = R::make_pattern(ctx, hg, doms);
                const std::size_t cells = 10 * 9 * 8;
                std::vector<double*> dd(2);
                std::vector<float*> df(2);
                std::vector<int*> di(2);
                auto fill = [&](auto* dev, int dom, int k) {
                    using T = std::remove_pointer_t<decltype(dev)>;
                    std::vector<T> h(cells, T(-1));
                    const auto& f = doms[std::size_t(dom)].first();
                    for (int z = 0; z < 2; ++z)
                        for (int y = 0; y < 3; ++y)
                            for (int x = 0; x < 4; ++x)
                                h[std::size_t(((z + 3) * 9 + y + 3) * 10 + x + 3)] =
                                    T(f[0] + x + long(G[0]) * (f[1] + y + long(G[1]) * (f[2] + z)) + k);
                    check_hip(hipMemcpy(dev, h.data(), cells * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
                };
                std::vector<std::unique_ptr<structured::field_descriptor<double, 3>>> fd;
                std::vector<std::unique_ptr<structured::field_descriptor<float, 3>>> ff;
                std::vector<std::unique_ptr<structured::field_descriptor<int, 3>>> fi;
                bulk_communication_object bco(ctx);
                for (int k = 0; k < 2; ++k)
                {
                    check_hip(hipMalloc(&dd[std::size_t(k)], cells * 8), "hipMalloc");
                    check_hip(hipMalloc(&df[std::size_t(k)], cells * 4), "hipMalloc");
                    check_hip(hipMalloc(&di[std::size_t(k)], cells * 4), "hipMalloc");
                    const int id = 2 * r + k;
                    fd.emplace_back(new structured::field_descriptor<double, 3>(id, dd[std::size_t(k)], {3, 3, 3}, {10, 9, 8}, {2, 1, 0}));
                    ff.emplace_back(new structured::field_descriptor<float, 3>(id, df[std::size_t(k)], {3, 3, 3}, {10, 9, 8}, {2, 1, 0}));
                    fi.emplace_back(new structured::field_descriptor<int, 3>(id, di[std::size_t(k)], {3, 3, 3}, {10, 9, 8}, {2, 1, 0}));
                }
                // registration order as the reference test: 1a 1b 2a 2b 3a 3b
                bco.add_field(pattern(*fd[0]));
                bco.add_field(pattern(*fd[1]));
                bco.add_field(pattern(*ff[0]));
                bco.add_field(pattern(*ff[1]));
                bco.add_field(pattern(*fi[0]));
                bco.add_field(pattern(*fi[1]));
                bco.init();
                long b = 0;
                for (int rep = 0; rep < 2; ++rep)
                {
                    for (int k = 0; k < 2; ++k)
                    {
                        fill(dd[std::size_t(k)], k, 0);
                        fill(df[std::size_t(k)], k, 1);
                        fill(di[std::size_t(k)], k, 2);
                    }
                    bco.exchange().wait();
                    for (int k = 0; k < 2; ++k)
                    {
                        std::vector<double> hd(cells);
                        std::vector<float> hf(cells);
                        std::vector<int> hi(cells);
                        check_hip(hipMemcpy(hd.data(), dd[std::size_t(k)], cells * 8, hipMemcpyDeviceToHost), "hipMemcpy");
                        check_hip(hipMemcpy(hf.data(), df[std::size_t(k)], cells * 4, hipMemcpyDeviceToHost), "hipMemcpy");
                        check_hip(hipMemcpy(hi.data(), di[std::size_t(k)], cells * 4, hipMemcpyDeviceToHost), "hipMemcpy");
                        const auto& f = doms[std::size_t(k)].first();
                        b += rma_check(hd, f, G, 0) + rma_check(hf, f, G, 1) + rma_check(hi, f, G, 2);
                    }
                }
                std::printf("{\"mode\":\"rma\",\"rank\":%d,\"puts\":%zu,\"bad\":%ld}\n", r, bco.num_puts(), b);
                bad += b;
                for (int k = 0; k < 2; ++k)
                {
                    (void)hipFree(dd[std::size_t(k)]);
                    (void)hipFree(df[std::size_t(k)]);
                    (void)hipFree(di[std::size_t(k)]);
                }
            }
            catch (const std::exception& e)
            {
                std::printf("{\"rank\":%d,\"error\":\"%s\"}\n", r, e.what());
                ++errors;
            }
        });
    for (auto& t : th) t.join();
    return (bad == 0 && errors == 0) ? 0 : 1;
}

// one rank per process over the shm transport (see the header)
int shm_rank(const char* name, int rank, int px, int py, int pz, int N, int H, const std::string& mode,
             int hosts)
{
    if (mode != "plain" && mode != "pipe" && mode != "bulk" && mode != "direct")
        throw std::runtime_error("MODE: plain|pipe|bulk|direct");
    const int n = px * py * pz;
    // channels sized for the largest message group of the test geometries (two fields)
    const std::size_t face = std::size_t(N + 2 * H) * std::size_t(N + 2 * H) * std::size_t(H) * 12;
    shm_transport t(name, rank, n, std::size_t(1) << 20, 8 + 26 * (16 + 8) + 26 * face);
    communication_object::options opt;
    opt.pipelined = mode == "pipe";
    opt.direct = mode == "direct";
    return run_structured_rank(t, {px, py, pz}, N, H, opt, 2, mode == "bulk", hosts) == 0 ? 0 : 1;
}

int shm_gather(const char* name, int rank, int world, int rounds, double timeout_s)
{
    shm_transport t(name, rank, world, std::size_t(1) << 16, 4096, timeout_s);
    long bad = 0;
    for (int round = 0; round < rounds; ++round)
    {
        std::vector<char> mine(std::size_t((rank * 131 + round * 17) % 4000), char(rank * 7 + round));
        const auto all = t.all_gather(mine);
        bad += all.size() != std::size_t(world);
        for (int q = 0; q < world && q < int(all.size()); ++q)
        {
            bad += all[std::size_t(q)].size() != std::size_t((q * 131 + round * 17) % 4000);
            for (char c : all[std::size_t(q)]) bad += c != char(q * 7 + round);
        }
        if (round % 7 == 3) t.barrier();
    }
    std::printf("{\"mode\":\"shmgather\",\"rank\":%d,\"rounds\":%d,\"bad\":%ld}\n", rank, rounds, bad);
    return bad == 0 ? 0 : 1;
}

int bench(int N, int H, int iters)
{
    check_hip(hipSetDevice(0), "hipSetDevice");
    loopback_hub hub(1);
    loopback_transport t(hub, 0);
    context ctx(t);
    const int E = N + 2 * H;
    R::domain_descriptor dom(0, {0, 0, 0}, {N - 1, N - 1, N - 1});
    R::halo_generator hg{{0, 0, 0}, {N - 1, N - 1, N - 1}, {H, H, H, H, H, H}, {true, true, true}};
    auto pattern = R::make_pattern(ctx, hg, {dom});
    double* dd = nullptr;
    check_hip(hipMalloc(&dd, std::size_t(E) * E * E * 8), "hipMalloc");
    check_hip(hipMemset(dd, 0, std::size_t(E) * E * E * 8), "hipMemset");
    structured::field_descriptor<double, 3> fd(0, dd, {H, H, H}, {E, E, E}, {2, 1, 0});
    auto co = make_communication_object(ctx);
    for (int i = 0; i < 10; ++i) co.exchange(pattern(fd)).wait();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) co.exchange(pattern(fd)).wait();
    const double us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    const double bytes = 4.0 * (double(E) * E * E - double(N) * N * N) * 8;
    std::printf("{\"mode\":\"bench\",\"N\":%d,\"H\":%d,\"us_per_exchange\":%.2f,\"GBps\":%.1f}\n", N, H, us,
                bytes / us / 1e3);
    (void)hipFree(dd);
    return 0;
}
}  // namespace

int main(int argc, char** argv)
{
    try
    {
        const std::string mode = argc > 1 ? argv[1] : "";
        if (mode == "loopback" && argc == 7)
            return loopback(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                            std::atoi(argv[6]));
        if (mode == "pipeloop" && argc == 7)
            return loopback(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                            std::atoi(argv[6]), true);
        if (mode == "bulkloop" && argc == 7)
            return loopback(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                            std::atoi(argv[6]), false, true);
        if (mode == "bulkhosts" && argc == 8)
            return loopback(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                            std::atoi(argv[6]), false, true, std::atoi(argv[7]));
        if (mode == "rma" && argc == 3) return rma_case(std::atoi(argv[2]));
        if (mode == "rccl" && argc == 5) return rccl(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]));
        if (mode == "rccl" && argc == 6)
            return rccl(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]));
        if (mode == "unstructured" && argc == 4) return unstructured_case(argv[2], std::atoi(argv[3]));
        if (mode == "bench" && argc == 5) return bench(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]));
        if (mode == "shm" && (argc == 10 || argc == 11))
            return shm_rank(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), std::atoi(argv[6]),
                            std::atoi(argv[7]), std::atoi(argv[8]), argv[9], argc == 11 ? std::atoi(argv[10]) : 0);
        if (mode == "shmgather" && (argc == 6 || argc == 7))
            return shm_gather(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]),
                              argc == 7 ? std::atof(argv[6]) : 60.0);
    }
    catch (const std::exception& e)
    {
        std::printf("{\"error\":\"%s\"}\n", e.what());
        return 2;
    }
    std::fprintf(stderr, "usage: see the header of co_demo.cpp\n");
    return 2;
}
