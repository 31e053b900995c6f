// ghx_copier.hip — device<->host staging copies on chosen SDMA engines (the NIC-side path of the
// halo exchange: D2H after the pack, H2D before the unpack; SURVEY §8(f) #3, reference
// arch_traits.hpp:51-75 / communication_object.hpp:611-637, 715-729, where oomph stages).
//
// Why not hipMemcpyAsync: the runtime picks the copy engine itself, and on the MI355X boxes both
// directions often land on one engine (they then serialise: 25.4 MB each way in 0.91 ms,
// ~56 GB/s together) or one direction on an engine that is slow or shared (measured 12.7-30 GB/s
// D2H on some engines, 56 GB/s on others; profiles/r03_sdma_engines_box*.jsonl). With D2H and
// H2D on two distinct fast engines both directions run at once: 88-95 GB/s together.
// ghx_copier_create probes engines 0-3 with short copies, ranks them per direction, and keeps
// the pair with the best concurrent rate; copies then go through
// hsa_amd_memory_async_copy_on_engine on those engines. Completion is an HSA signal per copy
// (a small ring); an H2D copy may depend on a D2H copy's signal (the SDMA engine waits for it, no
// host round trip), which is how a chunked round trip overlaps the two directions. Every host
// wait has a deadline: a copy that does not complete reports an error instead of hanging.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "ghx_guard.hpp"

namespace ghx
{
namespace
{
constexpr int kRing = 256;         // signals in flight per copier
constexpr int kProbeEngines = 4;   // engines 0-3 serve host copies at full rate (4+ do not)

struct agents
{
    hsa_agent_t gpu{}, cpu{};
    bool have_gpu = false, have_cpu = false;
    uint32_t bdf = 0, domain = 0;
};

hsa_status_t find_agents(hsa_agent_t a, void* data)
{
    auto* g = static_cast<agents*>(data);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !g->have_cpu)
    {
        g->cpu = a;
        g->have_cpu = true;
    }
    if (t == HSA_DEVICE_TYPE_GPU && !g->have_gpu)
    {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_BDFID), &bdf);
        hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
        if (bdf == g->bdf && dom == g->domain)
        {
            g->gpu = a;
            g->have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

// One wave per workgroup, 32 workgroups per XCD of the queried count (blocks are dealt
// round-robin over the XCDs): a system-scope acquire invalidates the XCD's L2, so kernels queued after it
// cannot hit lines that a copy engine has replaced behind the caches' back (copies issued
// through HSA are invisible to the HIP runtime, which would otherwise add this acquire itself).
__global__ __launch_bounds__(64) void k_acquire()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

void hsa_check(hsa_status_t s, const char* what)
{
    if (s != HSA_STATUS_SUCCESS)
    {
        const char* msg = nullptr;
        hsa_status_string(s, &msg);
        throw invalid(std::string(what) + ": " + (msg ? msg : "HSA error"));
    }
}
}  // namespace
}  // namespace ghx

using namespace ghx;

struct ghx_copier
{
    agents ag;
    int engine[2] = {0, 1};        // [0] D2H, [1] H2D
    float rate[3] = {0, 0, 0};     // GB/s: D2H alone, H2D alone, both at once (probe)
    hsa_signal_t sig[kRing];
    uint64_t next = 0;             // tickets: next one to hand out
    double timeout_s = 30.0;
    bool inited = false;
    int nsig = 0;
    int acquire_groups = 256;      // k_acquire grid: 32 per XCD

    ~ghx_copier()
    {
        for (int i = 0; i < nsig; ++i)
        {
            // a copy still in flight keeps its signal: wait (bounded) before destroying it
            hsa_signal_wait_scacquire(sig[i], HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_BLOCKED);
            hsa_signal_destroy(sig[i]);
        }
        // hsa_init is reference counted and the HIP runtime holds the runtime open anyway; no
        // hsa_shut_down here, so a copier destroyed late in process teardown cannot be the one
        // that closes the runtime under HIP
    }

    hsa_signal_t& slot(uint64_t ticket) { return sig[ticket % kRing]; }

    // enqueue one copy; dep: ticket whose completion it waits for on the engine (or ~0)
    uint64_t submit(void* dst, const void* src, size_t n, int dir, uint64_t dep, bool force_engine = true)
    {
        const uint64_t t = next;
        hsa_signal_t d{};
        uint32_t nd = 0;
        if (dep != ~uint64_t(0))
        {
            if (dep >= t || t - dep > kRing - 1) throw invalid("dependency ticket out of the window");
            d = slot(dep);
            nd = 1;
        }
        if (t >= kRing) wait(t - kRing);  // the slot's previous copy must be done before reuse
        hsa_signal_t& s = slot(t);
        hsa_signal_store_screlease(s, 1);
        const auto eng = hsa_amd_sdma_engine_id_t(1u << engine[dir]);
        const hsa_status_t st =
            dir == 0 ? hsa_amd_memory_async_copy_on_engine(dst, ag.cpu, src, ag.gpu, n, nd, nd ? &d : nullptr, s,
                                                           eng, force_engine)
                     : hsa_amd_memory_async_copy_on_engine(dst, ag.gpu, src, ag.cpu, n, nd, nd ? &d : nullptr, s,
                                                           eng, force_engine);
        if (st != HSA_STATUS_SUCCESS)
        {
            // refused: the slot stays free (a signal left at 1 would read as a copy that never ends)
            hsa_signal_store_screlease(s, 0);
            hsa_check(st, dir == 0 ? "hsa_amd_memory_async_copy_on_engine(D2H)"
                                   : "hsa_amd_memory_async_copy_on_engine(H2D)");
        }
        next = t + 1;
        return t;
    }

    void wait(uint64_t ticket)
    {
        if (ticket >= next) throw invalid("unknown copy ticket");
        if (next - ticket > kRing) return;  // long done: its slot was reused after it completed
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
        while (hsa_signal_wait_scacquire(slot(ticket), HSA_SIGNAL_CONDITION_LT, 1, 100000000ull,
                                         HSA_WAIT_STATE_BLOCKED) >= 1)
            if (std::chrono::steady_clock::now() > deadline)
                throw invalid("staging copy did not complete within the timeout");
    }
};

namespace
{
double probe_us(ghx_copier& c, const std::vector<std::pair<int, int>>& copies, void* dev, void* host,
                size_t n)
{
    // copies: (direction, engine); all at once; median of 5 after one warm-up
    std::vector<double> t;
    for (int rep = 0; rep < 6; ++rep)
    {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<uint64_t> tk;
        for (size_t k = 0; k < copies.size(); ++k)
        {
            const int dir = copies[k].first;
            const int keep = c.engine[dir];
            c.engine[dir] = copies[k].second;
            char* d = static_cast<char*>(dir == 0 ? host : dev) + k * n;
            const char* s = static_cast<const char*>(dir == 0 ? dev : host) + k * n;
            tk.push_back(c.submit(d, s, n, dir, ~uint64_t(0)));
            c.engine[dir] = keep;
        }
        for (auto x : tk) c.wait(x);
        if (rep) t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}
}  // namespace

extern "C" {

int ghx_copier_create(uint64_t probe_bytes, double timeout_s, ghx_copier** out)
{
    return guarded([&] {
        if (!out) throw invalid("null out");
        *out = nullptr;
        if (probe_bytes < 4096 || probe_bytes > (uint64_t(1) << 30)) throw invalid("probe_bytes must be in [4 KiB, 1 GiB]");
        if (!(timeout_s > 0)) throw invalid("timeout must be > 0");
        auto c = std::make_unique<ghx_copier>();
        c->timeout_s = timeout_s;
        int dev = 0, bus = 0, devno = 0, dom = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
            hipDeviceGetAttribute(&devno, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
            hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dev) != hipSuccess)
            throw hip_error("hipDeviceGetAttribute(PCI location)");
        // the acquire kernel must reach every XCD (each has its own L2): 32 one-wave workgroups
        // per XCD of the queried count (blocks are dealt round-robin over the XCDs)
        int xcc = 0;
        if (hipDeviceGetAttribute(&xcc, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || xcc < 1)
            throw hip_error("hipDeviceGetAttribute(number of XCCs)");
        c->acquire_groups = 32 * xcc;
        hsa_check(hsa_init(), "hsa_init");
        c->inited = true;
        c->ag.bdf = uint32_t(bus) << 8 | uint32_t(devno) << 3;
        c->ag.domain = uint32_t(dom);
        hsa_check(hsa_iterate_agents(find_agents, &c->ag), "hsa_iterate_agents");
        if (!c->ag.have_gpu || !c->ag.have_cpu) throw invalid("no HSA agent for this device / the host");
        for (int i = 0; i < kRing; ++i)
        {
            hsa_check(hsa_signal_create(0, 0, nullptr, &c->sig[i]), "hsa_signal_create");
            c->nsig = i + 1;
        }
        uint32_t m_d2h = 0, m_h2d = 0;
        hsa_check(hsa_amd_memory_copy_engine_status(c->ag.cpu, c->ag.gpu, &m_d2h), "copy_engine_status");
        hsa_check(hsa_amd_memory_copy_engine_status(c->ag.gpu, c->ag.cpu, &m_h2d), "copy_engine_status");
        // probe buffers: two of each kind (concurrent copies use disjoint halves)
        const size_t n = size_t(probe_bytes);
        void *d = nullptr, *h = nullptr;
        if (hipMalloc(&d, 2 * n) != hipSuccess) throw hip_error("hipMalloc(probe)");
        if (hipHostMalloc(&h, 2 * n, hipHostMallocDefault) != hipSuccess)
        {
            (void)hipFree(d);
            throw hip_error("hipHostMalloc(probe)");
        }
        std::memset(h, 0, 2 * n);
        try
        {
            // the status masks say which engines are idle at this instant (another process may
            // be copying); a busy engine still serves copies, so every engine 0-3 is probed and
            // only one that refuses a copy is left out
            (void)m_d2h;
            (void)m_h2d;
            double best[2][kProbeEngines];
            for (int dir = 0; dir < 2; ++dir)
                for (int e = 0; e < kProbeEngines; ++e)
                {
                    try
                    {
                        best[dir][e] = probe_us(*c, {{dir, e}}, d, h, n);
                    }
                    catch (const invalid&)
                    {
                        best[dir][e] = 1e30;
                    }
                }
            double pair_us = 1e30;
            for (int a = 0; a < kProbeEngines; ++a)
                for (int b = 0; b < kProbeEngines; ++b)
                {
                    if (a == b || best[0][a] > 1e29 || best[1][b] > 1e29) continue;
                    // (host buffer halves: D2H writes h[0,n), H2D reads h[n,2n) — disjoint)
                    double us = 1e30;
                    try
                    {
                        us = probe_us(*c, {{0, a}, {1, b}}, d, h, n);
                    }
                    catch (const invalid&)
                    {
                        continue;
                    }
                    if (us < pair_us)
                    {
                        pair_us = us;
                        c->engine[0] = a;
                        c->engine[1] = b;
                    }
                }
            if (pair_us > 1e29) throw invalid("no SDMA engine pair available for host copies");
            c->rate[0] = float(double(n) / best[0][c->engine[0]] / 1e3);
            c->rate[1] = float(double(n) / best[1][c->engine[1]] / 1e3);
            c->rate[2] = float(2.0 * double(n) / pair_us / 1e3);
        }
        catch (...)
        {
            (void)hipFree(d);
            (void)hipHostFree(h);
            throw;
        }
        (void)hipFree(d);
        (void)hipHostFree(h);
        *out = c.release();
        return GHX_OK;
    });
}

int ghx_copier_info(const ghx_copier* c, int32_t* d2h_engine, int32_t* h2d_engine, float* d2h_GBps,
                    float* h2d_GBps, float* both_GBps)
{
    return guarded([&] {
        if (!c) throw invalid("null copier");
        if (d2h_engine) *d2h_engine = c->engine[0];
        if (h2d_engine) *h2d_engine = c->engine[1];
        if (d2h_GBps) *d2h_GBps = c->rate[0];
        if (h2d_GBps) *h2d_GBps = c->rate[1];
        if (both_GBps) *both_GBps = c->rate[2];
        return GHX_OK;
    });
}

int ghx_copier_submit(ghx_copier* c, void* dst, const void* src, uint64_t bytes, int32_t direction,
                      int64_t after_ticket, uint64_t* ticket)
{
    return guarded([&] {
        if (!c || !dst || !src || !ticket) throw invalid("null argument");
        if (direction != 0 && direction != 1) throw invalid("direction must be 0 (D2H) or 1 (H2D)");
        if (bytes == 0) throw invalid("empty copy");
        *ticket = c->submit(dst, src, size_t(bytes), direction,
                            after_ticket < 0 ? ~uint64_t(0) : uint64_t(after_ticket));
        return GHX_OK;
    });
}

int ghx_copier_wait(ghx_copier* c, uint64_t ticket)
{
    return guarded([&] {
        if (!c) throw invalid("null copier");
        c->wait(ticket);
        return GHX_OK;
    });
}

int ghx_copier_acquire(const ghx_copier* c, ghx_stream stream)
{
    return guarded([&] {
        if (!c) throw invalid("null copier");
        hipLaunchKernelGGL(k_acquire, dim3(c->acquire_groups), dim3(64), 0, static_cast<hipStream_t>(stream));
        if (hipGetLastError() != hipSuccess) throw hip_error("k_acquire launch");
        return GHX_OK;
    });
}

int ghx_copier_destroy(ghx_copier* c)
{
    delete c;
    return GHX_OK;
}

}  // extern "C"
