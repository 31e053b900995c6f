// sync_latency.hip — what the device epochs' building blocks cost on this GPU (developer
// measurement behind DESIGN §5: the fixed cost of the zero-copy exchanges). One wave, timed in
// the kernel with the 100 MHz wall clock, each figure the mean over `reps` dependent repetitions:
//   host_load_sys      relaxed system-scope 8-B load of pinned host memory (a flag in the shm block)
//   dev_load_agent     relaxed agent-scope 8-B load of device memory (sc1)
//   dev_load_sys       relaxed system-scope 8-B load of device memory (sc0 sc1)
//   wbl2_clean         system-scope release (buffer_wbl2 sc0 sc1 + wait), nothing dirty
//   wbl2_dirty64k      the same after this wave stored 64 KiB
//   inv_sys            system-scope acquire (buffer_inv sc0 sc1 + wait)
// and, from the host, the per-launch time of chains of empty launches in one hipGraph:
//   graph_empty_1wg / graph_empty_32wg   (the floor of any extra launch per exchange)
//   handoff_one_way.*  one flag hand-off between two kernels on two streams (ping-pong / 2),
//                      flags in pinned host memory, fine-grained / uncached / plain device memory
// Output: one JSON line. Build: make -C tools bin/sync_latency.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
    do                                                                                  \
    {                                                                                   \
        if ((x) != hipSuccess)                                                          \
        {                                                                               \
            std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(x), __FILE__, \
                         __LINE__);                                                     \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

enum
{
    kHostSys,
    kDevAgent,
    kDevSys,
    kWblClean,
    kWblDirty,
    kInv,
    kN
};

__global__ __launch_bounds__(64) void k_lat(uint64_t* host, uint64_t* dev, uint64_t* scratch,
                                            int reps, uint64_t* out)
{
    const int lane = threadIdx.x;
    uint64_t acc = 0;
    uint64_t t[kN];
    // dependent loads: each address depends on the previous value (0 in memory)
    uint64_t t0 = wall_clock64();
    for (int i = 0; i < reps; ++i)
        acc += __hip_atomic_load(host + (acc & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    t[kHostSys] = wall_clock64() - t0;
    t0 = wall_clock64();
    for (int i = 0; i < reps; ++i)
        acc += __hip_atomic_load(dev + (acc & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t[kDevAgent] = wall_clock64() - t0;
    t0 = wall_clock64();
    for (int i = 0; i < reps; ++i)
        acc += __hip_atomic_load(dev + (acc & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    t[kDevSys] = wall_clock64() - t0;
    t0 = wall_clock64();
    for (int i = 0; i < reps; ++i)
    {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    t[kWblClean] = wall_clock64() - t0;
    uint64_t dirty = 0;
    for (int i = 0; i < reps; ++i)
    {
        uint4* s = reinterpret_cast<uint4*>(scratch);
        for (int k = 0; k < 64; ++k) s[k * 64 + lane] = make_uint4(i, k, lane, 0);  // 64 KiB
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t a = wall_clock64();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        dirty += wall_clock64() - a;
    }
    t[kWblDirty] = dirty;
    t0 = wall_clock64();
    for (int i = 0; i < reps; ++i)
    {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    t[kInv] = wall_clock64() - t0;
    if (lane == 0)
        for (int k = 0; k < kN; ++k) out[k] = t[k];
    if (acc == 12345) out[kN] = acc;  // keep the loads
}

__global__ void k_empty() {}

// Ping-pong between two one-wave kernels on two streams through two flags in the memory kind
// under test: one-way flag latency = round trip / 2 (the cost of one cross-rank hand-off of the
// epochs, without the host in between).
__global__ __launch_bounds__(64) void k_pingpong(uint64_t* mine, uint64_t* theirs, int n, int first,
                                                 uint64_t timeout, uint64_t* out)
{
    const uint64_t t0 = wall_clock64();
    for (int i = 0; i < n; ++i)
    {
        if (!first || i > 0)
        {
            const uint64_t want = uint64_t(i) + (first ? 0 : 1);
            while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want)
                if (wall_clock64() - t0 > timeout) return;
        }
        __hip_atomic_store(mine, uint64_t(i) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (threadIdx.x == 0) *out = wall_clock64() - t0;
}

static double pingpong_us(uint64_t* a, uint64_t* b, int khz)
{
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    uint64_t* out;
    CK(hipMalloc(&out, 16));
    double best = 1e30;
    for (int r = 0; r < 3; ++r)
    {
        CK(hipMemset(a, 0, 8));
        CK(hipMemset(b, 0, 8));
        CK(hipDeviceSynchronize());
        const int n = 2000;
        const uint64_t tmo = uint64_t(khz) * 1000ull * 5;  // 5 s
        hipLaunchKernelGGL(k_pingpong, dim3(1), dim3(64), 0, s1, a, b, n, 1, tmo, out);
        hipLaunchKernelGGL(k_pingpong, dim3(1), dim3(64), 0, s2, b, a, n, 0, tmo, out + 1);
        CK(hipDeviceSynchronize());
        uint64_t h[2];
        CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
        const double us = double(h[0]) / (double(khz) * 1e-3) / n / 2;  // one way
        if (us < best) best = us;
    }
    CK(hipFree(out));
    CK(hipStreamDestroy(s1));
    CK(hipStreamDestroy(s2));
    return best;
}

static double graph_chain_us(int groups, int n)
{
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(groups), dim3(64), 0, s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r)
    {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
    return best * 1e3 / n;
}

int main()
{
    const int reps = 200;
    uint64_t *host, *hdev, *dev, *scratch, *out;
    CK(hipHostMalloc(&host, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    for (int i = 0; i < 512; ++i) host[i] = 0;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), host, 0));
    CK(hipMalloc(&dev, 4096));
    CK(hipMemset(dev, 0, 4096));
    CK(hipMalloc(&scratch, 1 << 16));
    CK(hipMalloc(&out, 64 * 8));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    uint64_t h[kN];
    double best[kN];
    for (int k = 0; k < kN; ++k) best[k] = 1e30;
    for (int r = 0; r < 5; ++r)
    {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, hdev, dev, scratch, reps, out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
        for (int k = 0; k < kN; ++k)
        {
            const double us = double(h[k]) / (double(khz) * 1e-3) / reps;
            if (us < best[k]) best[k] = us;
        }
    }
    const double g1 = graph_chain_us(1, 200), g32 = graph_chain_us(32, 200);
    // one-way flag hand-off between two kernels, per memory kind
    uint64_t *hp, *hp_d, *fg, *uc, *pl;
    CK(hipHostMalloc(&hp, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hp_d), hp, 0));
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fg), 4096, hipDeviceMallocFinegrained));
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&uc), 4096, hipDeviceMallocUncached));
    CK(hipMalloc(&pl, 4096));
    const double pp_host = pingpong_us(hp_d, hp_d + 8, khz);
    const double pp_fine = pingpong_us(fg, fg + 8, khz);
    const double pp_unc = pingpong_us(uc, uc + 8, khz);
    const double pp_plain = pingpong_us(pl, pl + 8, khz);
    std::printf("{\"tool\": \"tools/sync_latency.hip\", \"unit\": \"us\", \"reps\": %d, "
                "\"host_load_sys\": %.3f, \"dev_load_agent\": %.3f, \"dev_load_sys\": %.3f, "
                "\"wbl2_clean\": %.3f, \"wbl2_dirty64k\": %.3f, \"inv_sys\": %.3f, "
                "\"graph_empty_1wg\": %.3f, \"graph_empty_32wg\": %.3f, "
                "\"handoff_one_way\": {\"host_pinned\": %.3f, \"device_finegrained\": %.3f, "
                "\"device_uncached\": %.3f, \"device_plain\": %.3f}}\n",
                reps, best[kHostSys], best[kDevAgent], best[kDevSys], best[kWblClean],
                best[kWblDirty], best[kInv], g1, g32, pp_host, pp_fine, pp_unc, pp_plain);
    return 0;
}
