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
    std::printf("{\"tool\": \"tools/sync_latency.hip\", \"unit\": \"us\", \"reps\": %d, "
                "\"host_load_sys\": %.3f, \"dev_load_agent\": %.3f, \"dev_load_sys\": %.3f, "
                "\"wbl2_clean\": %.3f, \"wbl2_dirty64k\": %.3f, \"inv_sys\": %.3f, "
                "\"graph_empty_1wg\": %.3f, \"graph_empty_32wg\": %.3f}\n",
                reps, best[kHostSys], best[kDevAgent], best[kDevSys], best[kWblClean],
                best[kWblDirty], best[kInv], g1, g32);
    return 0;
}
