// sdma_bench.cpp — developer measurement (not product): why device<->host staging of the 512^3
// H=2 message (25,362,944 B per direction) moves ~63 GB/s with both directions at once instead
// of ~2 x 53-55. Separates the candidate limits:
//   host_memcpy      host DRAM bandwidth between two pinned buffers (1 and 16 threads)
//   hip_d2h / hip_h2d / hip_both   hipMemcpyAsync on one / two streams (what ghex_amd uses)
//   sdma e_d2h,e_h2d  hsa_amd_memory_async_copy_on_engine with explicit SDMA engines: each
//                     direction alone per engine, and both directions on the same / on
//                     distinct engines
// Every figure is the median of `reps` runs; one JSON line each.
// Build: hipcc -O2 --offload-arch=gfx950 tools/sdma_bench.cpp -o tools/bin/sdma_bench -lhsa-runtime64 -pthread
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#define CK(x)                                                                     \
    do                                                                            \
    {                                                                             \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess)                                                     \
        {                                                                         \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)
#define HK(x)                                                         \
    do                                                                \
    {                                                                 \
        hsa_status_t s_ = (x);                                        \
        if (s_ != HSA_STATUS_SUCCESS)                                 \
        {                                                             \
            printf("HSA error %d at line %d\n", int(s_), __LINE__);   \
            exit(1);                                                  \
        }                                                             \
    } while (0)

static hsa_agent_t g_gpu{}, g_cpu{};
static bool g_have_gpu = false, g_have_cpu = false;

static hsa_status_t pick(hsa_agent_t a, void*)
{
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) g_gpu = a, g_have_gpu = true;
    if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) g_cpu = a, g_have_cpu = true;
    return HSA_STATUS_SUCCESS;
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static double time_us(int reps, const std::function<void()>& f)
{
    std::vector<double> t;
    f();  // warm
    for (int i = 0; i < reps; ++i)
    {
        auto t0 = std::chrono::steady_clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    return median(t);
}

int main(int argc, char** argv)
{
    const size_t n = argc > 1 ? size_t(atoll(argv[1])) : size_t(25362944);
    const int reps = argc > 2 ? atoi(argv[2]) : 15;
    CK(hipSetDevice(0));
    void *d_a, *d_b, *h_a, *h_b, *h_c;
    CK(hipMalloc(&d_a, n));
    CK(hipMalloc(&d_b, n));
    CK(hipHostMalloc(&h_a, n, hipHostMallocDefault));
    CK(hipHostMalloc(&h_b, n, hipHostMallocDefault));
    CK(hipHostMalloc(&h_c, n, hipHostMallocDefault));
    memset(h_a, 1, n);
    memset(h_b, 2, n);
    memset(h_c, 3, n);
    CK(hipMemset(d_a, 4, n));
    CK(hipMemset(d_b, 5, n));
    CK(hipDeviceSynchronize());
    auto line = [&](const char* what, double us, size_t bytes) {
        printf("{\"what\": \"%s\", \"bytes\": %zu, \"us\": %.1f, \"GBps\": %.2f}\n", what, bytes, us,
               double(bytes) / us / 1e3);
        fflush(stdout);
    };

    // host DRAM control: pinned -> pinned memcpy, 1 and 16 threads
    line("host_memcpy_1thread", time_us(reps, [&] { memcpy(h_c, h_a, n); }), 2 * n);
    line("host_memcpy_16threads", time_us(reps, [&] {
             std::vector<std::thread> th;
             const size_t c = n / 16;
             for (int i = 0; i < 16; ++i)
                 th.emplace_back([&, i] { memcpy((char*)h_c + i * c, (char*)h_a + i * c, i == 15 ? n - 15 * c : c); });
             for (auto& t : th) t.join();
         }),
         2 * n);

    // hipMemcpyAsync, as ghex_amd's staging does
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    line("hip_d2h", time_us(reps, [&] { CK(hipMemcpyAsync(h_a, d_a, n, hipMemcpyDeviceToHost, s1)); CK(hipStreamSynchronize(s1)); }), n);
    line("hip_h2d", time_us(reps, [&] { CK(hipMemcpyAsync(d_b, h_b, n, hipMemcpyHostToDevice, s2)); CK(hipStreamSynchronize(s2)); }), n);
    line("hip_both_two_streams", time_us(reps, [&] {
             CK(hipMemcpyAsync(h_a, d_a, n, hipMemcpyDeviceToHost, s1));
             CK(hipMemcpyAsync(d_b, h_b, n, hipMemcpyHostToDevice, s2));
             CK(hipStreamSynchronize(s1));
             CK(hipStreamSynchronize(s2));
         }),
         2 * n);

    // the same pair of copies on other kinds of streams (torch's pool streams are created with a
    // priority; ghex_amd's pipeline lanes with the greatest priority)
    {
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t p1, p2, b1, b2;
        CK(hipStreamCreateWithPriority(&p1, hipStreamNonBlocking, hi));
        CK(hipStreamCreateWithPriority(&p2, hipStreamNonBlocking, hi));
        CK(hipStreamCreate(&b1));
        CK(hipStreamCreate(&b2));
        auto pair = [&](hipStream_t a, hipStream_t b) {
            CK(hipMemcpyAsync(h_a, d_a, n, hipMemcpyDeviceToHost, a));
            CK(hipMemcpyAsync(d_b, h_b, n, hipMemcpyHostToDevice, b));
            CK(hipStreamSynchronize(a));
            CK(hipStreamSynchronize(b));
        };
        line("hip_both_priority_streams", time_us(reps, [&] { pair(p1, p2); }), 2 * n);
        line("hip_both_blocking_streams", time_us(reps, [&] { pair(b1, b2); }), 2 * n);
        line("hip_both_one_stream", time_us(reps, [&] { pair(s1, s1); }), 2 * n);
        line("hip_both_null_and_stream", time_us(reps, [&] { pair(nullptr, s2); }), 2 * n);
        // chunked D2H -> H2D of the same bytes (the host-staged step's dependency), 4 chunks
        hipEvent_t ev[8];
        for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (int chunks : {2, 4, 8})
        {
            const size_t c = (n + chunks - 1) / chunks;
            char name[64];
            snprintf(name, sizeof name, "hip_chunked_roundtrip_%d", chunks);
            line(name, time_us(reps, [&] {
                     for (int k = 0; k < chunks; ++k)
                     {
                         const size_t o = k * c, m = std::min(c, n - o);
                         CK(hipMemcpyAsync((char*)h_a + o, (char*)d_a + o, m, hipMemcpyDeviceToHost, s1));
                         CK(hipEventRecord(ev[k], s1));
                         CK(hipStreamWaitEvent(s2, ev[k], 0));
                         CK(hipMemcpyAsync((char*)d_b + o, (char*)h_a + o, m, hipMemcpyHostToDevice, s2));
                     }
                     CK(hipStreamSynchronize(s2));
                 }),
                 2 * n);
        }
        line("hip_serial_roundtrip", time_us(reps, [&] {
                 CK(hipMemcpyAsync(h_a, d_a, n, hipMemcpyDeviceToHost, s1));
                 CK(hipMemcpyAsync(d_b, h_a, n, hipMemcpyHostToDevice, s1));
                 CK(hipStreamSynchronize(s1));
             }),
             2 * n);
        for (auto& e : ev) CK(hipEventDestroy(e));
    }

    // explicit SDMA engines
    HK(hsa_iterate_agents(pick, nullptr));
    if (!g_have_gpu || !g_have_cpu)
    {
        printf("{\"error\": \"no HSA GPU/CPU agent\"}\n");
        return 0;
    }
    uint32_t m_d2h = 0, m_h2d = 0;
    HK(hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &m_d2h));
    HK(hsa_amd_memory_copy_engine_status(g_gpu, g_cpu, &m_h2d));
    printf("{\"engines_free_d2h_mask\": %u, \"engines_free_h2d_mask\": %u}\n", m_d2h, m_h2d);
    hsa_signal_t sa, sb;
    HK(hsa_signal_create(1, 0, nullptr, &sa));
    HK(hsa_signal_create(1, 0, nullptr, &sb));
    auto copy = [&](bool d2h, int eng, hsa_signal_t sig) {
        hsa_signal_store_relaxed(sig, 1);
        if (d2h)
            HK(hsa_amd_memory_async_copy_on_engine(h_a, g_cpu, d_a, g_gpu, n, 0, nullptr, sig,
                                                   hsa_amd_sdma_engine_id_t(1u << eng), true));
        else
            HK(hsa_amd_memory_async_copy_on_engine(d_b, g_gpu, h_b, g_cpu, n, 0, nullptr, sig,
                                                   hsa_amd_sdma_engine_id_t(1u << eng), true));
    };
    auto wait = [&](hsa_signal_t sig) {
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    };
    const int n_eng = 16;
    std::vector<int> engs;
    for (int e = 0; e < n_eng; ++e)
        if (((m_d2h | m_h2d) >> e) & 1u) engs.push_back(e);
    char buf[128];
    for (int e : engs)
    {
        snprintf(buf, sizeof buf, "sdma_d2h_engine%d", e);
        line(buf, time_us(reps, [&] { copy(true, e, sa); wait(sa); }), n);
        snprintf(buf, sizeof buf, "sdma_h2d_engine%d", e);
        line(buf, time_us(reps, [&] { copy(false, e, sb); wait(sb); }), n);
    }
    for (int a : engs)
        for (int b : engs)
        {
            if (a > 4 || b > 4) continue;  // engines 4+ are far slower for host copies (see singles)
            snprintf(buf, sizeof buf, "sdma_both_d2h%d_h2d%d", a, b);
            line(buf, time_us(reps, [&] { copy(true, a, sa); copy(false, b, sb); wait(sa); wait(sb); }), 2 * n);
        }
    hsa_signal_destroy(sa);
    hsa_signal_destroy(sb);
    CK(hipFree(d_a));
    CK(hipFree(d_b));
    CK(hipHostFree(h_a));
    CK(hipHostFree(h_b));
    CK(hipHostFree(h_c));
    return 0;
}
