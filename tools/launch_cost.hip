// launch_cost.hip — developer micro-benchmark (not product): the HOST time of one kernel launch
// by kernel-argument size, with the device kept busy (so the launch never waits for it), and
// the synchronous round trip (launch + hipStreamSynchronize) of an empty kernel.
//   args_16      an empty kernel with a 16-B argument struct
//   args_1600    an empty kernel with a 1,600-B argument struct (libghx's kargs: 3 x 64 slots)
//   args_1600_tl the same launched through hipExtLaunchKernelGGL (no events)
// One JSON line. Build: make -C tools bin/launch_cost
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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

template<int B>
struct args_t
{
    unsigned long long w[B / 8];
};

template<int B>
__global__ void k_empty(args_t<B> a)
{
    if (a.w[0] == 0x1234567ull && threadIdx.x == 1000) a.w[1] = 0;  // never true
}

__global__ void k_busy(float* p, int n, int reps)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float v = p[i];
    for (int r = 0; r < reps; ++r) v = v * 1.0000001f + 1e-7f;
    p[i] = v;
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* p;
    const int n = 1 << 20;
    CK(hipMalloc(&p, n * sizeof(float)));
    CK(hipMemset(p, 0, n * sizeof(float)));
    args_t<16> a16{};
    args_t<1600> a1600{};
    auto host_cost = [&](auto launch) {
        std::vector<double> t;
        for (int rep = 0; rep < 7; ++rep)
        {
            hipLaunchKernelGGL(k_busy, dim3(n / 256), dim3(256), 0, s, p, n, 200000);  // ~ms busy
            const double t0 = now_us();
            for (int i = 0; i < 200; ++i) launch();
            t.push_back((now_us() - t0) / 200);
            CK(hipStreamSynchronize(s));
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    auto roundtrip = [&](auto launch) {
        std::vector<double> t;
        for (int rep = 0; rep < 7; ++rep)
        {
            CK(hipStreamSynchronize(s));
            const double t0 = now_us();
            for (int i = 0; i < 500; ++i)
            {
                launch();
                CK(hipStreamSynchronize(s));
            }
            t.push_back((now_us() - t0) / 500);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    auto l16 = [&] { hipLaunchKernelGGL(k_empty<16>, dim3(1), dim3(64), 0, s, a16); };
    auto l1600 = [&] { hipLaunchKernelGGL(k_empty<1600>, dim3(1), dim3(64), 0, s, a1600); };
    auto l1600x = [&] { hipExtLaunchKernelGGL(k_empty<1600>, dim3(1), dim3(64), 0, s, nullptr, nullptr, 0, a1600); };
    for (int i = 0; i < 100; ++i)
    {
        l16();
        l1600();
    }
    CK(hipStreamSynchronize(s));
    printf("{\"host_launch_us\": {\"args_16\": %.2f, \"args_1600\": %.2f, \"args_1600_ext\": %.2f}, "
           "\"sync_roundtrip_us\": {\"args_16\": %.2f, \"args_1600\": %.2f}}\n",
           host_cost(l16), host_cost(l1600), host_cost(l1600x), roundtrip(l16), roundtrip(l1600));
    CK(hipDeviceSynchronize());
    return 0;
}
