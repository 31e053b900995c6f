// udata_cost.hip — developer measurement (not product): the host cost of one drop-in
// unstructured pack call, ghex_amd::unstructured::data_descriptor::pack(buffer, container,
// &stream), at BASELINE config 5's list size (one neighbour list of `n_lids` random lids into a
// 10.5M-cell fp64 field, levels 1), against the device time of the gather it enqueues.
//
//   adaptor   data_descriptor::pack (plan found by the list's address, the list compared with
//             the plan's copy in full: the default since round 6)
//   adaptor_sampled   the same with assume_immutable_index_lists(true) (16 sampled entries:
//             O(1) host work; round 5's default)
//   c_entry   ghx_unstructured_pack (the plain C entry point: compares the whole list with the
//             cached copy on every call — what the adaptor called before round 5)
//   launch    ghx_uplan_execute of a prepared plan (the launch alone: the floor of any call)
// host_us is measured while the device is kept busy by a spin kernel queued first, so it is the
// host's own time per call; device_us is the gather's time from events around 100 calls.
// Output: one JSON line.
#include <hip/hip_runtime.h>

#include <ghex_amd/data_descriptor.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define HCK(x)                                                                               \
    do                                                                                       \
    {                                                                                        \
        if ((x) != hipSuccess)                                                               \
        {                                                                                    \
            std::fprintf(stderr, "HIP error at %d\n", __LINE__);                             \
            std::exit(2);                                                                    \
        }                                                                                    \
    } while (0)

__global__ void spin(long long cycles)
{
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

struct iteration_space
{
    std::vector<int32_t> m_lids;
    const std::vector<int32_t>& local_indices() const { return m_lids; }
};

template<typename F>
double host_us(hipStream_t s, F&& call, int reps)
{
    std::vector<double> t;
    for (int r = 0; r < 5; ++r)
    {
        spin<<<1, 1, 0, s>>>(400000000LL);  // ~0.2 s: the device stays busy
        const auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) call();
        const auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count() / reps);
        HCK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

template<typename F>
double device_us(hipStream_t s, F&& call, int reps)
{
    hipEvent_t e0, e1;
    HCK(hipEventCreate(&e0));
    HCK(hipEventCreate(&e1));
    std::vector<double> t;
    for (int r = 0; r < 5; ++r)
    {
        HCK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; ++i) call();
        HCK(hipEventRecord(e1, s));
        HCK(hipEventSynchronize(e1));
        float ms = 0;
        HCK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(double(ms) * 1e3 / reps);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv)
{
    const int64_t cells = 10500000;
    const int64_t n_lids = argc > 1 ? std::atoll(argv[1]) : 500000;
    std::mt19937_64 g(20260715);
    std::vector<iteration_space> c(1);
    std::vector<int32_t> perm(static_cast<size_t>(cells));
    std::iota(perm.begin(), perm.end(), 0);
    std::shuffle(perm.begin(), perm.end(), g);
    c[0].m_lids.assign(perm.begin(), perm.begin() + n_lids);
    double *values, *buf;
    HCK(hipMalloc(&values, size_t(cells) * 8));
    HCK(hipMalloc(&buf, size_t(n_lids) * 8));
    HCK(hipMemset(values, 0, size_t(cells) * 8));
    hipStream_t s;
    HCK(hipStreamCreate(&s));
    ghex_amd::unstructured::data_descriptor<int, double> d(0, size_t(cells), values, 1, true);
    const auto& l = c[0].local_indices();
    auto adaptor = [&] { d.pack(buf, c, &s); };
    ghex_amd::unstructured::data_descriptor<int, double> d2(0, size_t(cells), values, 1, true);
    d2.assume_immutable_index_lists(true);
    auto sampled = [&] { d2.pack(buf, c, &s); };
    auto c_entry = [&] {
        ghex_amd::unstructured::check_u(
            ghx_unstructured_pack(&d.desc(), values, buf, l.data(), 4, int64_t(l.size()), s),
            "ghx_unstructured_pack");
    };
    std::vector<int64_t> wide(l.begin(), l.end());
    ghx_upack_entry e{};
    e.data = d.desc();
    e.lids = wide.data();
    e.n_lids = int64_t(wide.size());
    ghx_uplan* p = nullptr;
    ghex_amd::unstructured::check_u(ghx_uplan_create(&e, 1, 0, &p), "ghx_uplan_create");
    void* fp[1] = {values};
    void* bp[1] = {buf};
    auto launch = [&] { ghex_amd::unstructured::check_u(ghx_uplan_execute(p, fp, 1, bp, 1, s), "x"); };
    for (int i = 0; i < 20; ++i)
    {
        adaptor();
        sampled();
        c_entry();
        launch();
    }
    HCK(hipStreamSynchronize(s));
    const int reps = 200;
    const double h_ad = host_us(s, adaptor, reps), h_c = host_us(s, c_entry, reps),
                 h_l = host_us(s, launch, reps), h_sm = host_us(s, sampled, reps);
    const double d_ad = device_us(s, adaptor, 100), d_c = device_us(s, c_entry, 100),
                 d_l = device_us(s, launch, 100), d_sm = device_us(s, sampled, 100);
    std::printf("{\"n_lids\": %lld, \"cells\": %lld, \"levels\": 1, "
                "\"adaptor\": {\"host_us\": %.3f, \"device_us\": %.3f}, "
                "\"adaptor_sampled\": {\"host_us\": %.3f, \"device_us\": %.3f}, "
                "\"c_entry\": {\"host_us\": %.3f, \"device_us\": %.3f}, "
                "\"launch\": {\"host_us\": %.3f, \"device_us\": %.3f}, "
                "\"adaptor_overhead_us\": %.3f, \"adaptor_overhead_frac_of_device\": %.4f, "
                "\"c_entry_overhead_us\": %.3f, \"c_entry_overhead_frac_of_device\": %.4f}\n",
                (long long)n_lids, (long long)cells, h_ad, d_ad, h_sm, d_sm, h_c, d_c, h_l, d_l, h_ad - h_l,
                (h_ad - h_l) / d_l, h_c - h_l, (h_c - h_l) / d_l);
    ghx_uplan_destroy(p);
    HCK(hipFree(values));
    HCK(hipFree(buf));
    HCK(hipStreamDestroy(s));
    return 0;
}
