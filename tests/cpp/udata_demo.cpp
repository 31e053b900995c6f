// udata_demo.cpp — exercises include/ghex_amd/data_descriptor.hpp the way a GHEX
// communication_object drives an unstructured data descriptor: pack(T*, index container,
// &stream) of one neighbour's index list, then unpack(...) of a received buffer.
// Usage: udata_demo n_cells levels levels_first lid_bytes(4|8) lids_file out_prefix
//   lids_file: int64 local indices; values[i, l] = i*100 + l before the pack;
//   writes <out>.buf (packed buffer), <out>.values (after unpacking buffer[k] = 1e6 + k) and
//   <out>.buf2 (the list reversed in place, packed again from those values), <out>.buf3 (then
//   entries 1 and 2 swapped in place, packed again) and <out>.plans (plans kept after 5 more
//   lists through a cache bounded at 2).
#include <hip/hip_runtime.h>

#include <ghex_amd/data_descriptor.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

template<typename I>
struct iteration_space  // the shape of ghex's unstructured::pattern::iteration_space
{
    std::vector<I> m_lids;
    const std::vector<I>& local_indices() const { return m_lids; }
};

#define HCK(x)                                                                               \
    do                                                                                       \
    {                                                                                        \
        if ((x) != hipSuccess)                                                               \
        {                                                                                    \
            std::fprintf(stderr, "HIP error at %d\n", __LINE__);                             \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)

template<typename I>
int run(size_t n, int levels, bool lf, const std::vector<int64_t>& lids, const char* out)
{
    std::vector<iteration_space<I>> c(1);
    for (auto v : lids) c[0].m_lids.push_back(I(v));
    const size_t idx_stride = lf ? size_t(levels) : 1, lvl_stride = lf ? 1 : n;
    std::vector<double> host(n * size_t(levels));
    for (size_t i = 0; i < n; ++i)
        for (int l = 0; l < levels; ++l) host[i * idx_stride + size_t(l) * lvl_stride] = double(i) * 100 + l;
    double *values, *buf;
    const size_t nb = lids.size() * size_t(levels);
    HCK(hipMalloc(&values, host.size() * 8));
    HCK(hipMalloc(&buf, nb * 8 + 8));
    HCK(hipMemcpy(values, host.data(), host.size() * 8, hipMemcpyHostToDevice));
    hipStream_t s;
    HCK(hipStreamCreate(&s));
    ghex_amd::unstructured::data_descriptor<int, double> d(0, n, values, levels, lf);
    d.pack(buf, c, &s);
    HCK(hipStreamSynchronize(s));
    std::vector<double> hb(nb);
    HCK(hipMemcpy(hb.data(), buf, nb * 8, hipMemcpyDeviceToHost));
    std::ofstream(std::string(out) + ".buf", std::ios::binary)
        .write(reinterpret_cast<const char*>(hb.data()), std::streamsize(nb * 8));
    for (size_t k = 0; k < nb; ++k) hb[k] = 1e6 + double(k);
    HCK(hipMemcpy(buf, hb.data(), nb * 8, hipMemcpyHostToDevice));
    d.unpack(buf, c, &s);
    d.pack(buf, c, &s);  // cached plan reused
    HCK(hipStreamSynchronize(s));
    HCK(hipMemcpy(host.data(), values, host.size() * 8, hipMemcpyDeviceToHost));
    std::ofstream(std::string(out) + ".values", std::ios::binary)
        .write(reinterpret_cast<const char*>(host.data()), std::streamsize(host.size() * 8));
    // a different list at the same address (same length): the adaptor's sampled check must
    // build a new plan, so this pack gathers in the reversed order
    std::reverse(c[0].m_lids.begin(), c[0].m_lids.end());
    d.pack(buf, c, &s);
    HCK(hipStreamSynchronize(s));
    HCK(hipMemcpy(hb.data(), buf, nb * 8, hipMemcpyDeviceToHost));
    std::ofstream(std::string(out) + ".buf2", std::ios::binary)
        .write(reinterpret_cast<const char*>(hb.data()), std::streamsize(nb * 8));
    // entries 1 and 2 swapped in place: positions no sample covers (the sampled
    // check missed such a change); the exact check must build a new plan
    if (c[0].m_lids.size() > 2) std::swap(c[0].m_lids[1], c[0].m_lids[2]);
    d.pack(buf, c, &s);
    HCK(hipStreamSynchronize(s));
    HCK(hipMemcpy(hb.data(), buf, nb * 8, hipMemcpyDeviceToHost));
    std::ofstream(std::string(out) + ".buf3", std::ios::binary)
        .write(reinterpret_cast<const char*>(hb.data()), std::streamsize(nb * 8));
    // the cache stays bounded: 5 distinct lists through a cache of at most 2 plans
    d.set_max_plans(2);
    std::vector<iteration_space<I>> more(1);
    for (int k = 0; k < 5; ++k)
    {
        more[0].m_lids.assign(c[0].m_lids.begin(), c[0].m_lids.begin() + 1 + k);
        d.pack(buf, more, &s);
    }
    HCK(hipStreamSynchronize(s));
    std::ofstream(std::string(out) + ".plans") << d.num_plans() << "\n";
    HCK(hipFree(values));
    HCK(hipFree(buf));
    HCK(hipStreamDestroy(s));
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 7) return 1;
    const size_t n = size_t(std::atoll(argv[1]));
    const int levels = std::atoi(argv[2]);
    const bool lf = std::atoi(argv[3]) != 0;
    const int lb = std::atoi(argv[4]);
    std::ifstream in(argv[5], std::ios::binary | std::ios::ate);
    const auto bytes = size_t(in.tellg());
    in.seekg(0);
    std::vector<int64_t> lids(bytes / 8);
    in.read(reinterpret_cast<char*>(lids.data()), std::streamsize(bytes));
    try
    {
        return lb == 4 ? run<int32_t>(n, levels, lf, lids, argv[6])
                       : run<int64_t>(n, levels, lf, lids, argv[6]);
    }
    catch (const std::exception& e)
    {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
}
