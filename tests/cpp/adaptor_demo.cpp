// adaptor_demo.cpp — exercises include/ghex_amd/field_descriptor.hpp the way a GHEX
// communication_object would: a field-descriptor object, an index container of
// iteration_space_pair-shaped objects, pack(T*, container, &stream) / unpack(...).
// Self exchange of one periodic N^3 domain (fp64, halo H). Writes the packed buffer and the
// field after unpack to <out>.buf / <out>.field for tests/test_gpu_cpp.py to compare with the
// oracle.  Usage: adaptor_demo N H out_prefix
#include <hip/hip_runtime.h>

#include <ghex_amd/field_descriptor.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

// the shape of ghex::pattern<structured grid>::iteration_space_pair (pattern.hpp:95-120)
struct iteration_space
{
    std::array<int, 3> f, l;
    const std::array<int, 3>& first() const { return f; }
    const std::array<int, 3>& last() const { return l; }
};
struct iteration_space_pair
{
    iteration_space m_local, m_global;
    const iteration_space& local() const { return m_local; }
    const iteration_space& global() const { return m_global; }
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

int main(int argc, char** argv)
{
    if (argc < 4) return 1;
    const int N = std::atoi(argv[1]), H = std::atoi(argv[2]);
    const int E = N + 2 * H;
    const size_t n = size_t(E) * E * E;
    std::vector<double> host(n, -1.0);
    for (int z = 0; z < N; ++z)
        for (int y = 0; y < N; ++y)
            for (int x = 0; x < N; ++x)
                host[(size_t(z + H) * E + (y + H)) * E + (x + H)] = x + N * (y + N * double(z));
    double* field;
    HCK(hipMalloc(&field, n * sizeof(double)));
    HCK(hipMemcpy(field, host.data(), n * sizeof(double), hipMemcpyHostToDevice));

    // receive boxes of the periodic domain; the self message's send boxes are the same list in
    // the sender's local coordinates (global - first, structured/pattern.hpp:369-412)
    int32_t gf[3] = {0, 0, 0}, gl[3] = {N - 1, N - 1, N - 1}, halos[6] = {H, H, H, H, H, H};
    int32_t per[3] = {1, 1, 1}, df[3] = {0, 0, 0}, dl[3] = {N - 1, N - 1, N - 1};
    int32_t nb = 0;
    ghex_amd::check(ghx_regular_halo_boxes(3, gf, gl, halos, per, df, dl, nullptr, nullptr, 0, &nb),
                    "halo boxes");
    std::vector<ghx_box> loc(nb), glo(nb);
    ghex_amd::check(ghx_regular_halo_boxes(3, gf, gl, halos, per, df, dl, loc.data(), glo.data(), nb,
                                           &nb),
                    "halo boxes");
    std::vector<iteration_space_pair> send, recv;
    size_t elems = 0;
    for (int i = 0; i < nb; ++i)
    {
        iteration_space_pair r{}, s{};
        for (int d = 0; d < 3; ++d)
        {
            r.m_local.f[d] = loc[i].first[d];
            r.m_local.l[d] = loc[i].last[d];
            s.m_local.f[d] = glo[i].first[d];
            s.m_local.l[d] = glo[i].last[d];
        }
        size_t sz = 1;
        for (int d = 0; d < 3; ++d) sz *= size_t(r.m_local.l[d] - r.m_local.f[d] + 1);
        elems += sz;
        send.push_back(s);
        recv.push_back(r);
    }
    ghex_amd::structured::field_descriptor<double, 3> fd(0, field, {H, H, H}, {E, E, E}, {2, 1, 0});
    double* buf;
    HCK(hipMalloc(&buf, elems * sizeof(double)));
    hipStream_t stream;
    HCK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    void* arg = &stream;  // the reference passes a pointer to the stream (pack_kernels.hpp:219)
    fd.pack(buf, send, arg);
    fd.unpack(buf, recv, arg);
    HCK(hipStreamSynchronize(stream));
    std::vector<double> hbuf(elems);
    HCK(hipMemcpy(hbuf.data(), buf, elems * sizeof(double), hipMemcpyDeviceToHost));
    HCK(hipMemcpy(host.data(), field, n * sizeof(double), hipMemcpyDeviceToHost));
    std::string pre = argv[3];
    FILE* f = std::fopen((pre + ".buf").c_str(), "wb");
    std::fwrite(hbuf.data(), sizeof(double), elems, f);
    std::fclose(f);
    f = std::fopen((pre + ".field").c_str(), "wb");
    std::fwrite(host.data(), sizeof(double), n, f);
    std::fclose(f);
    std::printf("adaptor_demo: %d spaces, %zu elements\n", nb, elems);
    return 0;
}
