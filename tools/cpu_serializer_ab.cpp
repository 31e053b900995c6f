// CPU baseline calibration: the oracle's runtime-D row serializer
// (oracle/ghex_oracle.c batch_is, what bench.py's cpu_baseline times) against a compile-time
// restatement shaped like the reference's serialization<cpu>::pack_batch / unpack_batch
// (include/ghex/structured/pack_kernels.hpp:62-158): D and the layout map fixed at compile time,
// the loop nest generated like ghex::for_loop (include/ghex/util/for_each.hpp:85-149, slowest
// layout dim outermost, the contiguous dim one memcpy per row), the element type a template
// parameter. Same workload as SURVEY §6: 512^3 fp64, halo 2, one periodic domain, 26 neighbours,
// layout_map<2,1,0>; pack and unpack timed separately, min over reps, interleaved A/B so both
// see the same machine state. No reference source is compiled or included.
//
// Build: g++ -O3 -march=x86-64-v2 -std=c++17 tools/cpu_serializer_ab.cpp -o tools/bin/cpu_ab -ldl
// Run:   tools/bin/cpu_ab [N] [H] [reps]   (prints one JSON line)
#include <dlfcn.h>

#include <array>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace
{
using box = std::array<int32_t, 6>;  // first x,y,z, last x,y,z (local, halo-relative)

// 26 halo boxes of one periodic domain [0,N)^3, send side (inner cells next to each face /
// edge / corner) and recv side (the halo cells), in any fixed order (both serializers use it).
void boxes(int N, int H, std::vector<box>& send, std::vector<box>& recv)
{
    for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx)
            {
                if (!dx && !dy && !dz) continue;
                const int d[3] = {dx, dy, dz};
                box s, r;
                for (int k = 0; k < 3; ++k)
                {
                    // the receiver at -d gets my cells on side d; my halo on side d comes from
                    // the neighbour at d (its cells on side -d)
                    if (d[k] < 0) { s[k] = 0; s[k + 3] = H - 1; r[k] = -H; r[k + 3] = -1; }
                    else if (d[k] > 0) { s[k] = N - H; s[k + 3] = N - 1; r[k] = N; r[k + 3] = N + H - 1; }
                    else { s[k] = 0; s[k + 3] = N - 1; r[k] = 0; r[k + 3] = N - 1; }
                }
                send.push_back(s);
                recv.push_back(r);
            }
}

// compile-time restatement: layout_map<2,1,0> (x contiguous), D = 3
template<typename T, bool PACK>
size_t batch_ct(T* field, int64_t E, int H, const box& b, T* buf)
{
    const int64_t nx = b[3] - b[0] + 1, ny = b[4] - b[1] + 1;
    const size_t row = size_t(nx) * sizeof(T);
    // for_loop order: z (layout value 0) outermost, y inner; buffer dense in the same order
    for (int32_t z = b[2]; z <= b[5]; ++z)
        for (int32_t y = b[1]; y <= b[4]; ++y)
        {
            T* f = field + ((int64_t(z) + H) * E + (y + H)) * E + (b[0] + H);
            T* q = buf + ((int64_t(z) - b[2]) * ny + (y - b[1])) * nx;
            if (PACK) std::memcpy(q, f, row);
            else std::memcpy(f, q, row);
        }
    return size_t(nx) * ny * (b[5] - b[2] + 1);
}

using orc_fn = int64_t (*)(void*, void*, int, int64_t, const int32_t*, const int64_t*,
                           const int32_t*, const int32_t*, int, int);

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

int main(int argc, char** argv)
{
    const int N = argc > 1 ? std::atoi(argv[1]) : 512, H = argc > 2 ? std::atoi(argv[2]) : 2;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    const int64_t E = N + 2 * H;
    void* lib = dlopen("oracle/build/libghex_oracle.so", RTLD_NOW);
    if (!lib) { std::fprintf(stderr, "%s\n", dlerror()); return 1; }
    auto opack = reinterpret_cast<orc_fn>(dlsym(lib, "orc_structured_pack"));
    auto ounpack = reinterpret_cast<orc_fn>(dlsym(lib, "orc_structured_unpack"));
    std::vector<box> send, recv;
    boxes(N, H, send, recv);
    std::vector<double> field(size_t(E) * E * E, 0.0);
    for (size_t i = 0; i < field.size(); ++i) field[i] = double(i);
    size_t n = 0;
    for (auto& b : send) n += size_t(b[3] - b[0] + 1) * (b[4] - b[1] + 1) * (b[5] - b[2] + 1);
    std::vector<double> buf(n), buf2(n);
    // the oracle's argument form: boxes as (first[3], last[3]) in the field's (x, y, z) dims
    const int32_t layout[3] = {2, 1, 0};
    const int64_t strides[3] = {8, 8 * E, 8 * E * E};
    const int32_t offs[3] = {H, H, H};
    std::vector<int32_t> sb, rb;
    for (auto& b : send) sb.insert(sb.end(), b.begin(), b.end());
    for (auto& b : recv) rb.insert(rb.end(), b.begin(), b.end());
    double best[4] = {1e9, 1e9, 1e9, 1e9};  // oracle pack, unpack, ct pack, unpack
    auto run_oracle = [&] {
        double t = now();
        opack(field.data(), buf.data(), 3, 8, layout, strides, offs, sb.data(), int(send.size()), 0);
        best[0] = std::min(best[0], now() - t);
        t = now();
        ounpack(field.data(), buf.data(), 3, 8, layout, strides, offs, rb.data(), int(recv.size()), 0);
        best[1] = std::min(best[1], now() - t);
    };
    auto run_ct = [&] {
        double t = now();
        size_t o = 0;
        for (auto& b : send) o += batch_ct<double, true>(field.data(), E, H, b, buf2.data() + o);
        best[2] = std::min(best[2], now() - t);
        t = now();
        o = 0;
        for (auto& b : recv) o += batch_ct<double, false>(field.data(), E, H, b, buf2.data() + o);
        best[3] = std::min(best[3], now() - t);
    };
    for (int r = 0; r < reps; ++r)  // alternate which form goes first
    {
        if (r % 2) { run_ct(); run_oracle(); }
        else { run_oracle(); run_ct(); }
    }
    const bool same = std::memcmp(buf.data(), buf2.data(), n * 8) == 0;
    const double bytes = 2.0 * n * 8;  // per direction: read + write
    std::printf("{\"N\": %d, \"H\": %d, \"reps\": %d, \"elems\": %zu, \"buffers_equal\": %s, "
                "\"oracle_pack_ms\": %.3f, \"oracle_unpack_ms\": %.3f, \"oracle_GBps\": %.3f, "
                "\"compile_time_pack_ms\": %.3f, \"compile_time_unpack_ms\": %.3f, "
                "\"compile_time_GBps\": %.3f}\n",
                N, H, reps, n, same ? "true" : "false", best[0] * 1e3, best[1] * 1e3,
                2 * bytes / (best[0] + best[1]) / 1e9, best[2] * 1e3, best[3] * 1e3,
                2 * bytes / (best[2] + best[3]) / 1e9);
    return same ? 0 : 2;
}
