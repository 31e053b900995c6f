// config5_gen.cpp — the synthetic inputs of BASELINE config 5: one rank's
// unstructured domain. Bench / test input generation, not product code (tools/lib/libconfig5.so,
// loaded by bench.py and tests through ctypes).
//
// Definition (fixed here; the survey names the ingredients, this is the one procedure both the
// bench and the tests use, so every rank's domain is a pure function of (rank, world, cells,
// halo, seed)):
//   g = std::mt19937_64(seed + rank)                      seed 20260715
//   halo gids: repeat { owner = others[g() % (world-1)]   others = the ranks != rank, ascending
//                       cell  = g() % cells
//                       gid   = owner * 10^7 + cell }     until `halo` distinct gids (draw order)
//   storage  : [rank * 10^7 + i for i < cells] ++ halo gids, then Fisher-Yates with
//              j = g() % (i + 1) for i = n-1 .. 1
//   outer lids: the storage positions of the halo gids, ascending.
// Cell values (the reference's encoding, test/unstructured/unstructured_test_case.hpp:345-359):
// value(gid, level) = gid * 100 + level.
#include <cstdint>
#include <random>
#include <unordered_set>
#include <vector>

extern "C" int config5_generate(int32_t rank, int32_t world, int64_t cells, int64_t halo,
                                uint64_t seed, int64_t* gids, int64_t* outer_lids)
{
    if (world < 2 || rank < 0 || rank >= world || cells < 1 || halo < 0 ||
        halo > cells * int64_t(world - 1) / 2 || cells > 10000000)
        return -1;
    std::mt19937_64 g(seed + uint64_t(rank));
    std::vector<int64_t> others;
    for (int32_t r = 0; r < world; ++r)
        if (r != rank) others.push_back(r);
    const int64_t n = cells + halo;
    std::vector<uint8_t> is_halo(size_t(n), 0);
    for (int64_t i = 0; i < cells; ++i) gids[i] = int64_t(rank) * 10000000 + i;
    std::unordered_set<int64_t> seen;
    seen.reserve(size_t(halo) * 2);
    int64_t k = cells;
    while (k < n)
    {
        const int64_t owner = others[size_t(g() % uint64_t(others.size()))];
        const int64_t cell = int64_t(g() % uint64_t(cells));
        const int64_t gid = owner * 10000000 + cell;
        if (seen.insert(gid).second)
        {
            gids[k] = gid;
            is_halo[size_t(k)] = 1;
            ++k;
        }
    }
    for (int64_t i = n - 1; i >= 1; --i)
    {
        const int64_t j = int64_t(g() % uint64_t(i + 1));
        std::swap(gids[i], gids[j]);
        std::swap(is_halo[size_t(i)], is_halo[size_t(j)]);
    }
    int64_t o = 0;
    for (int64_t i = 0; i < n; ++i)
        if (is_halo[size_t(i)]) outer_lids[o++] = i;
    return 0;
}
