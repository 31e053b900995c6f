// TEST INFRASTRUCTURE ONLY — never linked into, loaded by or shipped with the product.
//
// Driver that runs the REFERENCE's own structured halo generator
// (/root/reference/include/ghex/structured/regular/halo_generator.hpp:93-160)
// on configurations read from stdin and prints the generated receive boxes and
// their intersections with a list of domains. This is the one piece of the
// reference's hot-path setup that compiles from its own headers with g++ alone
// (it needs only ghex/structured/grid.hpp, ghex/util/coordinate.hpp,
// ghex/util/math.hpp and ghex/structured/regular/domain_descriptor.hpp, all
// std-only). Everything else on the path needs gridtools/oomph/config.hpp,
// which are absent, so the rest of the reference is unbuildable here (see
// DESIGN.md "Oracle").
//
// Built by oracle/Makefile into oracle/_ref/ref_halo_boxes (git-ignored); output is used by
// tests/golden/make_ref_halo_boxes.py to pin oracle/ghex_oracle.c's restatement.
//
// stdin, one config per line (all ints):
//   D  gfirst[D] glast[D]  halos[2D]  periodic[D]  dom_first[D] dom_last[D]
//   K  (other_first[D] other_last[D]) x K
// stdout, per config:
//   "CONFIG <index> <nboxes>"
//   per box:  "BOX lf[D] ll[D] gf[D] gl[D]"
//   per (box, other domain) with a non-empty intersection (pattern.hpp:302-324 order):
//             "ISECT <box> <other> lf[D] ll[D] gf[D] gl[D]"
#include <ghex/structured/regular/halo_generator.hpp>

#include <iostream>
#include <vector>
#include <array>

template<int D>
static void run_one(int idx, std::istream& in)
{
    using dom_t = ghex::structured::regular::domain_descriptor<int, std::integral_constant<int, D>>;
    using hg_t = ghex::structured::regular::halo_generator<int, std::integral_constant<int, D>>;
    using coord_t = typename hg_t::coordinate_type;
    std::array<int, D> gf, gl, df, dl;
    std::array<int, 2 * D> halos;
    std::array<bool, D> periodic;
    for (auto& v : gf) in >> v;
    for (auto& v : gl) in >> v;
    for (auto& v : halos) in >> v;
    for (int d = 0; d < D; ++d) { int p; in >> p; periodic[d] = p != 0; }
    for (auto& v : df) in >> v;
    for (auto& v : dl) in >> v;
    int K;
    in >> K;
    std::vector<std::array<int, D>> of(K), ol(K);
    for (int k = 0; k < K; ++k)
    {
        for (auto& v : of[k]) in >> v;
        for (auto& v : ol[k]) in >> v;
    }
    hg_t hg(gf, gl, halos, periodic);
    dom_t dom(0, df, dl);
    auto boxes = hg(dom);
    std::cout << "CONFIG " << idx << " " << boxes.size() << "\n";
    auto pr = [](const coord_t& c) { for (int d = 0; d < D; ++d) std::cout << " " << c[d]; };
    for (auto& b : boxes)
    {
        std::cout << "BOX";
        pr(b.local().first()); pr(b.local().last()); pr(b.global().first()); pr(b.global().last());
        std::cout << "\n";
    }
    for (std::size_t b = 0; b < boxes.size(); ++b)
        for (int k = 0; k < K; ++k)
        {
            coord_t kf(of[k]), kl(ol[k]);
            auto x = hg.intersect(dom, boxes[b].local().first(), boxes[b].local().last(),
                boxes[b].global().first(), boxes[b].global().last(), kf, kl);
            if (x.global().first() <= x.global().last())
            {
                std::cout << "ISECT " << b << " " << k;
                pr(x.local().first()); pr(x.local().last()); pr(x.global().first()); pr(x.global().last());
                std::cout << "\n";
            }
        }
}

int main()
{
    int D, idx = 0;
    while (std::cin >> D)
    {
        switch (D)
        {
            case 1: run_one<1>(idx, std::cin); break;
            case 2: run_one<2>(idx, std::cin); break;
            case 3: run_one<3>(idx, std::cin); break;
            default: std::cerr << "bad D\n"; return 1;
        }
        ++idx;
    }
    return 0;
}
