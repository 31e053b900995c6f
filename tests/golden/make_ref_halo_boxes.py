"""Generate tests/golden/ref_halo_boxes.json by running the REFERENCE's own regular halo
generator (include/ghex/structured/regular/halo_generator.hpp, compiled from /root/reference by
oracle/Makefile into oracle/_ref/ref_halo_boxes).

Run in the build container only (needs /root/reference):  python tests/golden/make_ref_halo_boxes.py

The fixture holds, per configuration, the inputs and the reference's outputs: the generated
receive boxes (local + global, in generation order) and, for every box and every domain of the
decomposition, the non-empty intersections (halo_generator::intersect). tests/test_oracle.py pins
oracle/oracle.py's restatement against it; the GPU box never reads /root/reference.
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_halo_boxes")


def decompose(gsize, parts):
    """Cartesian split of [0, gsize) per dim into parts[d] near-equal pieces -> list of (first, last)."""
    D = len(gsize)
    cuts = []
    for d in range(D):
        n, p = gsize[d], parts[d]
        b = [n * i // p for i in range(p + 1)]
        cuts.append([(b[i], b[i + 1] - 1) for i in range(p)])
    doms = []
    # rank order: dim 0 fastest (r = x + px*(y + py*z)), as in SURVEY §8(e)
    for z in range(parts[2] if D > 2 else 1):
        for y in range(parts[1] if D > 1 else 1):
            for x in range(parts[0]):
                c = [x, y, z][:D]
                doms.append((tuple(cuts[d][c[d]][0] for d in range(D)),
                             tuple(cuts[d][c[d]][1] for d in range(D))))
    return doms


def configs():
    out = []
    # 3D cube, various halos / periodicity, decompositions 1, (2,1,1), (2,2,2)
    for gsize, parts in [((8, 8, 8), (1, 1, 1)), ((13, 13, 13), (1, 1, 1)),
                         ((16, 8, 8), (2, 1, 1)), ((16, 16, 16), (2, 2, 2)),
                         ((12, 10, 7), (3, 2, 1))]:
        doms = decompose(gsize, parts)
        for halos in [(1,) * 6, (2,) * 6, (3,) * 6, (0, 0, 1, 0, 1, 2), (2, 1, 1, 2, 1, 1),
                      (0, 1, 0, 0, 3, 0)]:
            for periodic in [(1, 1, 1), (0, 1, 1), (0, 0, 0)]:
                for di in range(min(len(doms), 3)):
                    out.append(dict(D=3, gfirst=[0, 0, 0], glast=[g - 1 for g in gsize],
                                    halos=list(halos), periodic=list(periodic),
                                    dom=list(map(list, doms[di])),
                                    others=[list(map(list, o)) for o in doms]))
    # the reference test geometry: test_regular_domain.cpp:105-121, 664-691 (4 ranks, 8 domains)
    local_ext, ranks = (4, 3, 2), 4
    glast = [local_ext[0] * 4 - 1, ((ranks - 1) // 2 + 1) * local_ext[1] - 1, local_ext[2] - 1]
    doms = []
    for r in range(ranks):
        for k in range(2):
            f = [((r % 2) * 2 + k) * local_ext[0], (r // 2) * local_ext[1], 0]
            l = [((r % 2) * 2 + k + 1) * local_ext[0] - 1, (r // 2 + 1) * local_ext[1] - 1,
                 local_ext[2] - 1]
            doms.append((f, l))
    for halos in [(0, 0, 1, 0, 1, 2), (2, 2, 2, 2, 2, 2)]:
        for di in range(len(doms)):
            out.append(dict(D=3, gfirst=[0, 0, 0], glast=glast, halos=list(halos),
                            periodic=[1, 1, 1], dom=list(map(list, doms[di])),
                            others=[list(map(list, o)) for o in doms]))
    # 2D: test_simple_regular_domain.cpp (DIM=8, HALO=3, periodic) and the python test sizes
    for gsize, parts, halos in [((16, 16), (2, 2), (3, 3, 3, 3)), ((48, 24), (2, 2), (2, 1, 1, 2)),
                                ((16, 8), (1, 1), (1, 2, 0, 1))]:
        doms = decompose(gsize + (1,), parts + (1,))
        doms = [(f[:2], l[:2]) for f, l in doms]
        for periodic in [(1, 1), (0, 1)]:
            for di in range(len(doms)):
                out.append(dict(D=2, gfirst=[0, 0], glast=[g - 1 for g in gsize],
                                halos=list(halos), periodic=list(periodic),
                                dom=list(map(list, doms[di])),
                                others=[list(map(list, o)) for o in doms]))
    # 1D
    for halos in [(2, 1), (0, 3)]:
        for periodic in [(1,), (0,)]:
            doms = [([0], [23]), ([24], [47])]
            for di in range(2):
                out.append(dict(D=1, gfirst=[0], glast=[47], halos=list(halos),
                                periodic=list(periodic), dom=list(map(list, doms[di])),
                                others=[list(map(list, o)) for o in doms]))
    # python-binding test, 3D sizes (48,24,16), halos ((2,1),(1,2),(1,1))
    doms = decompose((48, 24, 16), (2, 2, 2))
    for periodic in [(1, 1, 1), (0, 1, 1)]:
        for di in range(len(doms)):
            out.append(dict(D=3, gfirst=[0, 0, 0], glast=[47, 23, 15], halos=[2, 1, 1, 2, 1, 1],
                            periodic=list(periodic), dom=list(map(list, doms[di])),
                            others=[list(map(list, o)) for o in doms]))
    # halos wider than a domain and wider than the whole periodic extent (the wrap of a box that
    # starts more than one period before the domain: C++ truncating %, halo_generator.hpp:139-141)
    for gsize, parts, halos in [((8, 2, 2), (4, 1, 1), (3,) * 6), ((3, 3, 3), (3, 3, 3), (2,) * 6),
                                ((5, 2, 1), (5, 2, 1), (2,) * 6), ((8, 4, 4), (4, 2, 2), (3,) * 6),
                                ((4, 4, 4), (1, 1, 1), (5, 9, 1, 4, 6, 2))]:
        doms = decompose(gsize, parts)
        for periodic in [(1, 1, 1), (1, 0, 1)]:
            for di in range(min(len(doms), 4)):
                out.append(dict(D=3, gfirst=[0, 0, 0], glast=[g - 1 for g in gsize],
                                halos=list(halos), periodic=list(periodic),
                                dom=list(map(list, doms[di])),
                                others=[list(map(list, o)) for o in doms]))
    for halos in [(5, 2), (7, 7)]:
        out.append(dict(D=1, gfirst=[0], glast=[2], halos=list(halos), periodic=[1],
                        dom=[[0], [2]], others=[[[0], [2]]]))
    # the bench geometry at 512^3, H=1..3 (boxes only + the 2x2x2 split)
    for H in (1, 2, 3):
        out.append(dict(D=3, gfirst=[0, 0, 0], glast=[511, 511, 511], halos=[H] * 6,
                        periodic=[1, 1, 1], dom=[[0, 0, 0], [511, 511, 511]],
                        others=[[[0, 0, 0], [511, 511, 511]]]))
        doms = decompose((1024, 1024, 1024), (2, 2, 2))
        out.append(dict(D=3, gfirst=[0, 0, 0], glast=[1023] * 3, halos=[H] * 6,
                        periodic=[1, 1, 1], dom=list(map(list, doms[5])),
                        others=[list(map(list, o)) for o in doms]))
    return out


def main():
    if not os.path.exists(EXE):
        sys.exit(f"{EXE} missing: run make -C oracle ref")
    cfgs = configs()
    lines = []
    for c in cfgs:
        vals = [c["D"]] + c["gfirst"] + c["glast"] + c["halos"] + c["periodic"] + \
            c["dom"][0] + c["dom"][1] + [len(c["others"])]
        for f, l in c["others"]:
            vals += f + l
        lines.append(" ".join(map(str, vals)))
    res = subprocess.run([EXE], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.splitlines()
    cur = None
    for ln in res:
        t = ln.split()
        if t[0] == "CONFIG":
            cur = cfgs[int(t[1])]
            cur["boxes"], cur["isect"] = [], []
        elif t[0] == "BOX":
            cur["boxes"].append(list(map(int, t[1:])))
        elif t[0] == "ISECT":
            cur["isect"].append(list(map(int, t[1:])))
    with open(os.path.join(HERE, "ref_halo_boxes.json"), "w") as fh:
        json.dump({"source": "reference halo_generator.hpp:93-160 via oracle/ref_halo_boxes.cpp",
                   "configs": cfgs}, fh, separators=(",", ":"))
    print(f"wrote {len(cfgs)} configs")


if __name__ == "__main__":
    main()
