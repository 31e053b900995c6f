"""Staged patterns (make_staged_pattern, include/ghex/structured/regular/make_pattern.hpp:47-250):
libghx (through the C ABI, one emulated rank at a time) against the oracle's restatement, key by
key, tag by tag, space by space; and the property the reference's staged test relies on
(test/structured/regular/test_simple_regular_domain.cpp:215-236): running the stages in order on
the oracle fills every halo cell, corners included, exactly as the full 26/8-neighbour pattern
does on a periodic grid.
"""
import itertools

import numpy as np
import pytest

from oracle import oracle as orc


def _grid(G, parts, n_ranks):
    """Domains of a regular Cartesian split (dim 0 fastest in the numbering), dealt round-robin
    to ranks; lookup(id, offset) = the periodic neighbour's id (the reference test's d_lu)."""
    D = len(G)
    cuts = []
    for d in range(D):
        b, e = divmod(G[d], parts[d])
        f, lst = 0, []
        for p in range(parts[d]):
            n = b + (1 if p >= parts[d] - e else 0)
            lst.append((f, f + n - 1))
            f += n
        cuts.append(lst)
    coords = [tuple(reversed(c)) for c in itertools.product(*(range(p) for p in reversed(parts)))]
    ident = {c: i for i, c in enumerate(coords)}
    ranks = [[] for _ in range(n_ranks)]
    for i, c in enumerate(coords):
        dom = orc.RegularDomain(10 + 3 * i, tuple(cuts[d][c[d]][0] for d in range(D)),
                                tuple(cuts[d][c[d]][1] for d in range(D)))
        ranks[i % n_ranks].append(dom)

    def lookup(did, off):
        c = coords[(did - 10) // 3]
        return 10 + 3 * ident[tuple((c[d] + off[d]) % parts[d] for d in range(D))]
    return ranks, lookup


def _abi_stages(ranks, lookup, gf, gl, halos, periodic, my_rank):
    from ghex_amd.structured.regular import DomainDescriptor, make_staged_pattern

    class FakeCtx:
        def rank(self):
            return my_rank

        def size(self):
            return len(ranks)

        def all_gather_object(self, obj):
            D = len(gf)
            out = []
            for doms in ranks:
                lst = []
                for d in doms:
                    nb = []
                    for i in range(D):
                        for side, h in ((-1, halos[2 * i]), (1, halos[2 * i + 1])):
                            off = tuple(side if c == i else 0 for c in range(D))
                            nb.append(lookup(d.id, off) if h > 0 else -1)
                    lst.append((d.id, d.first, d.last, nb))
                out.append(lst)
            assert obj == out[my_rank], "the product's own look-up table differs"
            return out

    dds = [DomainDescriptor(d.id, d.first, d.last) for d in ranks[my_rank]]
    return make_staged_pattern(FakeCtx(), dds, lookup, gf, gl, halos, periodic)


CASES = [
    ((12,), (3,), 2, (1, 2), (True,)),
    ((12, 10), (2, 2), 4, (3, 3, 3, 3), (True, True)),        # the reference test's shape
    ((12, 10), (3, 2), 2, (2, 1, 0, 3), (True, False)),
    ((9, 8, 7), (2, 2, 2), 8, (1, 1, 1, 1, 1, 1), (True, True, True)),
    ((9, 8, 7), (3, 1, 2), 3, (2, 1, 1, 2, 0, 3), (True, False, True)),
    ((6, 6, 6), (1, 1, 1), 1, (2, 2, 2, 2, 2, 2), (True, True, True)),  # self messages
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_staged_pattern_matches_oracle(case):
    G, parts, n_ranks, halos, periodic = CASES[case]
    D = len(G)
    gf, gl = (0,) * D, tuple(g - 1 for g in G)
    ranks, lookup = _grid(G, parts, n_ranks)
    ostages = orc.staged_make_pattern(ranks, lookup, gf, gl, halos, periodic)
    for r in range(n_ranks):
        pcs = _abi_stages(ranks, lookup, gf, gl, halos, periodic, r)
        assert len(pcs) == D
        for i, pc in enumerate(pcs):
            ops = ostages[i][r]
            assert len(pc) == len(ops)
            for li, op in enumerate(ops):
                for direction, omap in ((0, op.send_items()), (1, op.recv_items())):
                    got = pc.halos(li, direction)
                    assert [(g[0], g[2], g[1]) for g in got] == \
                        [(oid, otag, orank) for (oid, otag), (orank, _) in omap]
                    for g, (_, (_, lst)) in zip(got, omap):
                        assert g[3] == [(s.lf, s.ll, s.gf, s.gl) for s in lst]
                assert pc.max_tag() == op.max_tag


def staged_fields(ranks, G, halos, dtype=np.float64):
    """Per rank, per domain: owned cell = global linear index + 1, halo = -1, layout with dim 0
    fastest (layout_map<D-1, ..., 0>)."""
    D = len(G)
    out = []
    for doms in ranks:
        lst = []
        for d in doms:
            n = [d.last[c] - d.first[c] + 1 for c in range(D)]
            E = [n[c] + halos[2 * c] + halos[2 * c + 1] for c in range(D)]
            a = np.full(E, -1.0)
            idx = np.meshgrid(*[np.arange(n[c]) + d.first[c] for c in range(D)], indexing="ij")
            lin = sum(idx[c] * int(np.prod(G[:c])) for c in range(D))
            a[tuple(slice(halos[2 * c], halos[2 * c] + n[c]) for c in range(D))] = lin + 1
            mem = np.ascontiguousarray(a.transpose(tuple(reversed(range(D))))).astype(dtype)
            lst.append(orc.FieldSpec(mem, mem.itemsize, tuple(D - 1 - c for c in range(D)),
                                     tuple(halos[2 * c] for c in range(D)), tuple(E)))
        out.append(lst)
    return out


@pytest.mark.parametrize("case", [1, 3, 5])
def test_staged_exchange_fills_corners_like_full_pattern(case):
    G, parts, n_ranks, halos, periodic = CASES[case]
    D = len(G)
    gf, gl = (0,) * D, tuple(g - 1 for g in G)
    ranks, lookup = _grid(G, parts, n_ranks)
    staged = staged_fields(ranks, G, halos)
    full = staged_fields(ranks, G, halos)
    for pats in orc.staged_make_pattern(ranks, lookup, gf, gl, halos, periodic):
        orc.regular_exchange([[(staged[r][k], d.id, k, 0) for k, d in enumerate(doms)]
                              for r, doms in enumerate(ranks)], {0: pats}, n_ranks)
    opat = orc.regular_make_pattern(ranks, gf, gl, halos, periodic)
    orc.regular_exchange([[(full[r][k], d.id, k, 0) for k, d in enumerate(doms)]
                          for r, doms in enumerate(ranks)], {0: opat}, n_ranks)
    for r in range(n_ranks):
        for a, b in zip(staged[r], full[r]):
            assert (b.data != -1).all()  # fully periodic: every halo cell received
            np.testing.assert_array_equal(a.data, b.data)


def test_reference_binding_index_set_signatures():
    """The reference binding builds descriptors from index sets
    (bindings/python/src/ghex/structured/regular.py:31-38, 111-135, and its test
    test/bindings/python/test_structured_domain_descriptor.py): DomainDescriptor(id, set) and
    HaloGenerator(glob_set, halos, periodicity) give the same boxes as the coordinate forms."""
    from ghex_amd.structured.regular import (DomainDescriptor, HaloGenerator, ProductSet,
                                             UnitRange)
    sub = ProductSet(UnitRange(3, 9), UnitRange(0, 5), UnitRange(2, 4))
    assert sub.ndim == 3 and sub.shape == (6, 5, 2)
    assert sub[(0, 0, 0)] == (3, 0, 2) and sub[(-1, -1, -1)] == (8, 4, 3)
    prod = UnitRange(3, 9) * UnitRange(0, 5) * UnitRange(2, 4)
    assert prod.shape == sub.shape and prod[(-1, -1, -1)] == sub[(-1, -1, -1)]
    dd = DomainDescriptor(7, sub)
    assert dd.domain_id() == 7 and dd.first() == (3, 0, 2) and dd.last() == (8, 4, 3)
    glob = ProductSet.from_coords((0, 0, 0), (11, 9, 7))
    assert glob[(-1, -1, -1)] == (11, 9, 7)
    a = HaloGenerator(glob, ((1, 0), 2, (0, 3)), (True, False, True))
    b = HaloGenerator((0, 0, 0), (11, 9, 7), (1, 0, 2, 2, 0, 3), (True, False, True))
    assert a.halos == b.halos and a.periodic == b.periodic
    assert a(dd) == b(DomainDescriptor(7, (3, 0, 2), (8, 4, 3))) and len(a(dd)) > 0
    boxes = a(dd)
    # .global_ / .local: the boxes' union as one index set (the reference's HaloContainer)
    from ghex_amd.structured.cartesian_sets import union
    assert boxes.global_ == union(*(ProductSet.from_coords(gf, gl) for (_, _, gf, gl) in boxes))
    assert boxes.local.size == boxes.global_.size == sum(
        ProductSet.from_coords(lf, ll).size for (lf, ll, _, _) in boxes)
    with pytest.raises(IndexError):
        UnitRange(0, 2)[2]
    with pytest.raises(ValueError):
        UnitRange(3, 2)


def test_architecture_argument_like_the_reference_binding():
    """make_field_descriptor(..., arch=Architecture.X) as in bindings/python/src/ghex/
    structured/regular.py:66-98: GPU accepted, CPU refused (device path, no CPU fallback)."""
    import torch
    from ghex_amd.structured.regular import DomainDescriptor, make_field_descriptor
    from ghex_amd.util import Architecture
    dd = DomainDescriptor(0, (0, 0, 0), (3, 3, 3))
    f = torch.zeros(6, 6, 6)
    with pytest.raises(ValueError):
        make_field_descriptor(dd, f, (1, 1, 1), (6, 6, 6), arch=Architecture.CPU)
    with pytest.raises(TypeError):  # GPU requested, but the tensor is in host memory
        make_field_descriptor(dd, f, (1, 1, 1), (6, 6, 6), arch=Architecture.GPU)
