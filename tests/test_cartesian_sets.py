"""ghex_amd.structured.cartesian_sets — the index sets of the reference Python binding
(bindings/python/src/ghex/structured/cartesian_sets.py) — and the reference binding's own
domain / halo-generator tests (test/bindings/python/test_structured_domain_descriptor.py) run
for every rank of emulated Cartesian decompositions (no MPI: each rank's coordinate is looped
over; the halo generator is libghx's, a host call)."""
import itertools

import pytest

from ghex_amd.structured.cartesian_sets import (IndexSpace, ProductSet, UnionCartesian,
                                                UnionRange, UnitRange, union)


def compute_dims(n, ndim):
    """MPI_Dims_create for an all-zero request: the most balanced factorisation of n into ndim
    factors, non-increasing."""
    f, p, m = [], 2, n
    while m > 1:
        while m % p == 0:
            f.append(p)
            m //= p
        p += 1
    dims = [1] * ndim
    for q in sorted(f, reverse=True):
        dims[dims.index(min(dims))] *= q
    return tuple(sorted(dims, reverse=True))


def cart_coords(rank, dims):
    """MPI_Cart_coords (row-major: the last dimension varies fastest)."""
    c = []
    for d in reversed(dims):
        c.append(rank % d)
        rank //= d
    return tuple(reversed(c))


def test_compute_dims_matches_mpi():
    assert [compute_dims(n, 3) for n in (1, 2, 3, 4, 6, 8, 12)] == [
        (1, 1, 1), (2, 1, 1), (3, 1, 1), (2, 2, 1), (3, 2, 1), (2, 2, 2), (3, 2, 2)]
    assert compute_dims(4, 2) == (2, 2) and compute_dims(4, 1) == (4,)
    assert [cart_coords(r, (2, 2, 1)) for r in range(4)] == [(0, 0, 0), (0, 1, 0), (1, 0, 0),
                                                             (1, 1, 0)]


def test_unit_range():
    r = UnitRange(3, 9)
    assert r.size == 6 and len(r) == 6 and list(r) == [3, 4, 5, 6, 7, 8]
    assert r[0] == 3 and r[-1] == 8 and r[1:-1] == UnitRange(4, 8) and r[:2] == UnitRange(3, 5)
    with pytest.raises(IndexError):
        r[6]
    with pytest.raises(ValueError):
        UnitRange(3, 2)
    assert UnitRange(5, 5).empty and UnitRange(5, 5).as_tuple() == (0, 0)
    assert r.intersect(UnitRange(7, 20)) == UnitRange(7, 9)
    assert r.intersect(UnitRange(20, 30)).empty
    assert r.without(UnitRange(5, 6)) == union(UnitRange(3, 5), UnitRange(6, 9))
    assert isinstance(r.without(UnitRange(5, 6)), UnionRange)
    assert r.without(UnitRange(0, 100)).empty
    assert r.extend(2) == UnitRange(1, 11) and r.extend((0, 1)) == UnitRange(3, 10)
    assert r.translate(-3) == UnitRange(0, 6)
    assert 3 in r and 9 not in r
    # complement within the universe: two unbounded halves
    c = r.complement()
    assert -10 ** 9 in c and 10 ** 9 in c and 5 not in c
    assert union(UnitRange(0, 2), UnitRange(2, 4)) == UnitRange(0, 4)
    assert isinstance(union(UnitRange(0, 2), UnitRange(2, 4)), UnitRange)  # fused
    u = union(UnitRange(0, 5), UnitRange(3, 8), simplify=False)  # overlap held once
    assert u.size == 8 and sorted(u) == list(range(8))


def test_product_set():
    b = UnitRange(0, 4) * UnitRange(10, 13) * UnitRange(-1, 1)
    assert isinstance(b, ProductSet) and b.ndim == 3 and b.shape == (4, 3, 2) and b.size == 24
    assert b[0, 0, 0] == (0, 10, -1) and b[-1, -1, -1] == (3, 12, 0)
    assert b[1:3, :, :] == UnitRange(1, 3) * UnitRange(10, 13) * UnitRange(-1, 1)
    pts = list(b)
    assert len(pts) == 24 and pts[:3] == [(0, 10, -1), (0, 10, 0), (0, 11, -1)]  # last fastest
    assert (3, 12, 0) in b and (4, 12, 0) not in b
    assert b.translate(1, -10, 1) == UnitRange(1, 5) * UnitRange(0, 3) * UnitRange(0, 2)
    e = b.extend(1, (0, 2), 0)
    assert e == UnitRange(-1, 5) * UnitRange(10, 15) * UnitRange(-1, 1)
    halo = e.without(b)
    assert isinstance(halo, UnionCartesian)
    assert halo.size == e.size - b.size and set(halo) == set(e) - set(b)
    assert halo.bounds == e and not halo.issubset(b) and b.issubset(e)
    assert union(halo, b) == e
    assert b.intersect(UnitRange(2, 9) * UnitRange(0, 11) * UnitRange(0, 5)) == \
        UnitRange(2, 4) * UnitRange(10, 11) * UnitRange(0, 1)
    ps = ProductSet.from_coords((3, 0, 2), (8, 4, 3))
    assert ps.shape == (6, 5, 2) and ps[(-1, -1, -1)] == (8, 4, 3)
    # a box minus an interior box: disjoint pieces, each cell once
    big = UnitRange(0, 6) * UnitRange(0, 6)
    hole = big.without(UnitRange(2, 4) * UnitRange(2, 4))
    assert hole.size == 32 and len(set(hole)) == 32 and (2, 2) not in hole
    assert big.complement(UnitRange(-1, 7) * UnitRange(-1, 7)).size == 64 - 36


def test_random_set_algebra_against_python_sets():
    """without / union / intersect / equality of random 2-D boxes against Python's sets."""
    import random
    rnd = random.Random(7)

    def box():
        a, b = sorted(rnd.sample(range(0, 12), 2))
        c, d = sorted(rnd.sample(range(0, 12), 2))
        return UnitRange(a, b) * UnitRange(c, d)

    for _ in range(300):
        xs = [box() for _ in range(rnd.randint(1, 4))]
        u = union(*xs, simplify=rnd.random() < 0.5)
        want = set().union(*(set(x) for x in xs))
        assert set(u) == want and u.size == len(want) and len(list(u)) == len(want)
        y = box()
        assert set(u.without(y)) == want - set(y)
        assert set(u.intersect(y)) == want & set(y)
        assert (u == y) == (want == set(y))
        assert u.issubset(u.bounds)


def test_index_space_decompose():
    g = IndexSpace.from_sizes(48, 24, 16)
    assert g.ndim == 3 and g.shape == (48, 24, 16) and g.default_origin == (0, 0, 0)
    parts = g.decompose((3, 2, 1))
    assert sorted(parts) == sorted(itertools.product(range(3), range(2), range(1)))
    assert parts[(2, 1, 0)].subset["definition"] == \
        UnitRange(32, 48) * UnitRange(12, 24) * UnitRange(0, 16)
    odd = IndexSpace.from_sizes(10).decompose((3,))  # floor(10/3) = 3: 3, 3, 4 cells
    assert [odd[(i,)].subset["definition"].shape for i in range(3)] == [(3,), (3,), (4,)]
    own = parts[(1, 0, 0)].subset["definition"]
    sg = IndexSpace({"definition": own, "halo": own.extend(1, 2, 0).without(own)})
    assert sg.bounds == own.extend(1, 2, 0)
    t = sg.translate(*(-o for o in sg.bounds[(0, 0, 0)]))
    assert t.bounds[(0, 0, 0)] == (0, 0, 0) and t.shape == sg.shape
    assert t.subset["definition"][(0, 0, 0)] == (1, 2, 0)


# ---- the reference binding's structured domain tests, per emulated rank -----------------------

Nx, Ny, Nz = 10, 10, 2
HALOSS = [(1, 0, 0), (1, 2, 3), ((1, 0), (0, 0), (0, 0)), ((1, 0), (0, 2), (2, 2))]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_domain_descriptor(world):
    """test_structured_domain_descriptor.py::test_domain_descriptor."""
    from ghex_amd.structured.regular import DomainDescriptor
    dims = compute_dims(world, 3)
    for rank in range(world):
        i, j, k = cart_coords(rank, dims)
        sub = (UnitRange(i * Nx, (i + 1) * Nx) * UnitRange(j * Ny, (j + 1) * Ny) *
               UnitRange(k * Nz, (k + 1) * Nz))
        dd = DomainDescriptor(rank, sub)
        assert dd.domain_id() == rank
        assert dd.first() == sub[0, 0, 0]
        assert dd.last() == sub[-1, -1, -1]


@pytest.mark.parametrize("halos", HALOSS)
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_halo_gen_call(world, halos):
    """test_structured_domain_descriptor.py::test_halo_gen_construction / test_halo_gen_call /
    test_domain_descriptor_grid: the generator's global halo of every rank's sub-grid equals
    owned.extend(*halos).without(owned) (non-periodic)."""
    from ghex_amd.structured.regular import DomainDescriptor, HaloGenerator
    dims = compute_dims(world, 3)
    periodicity = (False, False, False)
    glob = UnitRange(0, dims[0] * Nx) * UnitRange(0, dims[1] * Ny) * UnitRange(0, dims[2] * Nz)
    HaloGenerator(glob, halos, periodicity)  # construction from an index set
    global_grid = IndexSpace.from_sizes(Nx, Ny, Nz)
    sub_grids = global_grid.decompose(dims)
    for rank in range(world):
        p_coord = cart_coords(rank, dims)
        owned = sub_grids[p_coord].subset["definition"]
        sub_grid = IndexSpace({"definition": owned,
                               "halo": owned.extend(*halos).without(owned)})
        halo_gen = HaloGenerator(global_grid.subset["definition"], halos, periodicity)
        dd = DomainDescriptor(rank, owned)
        assert sub_grid.subset["halo"] == halo_gen(dd).global_, (world, rank, halos)
        assert dd.domain_id() == rank
        assert dd.first() == owned.bounds[0, 0, 0]
        assert dd.last() == owned.bounds[-1, -1, -1]


def test_index_space_prune_intersect_and_misc():
    own = UnitRange(0, 4) * UnitRange(0, 4)
    sp = IndexSpace({"definition": own, "halo": own.extend(1, 1).without(own),
                     "nothing": own.without(own)})
    assert not sp.empty and sp.ndim == 2 and sp.shape == (6, 6)
    pruned = sp.prune()
    assert set(pruned.subset) == {"definition", "halo"}
    cut = sp.intersect(UnitRange(0, 10) * UnitRange(-10, 2))
    assert cut.subset["definition"] == UnitRange(0, 4) * UnitRange(0, 2)
    assert set(cut.subset["halo"]) == {p for p in sp.subset["halo"] if p[0] >= 0 and p[1] < 2}
    assert IndexSpace({"definition": own.without(own)}).empty
    with pytest.raises(ValueError):
        IndexSpace({"halo": own})
    with pytest.deprecated_call():
        assert own.dim == 2
    assert hash(own) == hash(UnitRange(0, 4) * UnitRange(0, 4))
    assert repr(own) == "UnitRange(0, 4) * UnitRange(0, 4)"
    assert UnitRange(0, 3) * union(UnitRange(0, 1), UnitRange(2, 3)) == \
        union(UnitRange(0, 3) * UnitRange(0, 1), UnitRange(0, 3) * UnitRange(2, 3))
