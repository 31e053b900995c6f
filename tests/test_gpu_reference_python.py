"""The reference binding's structured pattern test (test/bindings/python/test_structured_pattern.py)
and unstructured domain test (test_unstructured_domain_descriptor.py::test_domain_descriptor)
run against ghex_amd with its own vocabulary (cartesian_sets.IndexSpace, DomainDescriptor,
HaloGenerator, make_pattern, make_field_descriptor, make_communication_object), the MPI ranks
emulated in one process on one GPU (tests/gpu_util.py: FakeContext + an in-process router for the
peer messages). Fields are device tensors in the reference's order="F" layout. Besides the
reference's own check (interior-index halo cells hold their owner's coordinates and rank), the
periodic halo cells are checked too, their owner found by wrapping the global index."""
import pytest

from tests.test_cartesian_sets import cart_coords, compute_dims

pytestmark = pytest.mark.gpu

SIZES = (48, 24, 16)
HALOS_PER_DIM = ((2, 1), (1, 2), (1, 1))


def _f_order_zeros(torch, shape):
    """np.zeros(shape, order="F") as a device tensor: dimension 0 fastest in memory."""
    return torch.zeros(tuple(reversed(shape)), dtype=torch.float64,
                       device="cuda").permute(*reversed(range(len(shape))))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("periodic", [True, False])
@pytest.mark.parametrize("ndim", [1, 2, 3])
def test_pattern(ndim, periodic, world):
    import torch
    from ghex_amd.structured.cartesian_sets import IndexSpace
    from ghex_amd.structured.regular import (DomainDescriptor, HaloGenerator,
                                             make_communication_object, make_field_descriptor,
                                             make_pattern)
    from tests.gpu_util import FakeContext, emulated_exchange

    dims = compute_dims(world, ndim)
    halos = tuple(HALOS_PER_DIM[d] for d in range(ndim))
    periodicity = tuple(periodic if d == 0 else True for d in range(ndim))
    global_grid = IndexSpace.from_sizes(*SIZES[:ndim])
    sub_grids = global_grid.decompose(dims)
    halo_gen = HaloGenerator(global_grid.subset["definition"], halos, periodicity)

    ranks = []
    for r in range(world):
        p_coord = cart_coords(r, dims)
        owned = sub_grids[p_coord].subset["definition"]
        sub_grid = IndexSpace({"definition": owned,
                               "halo": owned.extend(*halos).without(owned)})
        memory_local_grid = sub_grid.translate(*(-o for o in sub_grid.bounds[(0,) * ndim]))
        ranks.append(dict(coord=p_coord, owned=owned, sub_grid=sub_grid,
                          mem=memory_local_grid, dd=DomainDescriptor(r, owned)))
    table = {r: [(r, x["dd"].first(), x["dd"].last())] for r, x in enumerate(ranks)}
    cos, pats = [], []
    for r, x in enumerate(ranks):
        ctx = FakeContext(r, world, table)
        pats.append(make_pattern(ctx, halo_gen, [x["dd"]]))
        assert pats[-1].grid_type == "structured" and pats[-1].domain_id_type == "int"
        cos.append(make_communication_object(ctx))

    def make_field(x):
        f = _f_order_zeros(torch, x["mem"].bounds.shape)
        return f, make_field_descriptor(x["dd"], f, x["mem"].subset["definition"][(0,) * ndim],
                                        x["mem"].bounds.shape)

    fields, gfields, rank_fields, grank_fields = [], [], [], []
    for r, x in enumerate(ranks):
        fs, gs = zip(*(make_field(x) for _ in range(ndim)))
        for d, c in enumerate(x["coord"]):
            fs[d][...] = c
        fields.append(fs)
        gfields.append(gs)
        rf, grf = make_field(x)
        rf[...] = r
        rank_fields.append(rf)
        grank_fields.append(grf)
    emulated_exchange(cos, [[pats[r](g) for g in gfields[r]] for r in range(world)])
    emulated_exchange(cos, [[pats[r](grank_fields[r])] for r in range(world)])

    last = global_grid.subset["definition"][(-1,) * ndim]
    size = SIZES[:ndim]
    checked = wrapped = 0
    for r, x in enumerate(ranks):
        fh = [f.cpu().numpy() for f in fields[r]]
        rh = rank_fields[r].cpu().numpy()
        for m_idx, local_idx in zip(x["mem"].bounds, x["sub_grid"].bounds):
            owner_coord = tuple(int(fh[d][m_idx]) for d in range(ndim))
            inside = all(0 <= l <= last[d] for d, l in enumerate(local_idx))
            if inside:  # the reference's check
                assert local_idx in sub_grids[owner_coord].subset["definition"], (r, local_idx)
                assert rh[m_idx] == dims_rank(owner_coord, dims), (r, local_idx)
                checked += 1
            elif all(periodicity[d] or 0 <= l <= last[d] for d, l in enumerate(local_idx)):
                g = tuple(l % size[d] for d, l in enumerate(local_idx))
                if local_idx in x["sub_grid"].subset["halo"]:
                    assert g in sub_grids[owner_coord].subset["definition"], (r, local_idx)
                    assert rh[m_idx] == dims_rank(owner_coord, dims), (r, local_idx)
                    wrapped += 1
    assert checked > 0
    if any(periodicity):
        assert wrapped > 0


def dims_rank(coord, dims):
    """MPI_Cart_rank (row-major)."""
    r = 0
    for c, d in zip(coord, dims):
        r = r * d + c
    return r


@pytest.mark.parametrize("dtype", ["float64", "float32", "int32", "int64"])
def test_unstructured_domain_descriptor(golden_dir, dtype):
    """test/bindings/python/test_unstructured_domain_descriptor.py::test_domain_descriptor on 4
    emulated ranks (its fixture: tests/golden/unstructured_case.json "python_fixture"): each rank
    one domain with HaloGenerator.from_gids(outer), two fields of LEVELS=2 (order "C": levels
    first; order "F": levels as the outer stride) in one exchange; inner cells hold
    rank*1000 + 10*gid + level, halos -1 before; afterwards every halo value's last three digits
    are 10*gid + level, as the reference checks."""
    import json
    import os

    import numpy as np
    import torch
    from ghex_amd import unstructured as U
    from ghex_amd.context import LoopbackWorld
    from tests.gpu_util import FakeContext, emulated_exchange

    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        fx = json.load(fh)["python_fixture"]
    L, doms = fx["levels"], fx["domains"]
    W = 4

    def rank_fn(ctx):
        d = doms[str(ctx.rank())]
        dd = U.DomainDescriptor(ctx.rank(), d["all"], d["outer_lids"])
        return dd, U.make_pattern(ctx, U.HaloGenerator.from_gids(d["outer"]), [dd])

    pats = LoopbackWorld(W).run(rank_fn)
    table = {r: [] for r in range(W)}
    cos, bis, fields = [], [], []
    for r in range(W):
        d = doms[str(r)]
        dd, pattern = pats[r]
        assert dd.domain_id() == r
        assert dd.size() == len(d["all"])
        assert dd.inner_size() == len(d["inner"])
        inner = set(d["inner"])
        host = np.array([[r * 1000 + 10 * g + l if g in inner else -1 for l in range(L)]
                         for g in d["all"]], dtype=dtype)
        mine = []
        bis.append([])
        for order in ("C", "F"):
            a = np.array(host, order=order)
            t = torch.from_numpy(a).cuda() if order == "C" else \
                torch.from_numpy(np.ascontiguousarray(a.T)).cuda().t()
            fd = U.make_field_descriptor(dd, t)
            assert fd.levels_first == (order == "C")
            mine.append((order, t))
            bis[r].append(pattern(fd))
        fields.append(mine)
        cos.append(U.make_communication_object(FakeContext(r, W, table)))
    emulated_exchange(cos, bis)
    for r in range(W):
        d = doms[str(r)]
        inner = set(d["inner"])
        for order, t in fields[r]:
            got = t.cpu().numpy()
            for x, g in enumerate(d["all"]):
                for l in range(L):
                    if g in inner:
                        assert got[x, l] == r * 1000 + 10 * g + l, (r, order, x)
                    else:
                        v = int(got[x, l])
                        assert v - 1000 * int(v / 1000) == 10 * g + l, (r, order, x, v)


class _CudaArray:
    """A producer that exposes only __cuda_array_interface__ (as CuPy / Numba arrays do)."""

    def __init__(self, t):
        self._t = t
        self.__cuda_array_interface__ = t.__cuda_array_interface__


class _HipArray:
    """A producer that exposes only __hip_array_interface__."""

    def __init__(self, t):
        self._t = t
        self.__hip_array_interface__ = t.__cuda_array_interface__


@pytest.mark.parametrize("wrap", [_CudaArray, _HipArray])
def test_array_interface_fields(wrap):
    """make_field_descriptor on non-torch device arrays, as the reference binding takes them
    (__cuda_array_interface__ / __hip_array_interface__, structured/regular.py:66-98 and
    unstructured.py:38-60): the exchange writes the producer's own memory (zero-copy)."""
    import numpy as np
    import torch
    import ghex_amd
    from ghex_amd import unstructured as U
    from ghex_amd.structured import regular as R
    from tests import helpers as H
    N, Hw = 12, 2
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    expect = H.expected_linear_halo(a, dom, N, Hw, gl)
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    base = torch.from_numpy(a.copy()).cuda()          # memory order (z, y, x)
    arr = wrap(base.permute(2, 1, 0))                  # logical (x, y, z), x fastest
    fd = R.make_field_descriptor(dd, arr, (Hw,) * 3, (E,) * 3)
    assert fd.tensor.data_ptr() == base.data_ptr()
    R.make_communication_object(ctx).exchange([pc(fd)]).wait()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(base.cpu().numpy(), expect)
    # unstructured: one domain whose outer cells are its own inner cells' gids elsewhere in a
    # second domain of the same rank
    d0 = U.DomainDescriptor(0, [0, 1, 2, 10], [3])
    d1 = U.DomainDescriptor(1, [10, 11, 12, 0], [3])
    upc = U.make_pattern(ctx, U.HaloGenerator(), [d0, d1])
    v0 = torch.tensor([0.0, 1.0, 2.0, -1.0], device="cuda", dtype=torch.float64)
    v1 = torch.tensor([10.0, 11.0, 12.0, -1.0], device="cuda", dtype=torch.float64)
    f0, f1 = U.make_field_descriptor(d0, wrap(v0)), U.make_field_descriptor(d1, wrap(v1))
    U.make_communication_object(ctx).exchange([upc(f0), upc(f1)]).wait()
    torch.cuda.synchronize()
    assert v0.tolist() == [0.0, 1.0, 2.0, 10.0] and v1.tolist() == [10.0, 11.0, 12.0, 0.0]


def test_host_arrays_refused():
    import numpy as np
    import ghex_amd
    from ghex_amd.structured import regular as R
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (3, 3, 3))
    with pytest.raises(TypeError, match="host array"):
        R.make_field_descriptor(dd, np.zeros((6, 6, 6)), (1, 1, 1), (6, 6, 6))
    del ctx
