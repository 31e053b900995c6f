"""Maximum sizes: fields beyond 4 GiB (64-bit field byte offsets; the reference's strides are
32-bit `unsigned`, include/ghex/structured/field_descriptor.hpp:39-40) and iteration spaces
beyond 2^31 bytes (the planner splits them into segments below 2^31 along the slowest dim).

Checked on the device through the reference tests' own size-independent property: after an
exchange every cell of the (N+2H) box equals the periodic-wrapped global linear index
(test/structured/regular/test_regular_domain.cpp:739-800), owned cells unchanged."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def _exchange_and_check(N, halos, fuse):
    """One periodic domain of extent N (x, y, z) with halos (x-, x+, y-, y+, z-, z+); returns the
    number of wrong cells, checked one z-plane block at a time."""
    import torch
    import ghex_amd
    from ghex_amd.structured import regular as R
    dev = torch.device("cuda", 0)
    lo = (halos[0], halos[2], halos[4])
    E = tuple(N[d] + halos[2 * d] + halos[2 * d + 1] for d in range(3))
    base = torch.full((E[2], E[1], E[0]), -1.0, dtype=torch.float64, device=dev)
    ar = [torch.arange(N[d], device=dev, dtype=torch.float64) for d in range(3)]
    for z in range(N[2]):  # plane by plane: no full-size temporaries
        base[lo[2] + z, lo[1]:lo[1] + N[1], lo[0]:lo[0] + N[0]] = (
            ar[0].view(1, N[0]) + N[0] * (ar[1].view(N[1], 1) + N[1] * float(z)))
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), tuple(n - 1 for n in N))
    hg = R.HaloGenerator((0, 0, 0), tuple(n - 1 for n in N), tuple(halos), (True,) * 3)
    pc = R.make_pattern(ctx, hg, [dd])
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), lo, E)
    co = R.make_communication_object(ctx, fuse_self=fuse)
    co.exchange([pc(fd)]).wait()
    wx = ((torch.arange(E[0], device=dev) - lo[0]) % N[0]).to(torch.float64)
    wy = ((torch.arange(E[1], device=dev) - lo[1]) % N[1]).to(torch.float64)
    bad = 0
    step = max(1, (1 << 27) // (E[0] * E[1]))
    for z0 in range(0, E[2], step):
        z1 = min(E[2], z0 + step)
        wz = ((torch.arange(z0, z1, device=dev) - lo[2]) % N[2]).to(torch.float64)
        exp = wx.view(1, 1, -1) + N[0] * (wy.view(1, -1, 1) + N[1] * wz.view(-1, 1, 1))
        bad += int((base[z0:z1] != exp).sum().item())
    del base, co, fd, pc
    torch.cuda.empty_cache()
    return bad


@pytest.mark.parametrize("fuse", [True, False])
def test_field_over_4gib(fuse):
    """1024 x 1024 x 520 fp64 with halo 2 on every side: a 4.43 GB field, so the +z faces,
    edges and corners sit beyond byte offset 2^32; fused self exchange and pack + unpack."""
    assert _exchange_and_check((1024, 1024, 520), (2,) * 6, fuse) == 0


def test_iteration_space_over_2gib():
    """8192 x 8192 x 8 fp64 with halo 4 in z only: each z-face is 8192*8192*4*8 = 2^31 bytes,
    which the planner must split (segments < 2^31); 8.6 GB field."""
    assert _exchange_and_check((8192, 8192, 8), (0, 0, 0, 0, 4, 4), True) == 0


@pytest.mark.parametrize("levels,first", [(1, True), (2, False)])
def test_unstructured_list_beyond_one_segment(levels, first):
    """An index list whose message exceeds the 1 GiB a segment addresses (140M fp64 lids, or 70M
    lids x 2 levels levels-last): the planner splits it into index ranges (levels-last: level by
    level), and the gather and scatter still equal the oracle's get/set byte for byte (checked
    on a strided sample of the 1.1 GB buffer and in full through FNV-1a checksums)."""
    import ctypes
    import numpy as np
    import torch
    from ghex_amd import _ghx
    from oracle import oracle as orc
    n = 140_000_000 // levels
    rng = np.random.default_rng(31)
    lids = rng.permutation(n).astype(np.int64)
    vals = np.arange(n * levels, dtype=np.float64)
    dv = torch.from_numpy(vals).cuda()

    def plan(direction):
        e = _ghx.UPackEntry()
        e.data.elem_size, e.data.levels, e.data.levels_first = 8, levels, 1 if first else 0
        e.data.index_stride = levels if first else 1
        e.data.level_stride = 1 if first else n
        e.field_slot, e.buffer_slot, e.buffer_offset = 0, 0, 0
        e.lids = lids.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        e.n_lids = n
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", ctypes.byref(e), 1, direction, ctypes.byref(h))
        ns = ctypes.c_int32()
        _ghx.call("ghx_uplan_info", h, None, ctypes.byref(ns), None)
        return h, ns.value

    hp, ns = plan(0)
    assert ns >= 2  # split
    buf = torch.empty(n * levels * 8, dtype=torch.uint8, device="cuda")
    L = _ghx.lib()
    s = torch.cuda.current_stream().cuda_stream
    _ghx.check(L.ghx_uplan_execute(hp, _ghx.ptr_array([dv.data_ptr()]), 1,
                                   _ghx.ptr_array([buf.data_ptr()]), 1, s), "pack")
    torch.cuda.synchronize()
    ob = np.zeros(n * levels * 8, np.uint8)
    orc.unstructured_get(vals, ob, 8, lids, levels, first, levels if first else 1,
                         1 if first else n)
    got = buf.cpu().numpy()
    assert orc.fnv1a64(got) == orc.fnv1a64(ob)
    # scatter back into a zeroed field: every value returns to its place
    dv.zero_()
    hu, _ = plan(1)
    _ghx.check(L.ghx_uplan_execute(hu, _ghx.ptr_array([dv.data_ptr()]), 1,
                                   _ghx.ptr_array([buf.data_ptr()]), 1, s), "unpack")
    torch.cuda.synchronize()
    assert orc.fnv1a64(dv.cpu().numpy()) == orc.fnv1a64(vals)
    for h in (hp, hu):
        L.ghx_uplan_destroy(h)
