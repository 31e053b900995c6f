"""Edge cases of the device path: the smallest domains (1-3 cells per side, halo up to the domain
extent, so halo boxes wrap a whole period), index lists that are empty or hold one lid, and
exchanges that carry no message at all. Bytes and fields against the oracle."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as orc
from tests.test_gpu_parity import test_single_domain_periodic_fp64
from tests.test_gpu_self import fused_vs_unfused

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


@pytest.mark.parametrize("N,Hw", [(1, 1), (2, 1), (2, 2), (3, 2), (3, 3)])
@pytest.mark.parametrize("layout", [(2, 1, 0), (1, 0, 2)])
def test_tiny_periodic_domains(N, Hw, layout):
    """Two-launch pack/unpack (buffer bytes + fields vs the oracle) on 1^3..3^3 domains."""
    test_single_domain_periodic_fp64(layout, Hw, N)


@pytest.mark.parametrize("N,Hw", [(1, 1), (2, 2), (3, 3)])
def test_tiny_periodic_domains_fused(N, Hw):
    """The fused self exchange on the same tiny domains (one workgroup tile per segment)."""
    fused_vs_unfused(Hw, (2, 1, 0), N)


def test_unstructured_empty_and_single_lists():
    """A plan whose lists are empty, one lid long, and ordinary: the empty list moves nothing,
    the others match the oracle's get/set; an all-empty plan launches nothing."""
    import torch
    from ghex_amd import _ghx
    rng = np.random.default_rng(3)
    n = 1000
    vals = rng.random(n)
    dv = torch.from_numpy(vals).cuda()
    lists = [np.array([], np.int64), np.array([417], np.int64), rng.choice(n, 77, replace=False)]

    def plan(ls, direction):
        ents, keep = [], []
        for k, l in enumerate(ls):
            e = _ghx.UPackEntry()
            e.data.elem_size, e.data.levels, e.data.levels_first = 8, 1, 1
            e.data.index_stride, e.data.level_stride = 1, 1
            e.field_slot, e.buffer_slot, e.buffer_offset = 0, k, 0
            arr = np.ascontiguousarray(l, dtype=np.int64)
            keep.append(arr)
            e.lids = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            e.n_lids = len(arr)
            ents.append(e)
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", (_ghx.UPackEntry * len(ents))(*ents), len(ents), direction,
                  ctypes.byref(h))
        return h

    s = torch.cuda.current_stream().cuda_stream
    bufs = [torch.full((max(1, len(l)) * 8,), 7, dtype=torch.uint8, device="cuda") for l in lists]
    hp = plan(lists, 0)
    _ghx.call("ghx_uplan_execute", hp, _ghx.ptr_array([dv.data_ptr()]), 1,
              _ghx.ptr_array([b.data_ptr() for b in bufs]), len(bufs), s)
    torch.cuda.synchronize()
    assert (bufs[0].cpu().numpy() == 7).all(), "an empty list wrote its buffer"
    for l, b in zip(lists[1:], bufs[1:]):
        ob = np.zeros(len(l) * 8, np.uint8)
        orc.unstructured_get(vals, ob, 8, l, 1, True, 1, 1)
        assert np.array_equal(b.cpu().numpy(), ob)
    hu = plan(lists, 1)
    fresh = [rng.integers(0, 256, size=b.numel(), dtype=np.uint8) for b in bufs]
    rb = [torch.from_numpy(f).cuda() for f in fresh]
    _ghx.call("ghx_uplan_execute", hu, _ghx.ptr_array([dv.data_ptr()]), 1,
              _ghx.ptr_array([b.data_ptr() for b in rb]), len(rb), s)
    torch.cuda.synchronize()
    exp = vals.copy()
    for l, f in zip(lists[1:], fresh[1:]):
        orc.unstructured_set(exp, f, 8, l, 1, True, 1, 1)
    assert np.array_equal(dv.cpu().numpy().view(np.uint64), exp.view(np.uint64))
    he = plan([lists[0], lists[0]], 0)
    _ghx.call("ghx_uplan_execute", he, _ghx.ptr_array([dv.data_ptr()]), 1,
              _ghx.ptr_array([bufs[0].data_ptr(), bufs[0].data_ptr()]), 2, s)
    torch.cuda.synchronize()
    for h in (hp, hu, he):
        _ghx.lib().ghx_uplan_destroy(h)


def test_exchange_without_messages():
    """A non-periodic single domain has no neighbours: the exchange moves nothing, leaves the
    field untouched and completes (wait and is_ready)."""
    import torch
    import ghex_amd
    from ghex_amd.structured import regular as R
    N, Hw = 6, 2
    E = N + 2 * Hw
    t = torch.arange(E ** 3, dtype=torch.float64, device="cuda").view(E, E, E)
    before = t.clone()
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (Hw,) * 6, (False,) * 3),
                        [dd])
    fd = R.make_field_descriptor(dd, t.permute(2, 1, 0), (Hw,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx)
    h = co.exchange([pc(fd)])
    h.wait()
    assert torch.equal(t, before)
    h2 = co.exchange([pc(fd)])
    torch.cuda.synchronize()
    assert h2.is_ready()
    assert torch.equal(t, before)
