"""The fused self exchange (ghx_exchange_self): every message of the exchange stays on the
device, pack and unpack run as one launch. Checked against the oracle and against the unfused
two-launch path (same buffer bytes, same fields)."""
import numpy as np
import pytest

from oracle import oracle as orc
from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


@pytest.mark.parametrize("types", [(np.float64, np.float32, np.int32),
                                   (np.float64, np.float64, np.float64)])
def test_one_rank_eight_domains_two_patterns(types):
    """The reference test geometry (test_regular_domain.cpp) with all 8 domains on ONE rank:
    3 fields x 8 domains, 2 pattern containers, every message a self message (8 x 8 domain
    pairs), fused into one launch; bytes and fields vs the oracle."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field
    from tests.test_gpu_parity import _as_struct_elem, _mask_for
    ranks4, gf, gl = H.regular_test_domains(4)
    doms = [d for r in ranks4 for d in r]  # all 8 domains on rank 0
    ranks = [doms]
    table = {0: [(d.id, d.first, d.last) for d in doms]}
    pat_o = {1: orc.regular_make_pattern(ranks, gf, gl, H.HALOS_1, (1, 1, 1)),
             2: orc.regular_make_pattern(ranks, gf, gl, H.HALOS_2, (1, 1, 1))}
    ctx = FakeContext(0, 1, table)
    dds = [R.DomainDescriptor(d.id, d.first, d.last) for d in doms]
    pcs = {1: R.make_pattern(ctx, R.HaloGenerator(gf, gl, H.HALOS_1, (1, 1, 1)), dds),
           2: R.make_pattern(ctx, R.HaloGenerator(gf, gl, H.HALOS_2, (1, 1, 1)), dds)}
    bis, bases, arrays, rf = [], [], [], []
    for fi, (T, pcn) in enumerate(zip(types, (1, 2, 1))):
        for li, dom in enumerate(doms):
            a = H.coord_field(dom, T)
            base, logical = device_field(a.copy(), (2, 1, 0, 3), has_components=True)
            ext = (a.shape[2], a.shape[1], a.shape[0])
            fd = _as_struct_elem(R.make_field_descriptor(dds[li], logical, H.OFFSET, ext),
                                 a.itemsize * 3)
            bis.append(pcs[pcn](fd))
            bases.append(base)
            arrays.append(a)
            rf.append((H.coord_fieldspec(a), dom.id, li, pcn))
    obufs = orc.regular_exchange([rf], pat_o, 1)
    co = R.make_communication_object(ctx)
    plan = co.plan(bis)
    assert co.all_self(plan), "expected an all-self exchange"
    co.exchange(bis).wait()  # fused path
    for b, a in zip(bases, arrays):
        np.testing.assert_array_equal(b.cpu().numpy(), a)
    send, _ = co.buffers(plan, bases[0].device)
    items = [(k, f[1], pat_o[f[3]][0][f[2]], f[0].elem, f[0].data.dtype.alignment, 1, 0)
             for k, f in enumerate(rf)]
    pb = orc.plan_buffers(items, receive=False)
    for i, x in enumerate(plan.send):
        ob = obufs[(0, x["pair"])]
        m = _mask_for(pb[x["pair"]], {k: (f[0].elem, 1) for k, f in enumerate(rf)})
        np.testing.assert_array_equal(send[i][:x["size"]].cpu().numpy()[m], ob[m])


@pytest.mark.parametrize("Hw", [1, 2, 3])
@pytest.mark.parametrize("layout", [(2, 1, 0), (0, 2, 1)])
def test_fused_equals_unfused_and_oracle(Hw, layout):
    fused_vs_unfused(Hw, layout, 24)


def fused_vs_unfused(Hw, layout, N):
    """One periodic N^3 domain: the fused self exchange and the two-launch path both write the
    oracle's buffer bytes and fields."""
    from ghex_amd import make_context
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, spec = H.linear_index_field(dom, N, Hw, gl, layout=layout, seed=3)
    a0 = a.copy()
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    ((_, pair), ob), = orc.regular_exchange([[(spec, 0, 0, 0)]], {0: opat}, 1).items()
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    outs = []
    for fuse in (True, False):
        base, logical = device_field(a0, layout)
        fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
        co = R.make_communication_object(ctx, fuse_self=fuse)
        co.exchange([pc(fd)]).wait()
        send, _ = co.buffers(co.plan([pc(fd)]), fd.device)
        outs.append((base.cpu().numpy(), send[0][:ob.size].cpu().numpy()))
    for field, buf in outs:
        np.testing.assert_array_equal(field, a)
        np.testing.assert_array_equal(buf, ob)


@pytest.mark.parametrize("knobs", [{"self_tile_bytes": 8192}, {"self_tile_bytes": 4096},
                                   {"self_tile_bytes": 2048, "grid_cap": 5},
                                   {"self_tile_bytes": 65536, "xcd_pair": 0},
                                   {"short_pol": 3}, {"tile_records": 0},
                                   {"self_tile_bytes": 4096, "tile_records": 0, "grid_cap": 5},
                                   {"fast_addr": 0}, {"pack_tile_rows": 64}])
@pytest.mark.parametrize("Hw", [1, 2, 3])
def test_self_kernel_variants_stay_bit_exact(knobs, Hw):
    """The fused self kernel under its remaining knobs (tile sizes, a grid-stride loop, XCD
    pairing off, cache policies, the tile-table path instead of pair records) writes the
    oracle's buffer bytes and halos."""
    from ghex_amd import _ghx
    try:
        for k, v in knobs.items():
            _ghx.call("ghx_tune", k.encode(), v)
        test_fused_equals_unfused_and_oracle(Hw, (2, 1, 0))
        test_fused_equals_unfused_and_oracle(Hw, (0, 2, 1))
    finally:
        _ghx.call("ghx_tune", b"reset", 0)


@pytest.mark.parametrize("order", ["sender_first", "receiver_first"])
@pytest.mark.parametrize("fused", [True, False])
def test_receive_only_domain_field_slot(order, fused):
    """Two domains of ONE rank stacked in y, non-periodic, a y- halo only: the lower domain only
    sends, the upper only receives, so one field slot is named by unpack segments alone. Put
    last in the exchange() arguments it is the highest slot, which the fused launch must fill
    from the unpack plan (round-3 regression: it filled up to the pack plan's highest slot and
    the kernel wrote through a null field pointer). Every cell against the expected halo."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext
    gf, gl, halos = (0, 0, 0), (3, 7, 3), (0, 0, 2, 0, 0, 0)
    doms = {"lo": (10, (0, 0, 0), (3, 3, 3)), "hi": (11, (0, 4, 0), (3, 7, 3))}
    names = ["lo", "hi"] if order == "sender_first" else ["hi", "lo"]
    ctx = FakeContext(0, 1, {0: [doms[n] for n in names]})
    dds = [R.DomainDescriptor(*doms[n]) for n in names]
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, halos, (False,) * 3), dds)
    fields, expect, bis = [], [], []
    for n, dd in zip(names, dds):
        _, first, _ = doms[n]
        a = np.full((4, 6, 4), -1.0)  # memory order (z, y, x); y: 2 halo rows + 4 owned
        z, y, x = np.meshgrid(np.arange(4), np.arange(4), np.arange(4), indexing="ij")
        a[:, 2:, :] = x + 4 * (y + first[1] + 8 * z)
        e = a.copy()
        if n == "hi":  # halo rows = global y 2, 3 of the lower domain
            zz, yy, xx = np.meshgrid(np.arange(4), np.arange(2), np.arange(4), indexing="ij")
            e[:, :2, :] = xx + 4 * (yy + 2 + 8 * zz)
        base = torch.from_numpy(a).cuda()
        fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (0, 2, 0), (4, 6, 4))
        bis.append(pc(fd))
        fields.append(base)
        expect.append(e)
    co = R.make_communication_object(ctx)
    plan = co.plan(bis)
    assert co.all_self(plan)
    if fused:
        co.exchange(bis).wait()
    else:
        co.pack_only(bis)
        co.unpack_only(bis)
    torch.cuda.synchronize()
    for base, e in zip(fields, expect):
        np.testing.assert_array_equal(base.cpu().numpy(), e)
