"""Full-size parity at the BASELINE configs (GPU): configs 4 and 5 shapes at their full sizes on
one GPU, byte-exact against the oracle, plus size-independent properties."""
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


def test_config4_five_mixed_fields_256_h3():
    """5 fields 256^3, H=3, types [f64,f32,f64,f32,f64], one exchange (one periodic domain on one
    GPU: every message is a self message). Send buffer (pads masked) and all fields vs oracle."""
    import torch
    from ghex_amd import make_context
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 256, 3
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    types = [np.float64, np.float32, np.float64, np.float32, np.float64]
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    arrays, bases, bis, rf = [], [], [], []
    for k, T in enumerate(types):
        a, spec = H.linear_index_field(dom, N, Hw, gl, dtype=T, seed=k + 1)
        base, logical = device_field(a, (2, 1, 0))
        bis.append(pc(R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)))
        arrays.append(a)
        bases.append(base)
        rf.append((spec, 0, 0, 0))
    obufs = orc.regular_exchange([rf], {0: opat}, 1)
    co = R.make_communication_object(ctx)
    co.exchange(bis).wait()
    ((_, pair), ob), = obufs.items()
    send = co.buffers(co.plan(bis), bases[0].device)[0][0]
    items = [(k, 0, opat[0][0], f[0].elem, f[0].data.dtype.alignment, 1, 0) for k, f in enumerate(rf)]
    pb = orc.plan_buffers(items, receive=False)[pair]
    m = np.zeros(pb.size, bool)
    for pf in pb.fields:
        e = rf[pf.field_index][0].elem
        m[pf.offset:pf.offset + sum(b.size() for b in pf.boxes) * e] = True
    got = send[:ob.size].cpu().numpy()
    assert np.array_equal(got[m], ob[m])
    n_halo = E ** 3 - N ** 3
    assert m.sum() == n_halo * (3 * 8 + 2 * 4)  # 4*n*(3*8+2*4)/4 bytes per direction
    for base, a in zip(bases, arrays):
        assert np.array_equal(base.cpu().numpy(), a)


def _random_lists(rng, n_cells, n_halo, peers):
    """Config 5 shape: n_cells per rank (local storage order permuted), n_halo outer cells whose
    lids are scattered; send/recv lid lists split over `peers` neighbours."""
    perm = rng.permutation(n_cells)
    recv = np.sort(perm[:n_halo])  # outer cells' lids (any order is legal; sorted per peer)
    send = rng.choice(n_cells, size=n_halo, replace=False)
    cuts = np.sort(rng.choice(np.arange(1, n_halo), size=peers - 1, replace=False))
    return np.split(send, cuts), np.split(rng.permutation(recv), cuts)


@pytest.mark.parametrize("levels,levels_first", [(1, True), (8, True), (8, False), (3, False)])
def test_config5_unstructured_10M(levels, levels_first):
    """10M cells, 5% halo, 7 peers; fused gather (pack) and scatter (unpack) of every peer's
    index list vs the oracle's data_descriptor get/set, bit-exact."""
    _config5_case(levels, levels_first)


def _config5_case(levels, levels_first):
    import ctypes
    import torch
    from ghex_amd import _ghx
    rng = np.random.default_rng(20260715)
    n = 10_000_000
    nh = n // 20
    sends, recvs = _random_lists(rng, n, nh, 7)
    vals = rng.random(n * levels)
    dv = torch.from_numpy(vals).cuda()
    isd, lsd = (levels, 1) if levels_first else (1, n)

    def plan(lists, direction):
        ents, keep, off = [], [], 0
        offs = []
        for k, l in enumerate(lists):
            e = _ghx.UPackEntry()
            e.data.elem_size, e.data.levels = 8, levels
            e.data.levels_first = 1 if levels_first else 0
            e.data.index_stride, e.data.level_stride = isd, lsd
            e.field_slot, e.buffer_slot, e.buffer_offset = 0, k, 0
            arr = np.ascontiguousarray(l, dtype=np.int64)
            keep.append(arr)
            e.lids = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            e.n_lids = len(arr)
            ents.append(e)
        a = (_ghx.UPackEntry * len(ents))(*ents)
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", a, len(ents), direction, ctypes.byref(h))
        return h

    hp = plan(sends, 0)
    bufs = [torch.empty(len(l) * levels * 8, dtype=torch.uint8, device="cuda") for l in sends]
    s = torch.cuda.current_stream().cuda_stream
    _ghx.call("ghx_uplan_execute", hp, _ghx.ptr_array([dv.data_ptr()]), 1,
              _ghx.ptr_array([b.data_ptr() for b in bufs]), len(bufs), s)
    torch.cuda.synchronize()
    for l, b in zip(sends, bufs):
        ob = np.zeros(len(l) * levels * 8, np.uint8)
        orc.unstructured_get(vals, ob, 8, l, levels, levels_first, isd, lsd)
        assert np.array_equal(b.cpu().numpy(), ob)
    # unpack: scatter peer buffers (filled with fresh values) into the recv lids
    hu = plan(recvs, 1)
    rbufs, host_bufs = [], []
    for l in recvs:
        hb = rng.integers(0, 255, size=len(l) * levels * 8, dtype=np.uint8)
        host_bufs.append(hb)
        rbufs.append(torch.from_numpy(hb).cuda())
    _ghx.call("ghx_uplan_execute", hu, _ghx.ptr_array([dv.data_ptr()]), 1,
              _ghx.ptr_array([b.data_ptr() for b in rbufs]), len(rbufs), s)
    torch.cuda.synchronize()
    exp = vals.copy()
    for l, hb in zip(recvs, host_bufs):
        orc.unstructured_set(exp, hb, 8, l, levels, levels_first, isd, lsd)
    assert np.array_equal(dv.cpu().numpy().view(np.uint64), exp.view(np.uint64))
    _ghx.lib().ghx_uplan_destroy(hp)
    _ghx.lib().ghx_uplan_destroy(hu)


def test_unstructured_known_answer_on_device(golden_dir):
    """The reference's 4-domain known-answer case, emulated on one GPU: every rank's pattern
    from libghx, device gather/scatter, values checked with the test's own encoding
    (unstructured_test_case.hpp:345-388), levels 3, levels_first and levels_last."""
    import json
    import os
    import torch
    from ghex_amd import unstructured as U
    from tests.gpu_util import FakeContext, unstructured_patterns
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    L = 3
    table = {r: [] for r in range(4)}
    pats = unstructured_patterns([[(r, case["domains"][str(r)]["gids"],
                                    case["domains"][str(r)]["halo_lids"])] for r in range(4)])
    for levels_first in (True, False):
        pcs, fields, cos, bis = [], [], [], []
        for r in range(4):
            d = case["domains"][str(r)]
            (dd,), pc = pats[r]
            n = len(d["gids"])
            host = np.full((n, L), -1.0)
            for lid, gid in enumerate(d["gids"]):
                if lid not in d["halo_lids"]:
                    host[lid] = [r * 10000 + gid * 100 + l for l in range(L)]
            t = torch.from_numpy(host).cuda()
            if not levels_first:
                t = t.t().contiguous().t()  # (n, L) view with levels as the outer stride
            fields.append(t)
            fd = U.make_field_descriptor(dd, t)
            assert fd.levels_first == levels_first
            pcs.append(pc)
            cos.append(U.make_communication_object(FakeContext(r, 4, table)))
            bis.append([pc(fd)])
        from tests.gpu_util import emulated_exchange
        emulated_exchange(cos, bis)
        for r in range(4):
            d = case["domains"][str(r)]
            got = fields[r].cpu().numpy()
            for rid, rr, tag, lids in pcs[r].recv_halos(0):
                for lid in lids:
                    for l in range(L):
                        assert got[lid, l] == rid * 10000 + d["gids"][lid] * 100 + l


@pytest.mark.parametrize("levels,levels_first", [(1, True), (8, True), (3, False)])
def test_config5_product_pattern_full_size(levels, levels_first):
    """BASELINE config 5 at its size through the PRODUCT pattern: 8 emulated ranks, each 10M
    cells + 500k halo cells (tools/config5_gen.cpp), make_pattern<unstructured> run as 8 threads
    (reduced halos), CommunicationObject plans, fused device pack of every rank, messages routed,
    fused device unpack. Rank 0's packed send buffers equal the oracle's data_descriptor<cpu>::get
    over the same lid lists, bit for bit; every cell of every rank holds its owner's value
    (gid*100 + level) afterwards."""
    import torch
    from ghex_amd import unstructured as U
    from tests.gpu_util import FakeContext, emulated_exchange, unstructured_patterns
    from tools import config5 as C5
    W = 8
    doms = [C5.generate(r, W) for r in range(W)]
    pats = unstructured_patterns([[(r, g, o)] for r, (g, o) in enumerate(doms)])
    cos, bis, fields, hosts = [], [], [], []
    for r, ((dd,), pc) in enumerate(pats):
        g, o = doms[r]
        host = g.astype(np.float64)[:, None] * 100.0 + np.arange(levels)[None, :]
        init = host.copy()
        init[o] = -1.0
        t = torch.from_numpy(init).cuda()
        if not levels_first:
            t = t.t().contiguous().t()
        fd = U.make_field_descriptor(dd, t)
        assert fd.levels_first == levels_first
        fields.append(t)
        hosts.append(host)
        cos.append(U.make_communication_object(FakeContext(r, W, {q: [] for q in range(W)})))
        bis.append([pc(fd)])
    plans, bufs = emulated_exchange(cos, bis)
    # rank 0's send buffers vs the oracle's get (levels-first: index stride L; last: level
    # stride n)
    g0, o0 = doms[0]
    n0 = g0.size
    vals0 = np.ascontiguousarray(hosts[0] if levels_first else hosts[0].T).reshape(-1)
    isd, lsd = (levels, 1) if levels_first else (1, n0)
    sends = {(rr, tag): lids for rid, rr, tag, lids in pats[0][1].lid_arrays(0, 0)}
    for i, x in enumerate(plans[0].send):
        lids = sends[(x["rank"], x["tag"])]
        ob = np.zeros(len(lids) * levels * 8, np.uint8)
        orc.unstructured_get(vals0, ob, 8, lids, levels, levels_first, isd, lsd)
        assert np.array_equal(bufs[0][0][i][:x["size"]].cpu().numpy(), ob), x
    for r in range(W):
        got = fields[r].cpu().numpy()
        assert np.array_equal(got, hosts[r]), r
