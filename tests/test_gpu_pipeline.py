"""Per-buffer plans and the per-peer pipelined exchange on the GPU, bit-exact.

* ghx_exchange_pack_buffer / unpack_buffer (one launch per buffer, the reference's per-buffer
  packer call, include/ghex/communication_object.hpp:568-597) produce exactly the bytes of the
  fused ghx_exchange_pack / unpack, structured and unstructured.
* Emulated ranks on one GPU with the pipeline's event ordering: every buffer packed on its peer's
  own stream, each message routed on the receiver's peer stream only after the sender's pack
  event, unpacked there, the caller's stream joining all of them — fields checked against the
  oracle's exchange and the reference tests' halo property.
* The native pipeline (ghx_pipeline_*) with its RCCL path running on a one-GPU box: self messages
  routed through a 1-rank RCCL communicator (ncclSend/ncclRecv to self in one group per peer
  stream), and the all-local form.
* The unstructured convenience plan cache: a list mutated in place (an entry no sampling would
  see) gets the new bytes.
"""
import ctypes

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


def _cube_rank_setup(parts, N, Hw, r=None, fields=1):
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    table = {q: [(d.id, d.first, d.last) for d in ranks[q]] for q in range(nr)}
    out = []
    for q in range(nr) if r is None else [r]:
        ctx = FakeContext(q, nr, table)
        dd = R.DomainDescriptor(ranks[q][0].id, ranks[q][0].first, ranks[q][0].last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)), [dd])
        items = []
        for k in range(fields):
            a, spec = H.linear_index_field(ranks[q][0], N, Hw, gl, seed=k if k else None)
            base, logical = device_field(a.copy(), (2, 1, 0))
            fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
            items.append((a, spec, base, fd))
        co = R.make_communication_object(ctx)
        out.append(dict(ctx=ctx, pc=pc, items=items, co=co, bis=[pc(it[3]) for it in items]))
    return out, ranks, gf, gl


def _per_buffer_vs_fused(co, bis):
    import torch
    from ghex_amd import _ghx
    L = _ghx.lib()
    plan = co.plan(bis)
    co._split(plan)
    dev = bis[0].field.device
    s = torch.cuda.current_stream().cuda_stream
    fp = _ghx.ptr_array([b.field.data_ptr() for b in bis])
    ns, nr = len(plan.send), len(plan.recv)
    A = [torch.zeros(max(1, x["size"]), dtype=torch.uint8, device=dev) for x in plan.send]
    B = [torch.full((max(1, x["size"]),), 7, dtype=torch.uint8, device=dev) for x in plan.send]
    _ghx.check(L.ghx_exchange_pack(plan.h, fp, len(bis), _ghx.ptr_array([t.data_ptr() for t in A]),
                                   ns, s), "pack")
    bp = _ghx.ptr_array([t.data_ptr() for t in B])
    for i in reversed(range(ns)):  # any order: each launch touches its own buffer only
        _ghx.check(L.ghx_exchange_pack_buffer(plan.h, i, fp, len(bis), bp, ns, s), "pack_buffer")
    torch.cuda.synchronize()
    for i, x in enumerate(plan.send):
        assert torch.equal(A[i][:x["size"]], B[i][:x["size"]]), f"send buffer {i}"
    # unpack: the same random recv bytes through both paths into two copies of the fields
    g = torch.Generator(device="cpu").manual_seed(5)
    Rb = [torch.randint(0, 256, (max(1, x["size"]),), generator=g, dtype=torch.uint8).to(dev)
          for x in plan.recv]
    rp = _ghx.ptr_array([t.data_ptr() for t in Rb])
    snap = [b.field.tensor.clone() for b in bis]
    _ghx.check(L.ghx_exchange_unpack(plan.h, fp, len(bis), rp, nr, s), "unpack")
    torch.cuda.synchronize()
    fused = [b.field.tensor.clone() for b in bis]
    for b, t in zip(bis, snap):
        b.field.tensor.copy_(t)
    for j in range(nr):
        _ghx.check(L.ghx_exchange_unpack_buffer(plan.h, j, fp, len(bis), rp, nr, s), "unpack_buffer")
    torch.cuda.synchronize()
    for b, f in zip(bis, fused):
        assert torch.equal(b.field.tensor, f)
    return plan


@pytest.mark.parametrize("parts,Hw,fields", [((2, 2, 2), 2, 1), ((2, 1, 1), 3, 2), ((1, 1, 1), 1, 3)])
def test_per_buffer_plans_equal_fused(parts, Hw, fields):
    setups, *_ = _cube_rank_setup(parts, 11, Hw, r=0, fields=fields)
    plan = _per_buffer_vs_fused(setups[0]["co"], setups[0]["bis"])
    assert len(plan.send) == {1: 1, 2: 2, 8: 7}[parts[0] * parts[1] * parts[2]]


def test_per_buffer_plans_unstructured(golden_dir):
    import json
    import os
    import torch
    from ghex_amd import unstructured as U
    from tests.gpu_util import FakeContext, unstructured_patterns
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    table = {r: [] for r in range(4)}
    doms = [[(r, case["domains"][str(r)]["gids"], case["domains"][str(r)]["halo_lids"])]
            for r in range(4)]
    for r, ((dd,), pc) in enumerate(unstructured_patterns(doms)):
        d = case["domains"][str(r)]
        t = torch.arange(len(d["gids"]) * 3, dtype=torch.float64).view(-1, 3).cuda()
        co = U.make_communication_object(FakeContext(r, 4, table))
        _per_buffer_vs_fused(co, [pc(U.make_field_descriptor(dd, t))])


@pytest.mark.parametrize("parts", [(2, 2, 2), (2, 2, 1), (3, 1, 1)])
def test_emulated_per_peer_streams(parts):
    """Every rank's buffers packed on per-peer streams; each message copied on the receiver's
    peer stream after the sender's pack event (the pipeline's ordering), unpacked there; the
    caller's stream joins. Oracle bytes + halo property."""
    import torch
    from ghex_amd import _ghx
    L = _ghx.lib()
    N, Hw = 10, 2
    setups, ranks, gf, gl = _cube_rank_setup(parts, N, Hw)
    nr = len(setups)
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    orc.regular_exchange([[(st["items"][0][1], ranks[q][0].id, 0, 0)] for q, st in enumerate(setups)],
                         {0: opat}, nr)
    main = torch.cuda.current_stream()
    streams = {(q, p): torch.cuda.Stream(priority=-1) for q in range(nr) for p in range(nr)}
    st_of = []
    for q, st in enumerate(setups):
        co, bis = st["co"], st["bis"]
        plan = co.plan(bis)
        co._split(plan)
        send, recv = co.buffers(plan, bis[0].field.device)
        st_of.append((plan, send, recv, _ghx.ptr_array([b.field.data_ptr() for b in bis]),
                      _ghx.ptr_array([t.data_ptr() for t in send]),
                      _ghx.ptr_array([t.data_ptr() for t in recv])))
    start = torch.cuda.Event()
    start.record(main)
    packed = {}
    for q, (plan, send, recv, fp, sp, rp) in enumerate(st_of):  # phase 1: packs
        for i, x in enumerate(plan.send):
            s = streams[(q, x["rank"])] if x["rank"] != q else main
            s.wait_event(start)
            _ghx.check(L.ghx_exchange_pack_buffer(plan.h, i, fp, 1, sp, len(send), s.cuda_stream),
                       "pack_buffer")
            ev = torch.cuda.Event()
            ev.record(s)
            packed[(q, i)] = ev
    for q, (plan, send, recv, fp, sp, rp) in enumerate(st_of):  # phase 2: transport + unpack
        for j, x in enumerate(plan.recv):
            src = x["rank"]
            s = streams[(q, src)] if src != q else main
            if src != q:
                ps = st_of[src][0]
                i = next(i for i, y in enumerate(ps.send) if y["pair"] == x["pair"] and y["rank"] == q)
                s.wait_event(packed[(src, i)])
                with torch.cuda.stream(s):
                    recv[j][:x["size"]].copy_(st_of[src][1][i][:x["size"]], non_blocking=True)
            _ghx.check(L.ghx_exchange_unpack_buffer(plan.h, j, fp, 1, rp, len(recv), s.cuda_stream),
                       "unpack_buffer")
        for p in range(nr):
            main.wait_stream(streams[(q, p)])
    torch.cuda.synchronize()
    for q, st in enumerate(setups):
        a, _, base, _ = st["items"][0]
        np.testing.assert_array_equal(base.cpu().numpy(), a)
        np.testing.assert_array_equal(a, H.expected_linear_halo(a, ranks[q][0], N, Hw, gl))


@pytest.mark.parametrize("rccl_self", [True, False])
@pytest.mark.parametrize("N,Hw,doms", [(16, 2, 1), (9, 3, 1), (8, 1, 4)])
def test_native_pipeline_one_gpu(rccl_self, N, Hw, doms):
    """ghx_pipeline on one rank: with rccl_self every self message is sent and received through
    a 1-rank RCCL communicator on the peer stream; otherwise packed and unpacked locally. `doms`
    domains per rank along x (self messages between distinct domains), periodic."""
    import torch
    import ghex_amd
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    doms_o = [orc.RegularDomain(k, (k * N, 0, 0), ((k + 1) * N - 1, N - 1, N - 1)) for k in range(doms)]
    gf, gl = (0, 0, 0), (doms * N - 1, N - 1, N - 1)
    opat = orc.regular_make_pattern([doms_o], gf, gl, (Hw,) * 6, (1, 1, 1))
    ctx = ghex_amd.make_context()
    dds = [R.DomainDescriptor(d.id, d.first, d.last) for d in doms_o]
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), dds)
    arrs, specs, bases, bis = [], [], [], []
    for k, d in enumerate(doms_o):
        a, spec = H.linear_index_field(d, N, Hw, gl)
        base, logical = device_field(a.copy(), (2, 1, 0))
        arrs.append(a)
        specs.append((spec, d.id, k, 0))
        bases.append(base)
        bis.append(pc(R.make_field_descriptor(dds[k], logical, (Hw,) * 3, (N + 2 * Hw,) * 3)))
    orc.regular_exchange([specs], {0: opat}, 1)
    co = R.make_communication_object(ctx, pipelined=True, rccl_self=rccl_self)
    for _ in range(2):
        co.exchange(bis).wait()
    torch.cuda.synchronize()
    for a, base, d in zip(arrs, bases, doms_o):
        np.testing.assert_array_equal(base.cpu().numpy(), a)
        np.testing.assert_array_equal(a, H.expected_linear_halo(a, d, N, Hw, gl))
    if rccl_self:
        from ghex_amd import _ghx
        comms = dict(ctx._pair_comms)
        assert comms
        for comm, _ in comms.values():
            _ghx.call("ghx_rccl_comm_check", comm)
        # a second communication object of the same context reuses the pair communicators
        co2 = R.make_communication_object(ctx, pipelined=True, rccl_self=True)
        co2.exchange(bis).wait()
        assert {p: c.value for p, (c, _) in ctx._pair_comms.items()} == \
            {p: c.value for p, (c, _) in comms.items()}
        del co, co2
        import gc
        gc.collect()
        ctx.close()
        assert not ctx._pair_comms


def test_unstructured_cache_sees_in_place_change():
    """ghx_unstructured_pack twice with the same host list object; between the calls one entry
    far from any 256-point sample grid is changed in place: the second call packs the new lid."""
    import torch
    from ghex_amd import _ghx
    L = _ghx.lib()
    n, nl = 100_000, 40_000
    vals = torch.arange(n, dtype=torch.float64, device="cuda")
    rng = np.random.default_rng(3)
    lids = np.ascontiguousarray(rng.choice(n, size=nl, replace=False).astype(np.int32))
    d = _ghx.UDataDesc()
    d.elem_size, d.levels, d.levels_first, d.index_stride, d.level_stride = 8, 1, 1, 1, 1
    buf = torch.zeros(nl * 8, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    lp = lids.ctypes.data_as(ctypes.c_void_p)
    for change in (None, 157, 39_998):
        if change is not None:
            lids[change] = (int(lids[change]) + 1) % n
        _ghx.call("ghx_unstructured_pack", ctypes.byref(d), ctypes.c_void_p(vals.data_ptr()),
                  ctypes.c_void_p(buf.data_ptr()), lp, 4, nl, ctypes.c_void_p(s))
        torch.cuda.synchronize()
        got = buf.view(torch.float64).cpu().numpy()
        np.testing.assert_array_equal(got, lids.astype(np.float64))


@pytest.mark.parametrize("rccl_self", [True, False])
def test_native_pipeline_unstructured_self_exchange(golden_dir, rccl_self):
    """The reference Python test's fixture (repeated halo gids, a domain exchanging with itself,
    test/bindings/python/test_unstructured_domain_descriptor.py) with its 4 domains on ONE rank:
    every message a self message, routed through a 1-rank RCCL communicator (rccl_self) or
    packed/unpacked locally, per buffer, by the pipeline; value = owner*1000 + 10*gid + level."""
    import json
    import os
    import torch
    import ghex_amd
    from ghex_amd import unstructured as U
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        fx = json.load(fh)["python_fixture"]
    L = fx["levels"]
    items = sorted(fx["domains"].items())
    ctx = ghex_amd.make_context()
    dds = [U.DomainDescriptor(int(k), v["all"], v["outer_lids"]) for k, v in items]
    pc = U.make_pattern(ctx, U.HaloGenerator(), dds)
    fields, bis = [], []
    for (k, v), dd in zip(items, dds):
        f = np.full((len(v["all"]), L), -1, dtype=np.int64)
        outer = set(v["outer_lids"])
        for lid, gid in enumerate(v["all"]):
            if lid not in outer:
                f[lid] = [int(k) * 1000 + 10 * gid + l for l in range(L)]
        t = torch.from_numpy(f).cuda()
        fields.append(t)
        bis.append(pc(U.make_field_descriptor(dd, t)))
    co = U.make_communication_object(ctx, pipelined=True, rccl_self=rccl_self)
    co.exchange(bis).wait()
    torch.cuda.synchronize()
    for (k, v), t in zip(items, fields):
        got = t.cpu().numpy()
        for lid, gid in enumerate(v["all"]):
            for l in range(L):
                assert got[lid, l] % 1000 == 10 * gid + l, (k, lid, gid, int(got[lid, l]))
