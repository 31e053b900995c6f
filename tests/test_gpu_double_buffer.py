"""Double-buffered launches (ghx_exchange_set_parity): the direct exchange's one-launch epochs
keep every peer receive buffer twice and let the data launches pick the copy of the exchange's
parity ON THE DEVICE, from the epoch counter, so that a captured graph alternates on replay.
Here the counter is a device word the test controls: packs and unpacks of emulated ranks must
write / read exactly the copy (*word + add) & 1 selects — bit-exact against the plain launches —
for structured, mixed (pack_self) and unstructured plans, eagerly and from a replayed graph."""
import ctypes

import numpy as np
import pytest

from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def _dbl(n):
    return max(256, (n + 255) // 256 * 256)


def _ranks(parts, N, Hw, nf=1):
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    out = []
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        dom = ranks[r][0]
        dd = R.DomainDescriptor(dom.id, dom.first, dom.last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)), [dd])
        bis, bases, arrs, exps = [], [], [], []
        for k in range(nf):  # field k = linear index + k
            a, _ = H.linear_index_field(dom, N, Hw, gl, add=k)
            base, logical = device_field(a, (2, 1, 0))
            bis.append(pc(R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)))
            bases.append(base)
            arrs.append(a)
            exps.append(H.expected_linear_halo(a, dom, N, Hw, gl) + k)
        out.append(dict(co=R.make_communication_object(ctx), bis=bis, bases=bases, arrs=arrs,
                        exps=exps, rank=r))
    torch.cuda.synchronize()
    return out


def _set(plan, direction, word, add, offsets):
    from ghex_amd import _ghx
    _ghx.call("ghx_exchange_set_parity", plan.h, direction,
              ctypes.c_void_p(word.data_ptr() if word is not None else 0), add,
              (ctypes.c_int64 * max(1, len(offsets)))(*offsets), len(offsets))


_GEOMS = [((2, 1, 1), 12, 2, 1), ((2, 2, 1), 9, 1, 1), ((1, 1, 2), 10, 3, 1), ((2, 1, 1), 6, 1, 70)]


@pytest.mark.parametrize("parts,N,Hw,nf,mixed,graph,form",
                         [g + (m, gr, "whole") for g in _GEOMS for m in (False, True)
                          for gr in (False, True)] +
                         [g + (False, False, "per_buffer") for g in _GEOMS])
def test_launches_use_the_copy_of_the_device_parity(parts, N, Hw, nf, mixed, graph, form):
    """Each rank's send buffers and peer receive buffers exist twice (the odd copy at
    _dbl(size)). Exchange k packs with the device word at k - 1 and add 1, as before the epoch
    close, then unpacks with the word at k and add 0, as after it: both select copy k&1, and the
    test routes the packed copy into the receiver's copy of the same parity in between. Every
    packed byte must land in the selected copy only, and every cell must come out right — with
    the launches eager, or captured once and replayed; 70 fields cut the plans into launch
    groups (each with its own slot map of the copies' offsets). form="per_buffer": the same
    through the per-buffer launches (ghx_exchange_split + ghx_exchange_pack_buffer /
    unpack_buffer, one launch per buffer), which must select the same copies."""
    import torch
    from ghex_amd import _ghx
    rs = _ranks(parts, N, Hw, nf)
    L = _ghx.lib()
    word = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = []
    for x in rs:
        co, bis = x["co"], x["bis"]
        plan = co.plan(bis)
        me = x["rank"]
        m = mixed and co.mixed(plan)
        send = [torch.full((2 * _dbl(b["size"]),), 255, dtype=torch.uint8, device="cuda")
                for b in plan.send]
        recv = []
        for b in plan.recv:
            j = next((i for i, s in enumerate(plan.send) if s["pair"] == b["pair"] and b["rank"] == me),
                     None)
            recv.append(send[j] if j is not None else
                        torch.full((2 * _dbl(b["size"]),), 255, dtype=torch.uint8, device="cuda"))
        # self messages keep one copy (their receive buffer IS the send buffer)
        soff = [_dbl(b["size"]) if b["rank"] != me else 0 for b in plan.send]
        roff = [_dbl(b["size"]) if b["rank"] != me else 0 for b in plan.recv]
        _set(plan, 0, word, 1, soff)
        _set(plan, 1, word, 0, roff)
        f = _ghx.ptr_array([bi.field.data_ptr() for bi in bis])
        st.append(dict(x, plan=plan, send=send, recv=recv, soff=soff, roff=roff, f=f, mixed=m,
                       sp=_ghx.ptr_array([t.data_ptr() for t in send]),
                       rp=_ghx.ptr_array([t.data_ptr() for t in recv])))

    if form == "per_buffer":
        for x in st:
            _ghx.call("ghx_exchange_split", x["plan"].h)

    def pack(s):
        for x in st:
            if form == "per_buffer":
                for i in range(len(x["send"])):
                    _ghx.check(L.ghx_exchange_pack_buffer(x["plan"].h, i, x["f"], len(x["bis"]),
                                                          x["sp"], len(x["send"]), s), "pack_buffer")
                continue
            fn = L.ghx_exchange_pack_self if x["mixed"] else L.ghx_exchange_pack
            _ghx.check(fn(x["plan"].h, x["f"], len(x["bis"]), x["sp"], len(x["send"]), s), "pack")

    def unpack(s):
        for x in st:
            if form == "per_buffer":
                for i in range(len(x["recv"])):
                    _ghx.check(L.ghx_exchange_unpack_buffer(x["plan"].h, i, x["f"], len(x["bis"]),
                                                            x["rp"], len(x["recv"]), s), "unpack_buffer")
                continue
            fn = L.ghx_exchange_unpack_peers if x["mixed"] else L.ghx_exchange_unpack
            _ghx.check(fn(x["plan"].h, x["f"], len(x["bis"]), x["rp"], len(x["recv"]), s), "unpack")

    def route(k):
        """the transport: each peer message's copy k&1 into the receiver's copy k&1"""
        for x in st:
            for i, b in enumerate(x["plan"].recv):
                if b["rank"] == x["rank"]:
                    continue
                src = st[b["rank"]]
                j = next(j for j, sb in enumerate(src["plan"].send)
                         if sb["pair"] == b["pair"] and sb["rank"] == x["rank"])
                o_s = src["soff"][j] * (k & 1)
                o_r = x["roff"][i] * (k & 1)
                x["recv"][i][o_r:o_r + b["size"]].copy_(src["send"][j][o_s:o_s + b["size"]])

    s = torch.cuda.current_stream().cuda_stream
    if graph:
        gp, gu = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            pack(side.cuda_stream)
            unpack(side.cuda_stream)
        torch.cuda.current_stream().wait_stream(side)
        with torch.cuda.graph(gp):
            pack(torch.cuda.current_stream().cuda_stream)
        with torch.cuda.graph(gu):
            unpack(torch.cuda.current_stream().cuda_stream)
    for k in (1, 2, 3, 4):
        for x in st:  # reset the halos and both copies of every buffer
            for base, a in zip(x["bases"], x["arrs"]):
                base.copy_(torch.from_numpy(a).cuda())
            for t in x["send"] + x["recv"]:
                t.fill_(255)
        word.fill_(k - 1)  # the pack of exchange k reads k - 1 (+1): copy k&1
        torch.cuda.synchronize()
        gp.replay() if graph else pack(s)
        torch.cuda.synchronize()
        for x in st:  # the packed bytes are in copy k&1 of every peer send buffer only
            for j, b in enumerate(x["plan"].send):
                if x["soff"][j]:
                    other = x["soff"][j] * ((k + 1) & 1)
                    assert bool((x["send"][j][other:other + b["size"]] == 255).all()), (k, j)
                    mine = x["soff"][j] * (k & 1)
                    assert not bool((x["send"][j][mine:mine + b["size"]] == 255).all()), (k, j)
        route(k)
        word.fill_(k)  # the close advanced the counter: the unpack of exchange k reads k
        torch.cuda.synchronize()
        gu.replay() if graph else unpack(s)
        torch.cuda.synchronize()
        for x in st:
            for f, (base, exp) in enumerate(zip(x["bases"], x["exps"])):
                assert np.array_equal(base.cpu().numpy(), exp), (k, x["rank"], f)
    for x in st:  # back to single buffers
        _set(x["plan"], 0, None, 0, [])
        _set(x["plan"], 1, None, 0, [])


def test_parity_offsets_are_checked():
    from ghex_amd import _ghx
    import torch
    rs = _ranks((2, 1, 1), 8, 1)
    plan = rs[0]["co"].plan(rs[0]["bis"])
    word = torch.zeros(1, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError, match="one offset per buffer"):
        _set(plan, 0, word, 1, [256] * (len(plan.send) + 1))
    with pytest.raises(RuntimeError, match="multiples of 256"):
        _set(plan, 0, word, 1, [100] * len(plan.send))
