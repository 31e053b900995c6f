"""GPU parity against the committed checksum manifest (tests/golden/hash_manifest.json, made by
tests/golden/make_hash_manifest.py from the oracle): every packed message and every field after
unpack, FNV-1a 64, for 109 small cases (2 cube sizes x 3 halos x 6 layout maps x 3
decompositions + asymmetric halos) and the full-size cases (512^3 fp64 H=1/2/3 on one rank —
BASELINE config 2 — 2x2x2 ranks of 64^3, and 2x2x2 ranks of 512^3 H=2 — BASELINE config 3). Multi-rank cases are emulated in one process
(tests/gpu_util.emulated_exchange); single-rank cases run the communication object's own
exchange(), i.e. the fused self-exchange kernel the bench measures."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests import helpers as H

pytestmark = pytest.mark.gpu

MANIFEST = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "hash_manifest.json")))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def _parse(name):
    parts = dict((p[0], p[1:]) for p in name.split("_"))
    halos = tuple(int(c) for c in parts["A"]) if "A" in parts else None
    return (int(parts["N"]), int(parts["H"]), tuple(int(c) for c in parts["L"]),
            tuple(int(c) for c in parts["P"]), halos)


def _device_linear_field(dom, N, Hw, gl):
    """helpers.linear_index_field for layout (2,1,0), built on the device (full sizes): owned cell
    = global linear index x + Gx*(y + Gy*z), halos -1; memory order (z, y, x)."""
    import torch
    E = N + 2 * Hw
    G = [g + 1 for g in gl]
    base = torch.full((E, E, E), -1.0, dtype=torch.float64, device="cuda")
    ar = [torch.arange(N, device="cuda", dtype=torch.float64) + dom.first[d] for d in range(3)]
    base[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = (
        ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)))
    return base, base.permute(2, 1, 0)


def gpu_case(N, Hw, layout, parts, halos=None):
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field, emulated_exchange
    halos = tuple(halos) if halos is not None else (Hw,) * 6
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    E = N + 2 * Hw
    cos, bis, bases = [], [], []
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        dd = R.DomainDescriptor(ranks[r][0].id, ranks[r][0].first, ranks[r][0].last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, halos, (1, 1, 1)), [dd])
        if N >= 256 and layout == (2, 1, 0):
            base, logical = _device_linear_field(ranks[r][0], N, Hw, gl)
        else:
            a, _ = H.linear_index_field(ranks[r][0], N, Hw, gl, layout=layout)
            base, logical = device_field(a, layout)
            del a
        fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
        cos.append(R.make_communication_object(ctx))
        bis.append([pc(fd)])
        bases.append(base)
    if nr == 1:
        cos[0].exchange(bis[0]).wait()
        plan = cos[0].plan(bis[0])
        plans, bufs = [plan], [cos[0].buffers(plan, bases[0].device)]
    else:
        plans, bufs = emulated_exchange(cos, bis)
    torch.cuda.synchronize()
    msgs = {}
    for r in range(nr):
        for i, x in enumerate(plans[r].send):
            b = bufs[r][0][i][:x["size"]].cpu().numpy()
            msgs[f"{r}:{x['pair'][0]},{x['pair'][1]}"] = [int(x["size"]),
                                                          f"{orc.fnv1a64(b):016x}"]
    fields = [f"{orc.fnv1a64(b.cpu().numpy()):016x}" for b in bases]
    return {"messages": msgs, "fields": fields}


@pytest.mark.parametrize("name", sorted(MANIFEST["small"]))
def test_small_case_matches_manifest(name):
    got = gpu_case(*_parse(name))
    exp = MANIFEST["small"][name]
    assert got["messages"] == exp["messages"]
    assert got["fields"] == exp["fields"]


@pytest.mark.parametrize("name", sorted(MANIFEST["full"]))
def test_full_case_matches_manifest(name):
    import torch
    got = gpu_case(*_parse(name))
    exp = MANIFEST["full"][name]
    assert got["messages"] == exp["messages"]
    assert got["fields"] == exp["fields"]
    torch.cuda.empty_cache()


C4_TYPES = ["float64", "float32", "float64", "float32", "float64"]


def _device_c4_field(dom, N, Hw, gl, dtype, add):
    """helpers.linear_index_field(dtype, add) built on the device: owned = global linear index +
    add (computed in f64, rounded once to dtype), halos -1; memory order (z, y, x)."""
    import torch
    E = N + 2 * Hw
    G = [g + 1 for g in gl]
    T = getattr(torch, dtype)
    base = torch.full((E, E, E), -1, dtype=T, device="cuda")
    ar = [torch.arange(N, device="cuda", dtype=torch.float64) + dom.first[d] for d in range(3)]
    base[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = (
        ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)) + add
    ).to(T)
    return base, base.permute(2, 1, 0)


@pytest.mark.parametrize("name", sorted(MANIFEST.get("config4", {})))
def test_config4_five_fields_matches_manifest(name):
    """BASELINE config 4 (five fields [f64, f32, f64, f32, f64], H=3, 2x2x2, ONE exchange per
    rank): every packed message (pads zero on both sides) and every field after unpack."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, emulated_exchange
    p = dict((q[0], q[1:]) for q in name.split("_")[1:])
    N, Hw, parts = int(p["N"]), int(p["H"]), tuple(int(c) for c in p["P"])
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    cos, bis, bases = [], [], []
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        dd = R.DomainDescriptor(ranks[r][0].id, ranks[r][0].first, ranks[r][0].last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)), [dd])
        bl = []
        for k, T in enumerate(C4_TYPES):
            base, logical = _device_c4_field(ranks[r][0], N, Hw, gl, T, k)
            bl.append(pc(R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)))
            bases.append(base)
        co = R.make_communication_object(ctx)
        for t in co.buffers(co.plan(bl), torch.device("cuda", 0))[0]:
            t.zero_()  # pad bytes are never written by the pack: zero, as in the oracle
        cos.append(co)
        bis.append(bl)
    plans, bufs = emulated_exchange(cos, bis)
    torch.cuda.synchronize()
    exp = MANIFEST["config4"][name]
    msgs = {}
    for r in range(nr):
        for i, x in enumerate(plans[r].send):
            b = bufs[r][0][i][:x["size"]].cpu().numpy()
            msgs[f"{r}:{x['pair'][0]},{x['pair'][1]}"] = [int(x["size"]),
                                                          f"{orc.fnv1a64(b):016x}"]
    assert msgs == exp["messages"]
    assert [f"{orc.fnv1a64(b.cpu().numpy()):016x}" for b in bases] == exp["fields"]
    del bases
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", [n for n in sorted(MANIFEST["full"]) if n.endswith("_P111")])
def test_full_single_domain_two_launch_matches_manifest(name):
    """The headline's own kernels at the headline size: the single-domain
    512^3 plan run as the bench times it — ONE k_copy pack launch (ghx_exchange_pack), then ONE
    k_copy unpack launch (ghx_exchange_unpack), not the fused k_self of exchange() — on a field
    whose halos are -1 and a buffer preset to 0xFF. The packed message and the whole field after
    the unpack must hash as the oracle's (reference path replaced:
    include/ghex/structured/pack_kernels.hpp:161-248)."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext
    N, Hw, layout, parts, _ = _parse(name)
    ranks, gf, gl = H.cube_domains(N, parts)
    table = {0: [(d.id, d.first, d.last) for d in ranks[0]]}
    ctx = FakeContext(0, 1, table)
    dd = R.DomainDescriptor(ranks[0][0].id, ranks[0][0].first, ranks[0][0].last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)), [dd])
    base, logical = _device_linear_field(ranks[0][0], N, Hw, gl)
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
    co = R.make_communication_object(ctx)
    bis = [pc(fd)]
    plan = co.plan(bis)
    send, recv = co.buffers(plan, base.device)
    for t in send + recv:
        t.fill_(255)
    co.pack_only(bis)
    torch.cuda.synchronize()
    exp = MANIFEST["full"][name]
    (x,) = plan.send
    b = send[0][:x["size"]].cpu().numpy()
    assert {f"0:{x['pair'][0]},{x['pair'][1]}": [int(x["size"]), f"{orc.fnv1a64(b):016x}"]} \
        == exp["messages"]
    # the pack read only interior cells: the halos are still -1 here
    E = N + 2 * Hw
    assert bool((base[:Hw] == -1).all()) and bool((base[:, :, E - Hw:] == -1).all())
    del b
    co.unpack_only(bis)
    torch.cuda.synchronize()
    assert [f"{orc.fnv1a64(base.cpu().numpy()):016x}"] == exp["fields"]
    del base, logical, send, recv
    torch.cuda.empty_cache()
