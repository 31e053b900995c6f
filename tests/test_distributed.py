"""Multi-process (gloo, CPU) tests of the N>1 exchange path: setup all-gather + libghx patterns
per rank, the exchange planner's buffer list (peers, tags, sizes), and the point-to-point router
(ghex_amd.communication_object.route) over a real process group.

The device pack/unpack is not available on CPU: the bytes of each message are produced and
consumed here by the ORACLE (test infrastructure), into buffers sized, tagged and addressed by
the product's planner, and moved by the product's router. The halo property of the reference's
tests must hold on every rank afterwards (test_regular_domain.cpp:739-800)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as orc
from tests import helpers as H


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, fn, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = [q.get() for _ in range(world)] if not q.empty() else []
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert len(res) == world and all(r == "ok" for r in res), res


def _entry(rank, world, port, fn, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
        q.put("ok")
    except Exception as e:  # report to the parent
        import traceback
        q.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


def _structured_exchange_worker(rank, world, parts, Hw, N):
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.communication_object import _ExchangePlan, route
    from ghex_amd.structured import regular as R
    ctx = ghex_amd.make_context()
    assert ctx.size() == world and ctx.rank() == rank
    ranks, gf, gl = H.cube_domains(N, parts)
    dom = ranks[rank][0]
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)),
                        [R.DomainDescriptor(dom.id, dom.first, dom.last)])
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))[rank][0]
    # field descriptor (host-side description only; the C planner needs no device)
    a, spec = H.linear_index_field(dom, N, Hw, gl)
    E = N + 2 * Hw
    fd = _ghx.FieldDesc()
    fd.dim, fd.elem_size = 3, 8
    for d in range(3):
        fd.layout[d] = 2 - d
        fd.offsets[d] = Hw
        fd.extents[d] = E
    fd.byte_strides[0], fd.byte_strides[1], fd.byte_strides[2] = 8, 8 * E, 8 * E * E
    fd.num_components, fd.has_components = 1, 0
    it = _ghx.ExchangeItem()
    it.pattern, it.local_index, it.kind, it.field, it.align, it.tag_offset = \
        pc.handle, 0, 0, fd, 8, 0
    plan = _ExchangePlan([it])
    osend = orc.plan_buffers([(0, dom.id, opat, 8, 8, 1, 0)], receive=False)
    orecv = orc.plan_buffers([(0, dom.id, opat, 8, 8, 1, 0)], receive=True)
    assert [(b["pair"], b["rank"], b["tag"], b["size"]) for b in plan.send] == \
        [(k, b.rank, b.tag, b.size) for k, b in osend.items()]
    assert [(b["pair"], b["rank"], b["tag"], b["size"]) for b in plan.recv] == \
        [(k, b.rank, b.tag, b.size) for k, b in orecv.items()]
    # pack (oracle bytes) into product-planned buffers, route with the product router
    send_t = []
    for b in plan.send:
        buf = np.zeros(b["size"], np.uint8)
        ob = osend[b["pair"]]
        for pf in ob.fields:
            orc.structured_pack(spec, buf, pf.boxes, pf.offset)
        send_t.append(torch.from_numpy(buf))
    recv_t = [torch.zeros(b["size"], dtype=torch.uint8) for b in plan.recv]
    sends = [(b["rank"], b["tag"], t) for b, t in zip(plan.send, send_t) if b["rank"] != rank]
    recvs = [(b["rank"], b["tag"], t) for b, t in zip(plan.recv, recv_t) if b["rank"] != rank]
    for w in route(ctx, sends, recvs):
        w.wait()
    for i, b in enumerate(plan.recv):
        if b["rank"] == rank:  # self message: read the matching send buffer
            j = next(j for j, s in enumerate(plan.send) if s["pair"] == b["pair"])
            recv_t[i] = send_t[j]
        for pf in orecv[b["pair"]].fields:
            orc.structured_unpack(spec, recv_t[i].numpy(), pf.boxes, pf.offset)
    np.testing.assert_array_equal(a, H.expected_linear_halo(a, dom, N, Hw, gl))


@pytest.mark.parametrize("world,parts", [(2, (2, 1, 1)), (4, (2, 2, 1))])
@pytest.mark.parametrize("Hw", [1, 2])
def test_structured_exchange_gloo(world, parts, Hw):
    _run(world, _structured_exchange_worker, parts, Hw, 6)


def test_config1_128cube_two_ranks_gloo():
    """BASELINE config 1 at its full size (the reference's CPU-runnable case,
    benchmarks/simple_comm_test_halo_exchange_3D_generic_full.cpp): 128^3 fp64 per rank, H=1,
    periodic, (2,1,1) over 2 gloo ranks — product planning and routing, oracle bytes, every cell."""
    _run(2, _structured_exchange_worker, (2, 1, 1), 1, 128)


def _unstructured_worker(rank, world, case):
    import ghex_amd
    from ghex_amd.communication_object import route
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    ctx = ghex_amd.make_context()
    d = case["domains"][str(rank)]
    pc = make_pattern(ctx, HaloGenerator(), [DomainDescriptor(rank, d["gids"], d["halo_lids"])])
    # the reference's known-answer send/recv tables (unstructured_test_case.hpp:217-343)
    sends = {str(rid): lids for rid, rr, tag, lids in pc.send_halos(0)}
    recvs = {str(rid): lids for rid, rr, tag, lids in pc.recv_halos(0)}
    assert sends == case["send_maps"][str(rank)], sends
    assert recvs == case["recv_maps"][str(rank)], recvs
    # move the values: buf = field[lids] (levels=1), route, scatter
    gids = d["gids"]
    inner_lids = [l for l in range(len(gids)) if l not in set(d["halo_lids"])]
    f = np.full(len(gids), -1.0)
    for l in inner_lids:
        f[l] = rank * 10000 + gids[l] * 100
    st, rt = [], []
    for rid, rr, tag, lids in pc.send_halos(0):
        st.append((rr, tag, torch.from_numpy(f[lids].copy())))
    for rid, rr, tag, lids in pc.recv_halos(0):
        rt.append((rr, tag, torch.zeros(len(lids), dtype=torch.float64), lids, rid))
    for w in route(ctx, st, [(r, t, b) for r, t, b, _, _ in rt]):
        w.wait()
    for r, t, b, lids, rid in rt:
        f[lids] = b.numpy()
        for l in lids:
            assert f[l] == rid * 10000 + gids[l] * 100


def test_unstructured_known_answer_gloo(golden_dir):
    import json
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    _run(4, _unstructured_worker, case)


def _config5_worker(rank, world, cells):
    """BASELINE config 5's domains (gids rank*10^7 + i, 5 % halo from the other
    ranks, mt19937_64 seed 20260715, permuted storage) through the product's make_pattern over
    gloo; then every halo value moved with the pattern's lid lists and checked."""
    import time

    import ghex_amd
    from ghex_amd.communication_object import route
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    from tools import config5 as C5
    gids, outer = C5.generate(rank, world, cells)
    ctx = ghex_amd.make_context()
    dist.barrier()
    t0 = time.perf_counter()
    dd = DomainDescriptor(rank, gids, outer)
    pc = make_pattern(ctx, HaloGenerator(), [dd])
    t_setup = time.perf_counter() - t0
    # peak RSS of this process image (VmHWM: getrusage's ru_maxrss would also count the
    # pytest parent's pages this spawned child held before its exec)
    rss_gb = next(int(l.split()[1]) for l in open("/proc/self/status")
                  if l.startswith("VmHWM:")) / 2 ** 20
    f = gids.astype(np.float64) * 100.0
    f[outer] = -1.0
    st = [(rr, tag, torch.from_numpy(f[lids])) for rid, rr, tag, lids in pc.lid_arrays(0, 0)]
    rt = [(rr, tag, torch.empty(len(lids), dtype=torch.float64), lids)
          for rid, rr, tag, lids in pc.lid_arrays(0, 1)]
    assert sum(len(x[3]) for x in rt) == len(outer)  # every outer cell is received once
    for w in route(ctx, st, [(r, t, b) for r, t, b, _ in rt]):
        w.wait()
    for _, _, b, lids in rt:
        f[lids] = b.numpy()
    assert np.array_equal(f, gids.astype(np.float64) * 100.0)
    print(f"rank {rank}: make_pattern {t_setup:.2f} s, peak RSS {rss_gb:.2f} GB", flush=True)
    assert t_setup < 20.0, t_setup
    assert rss_gb < 2.0, rss_gb


def test_config5_pattern_full_size_gloo_two_ranks():
    """make_pattern<unstructured> at BASELINE config 5's size per rank (10M cells, 500k halo
    cells) over 2 gloo ranks: under 20 s and 2 GB peak RSS per rank (only reduced halos travel),
    and the exchanged halo values are exact."""
    _run(2, _config5_worker, 10_000_000)


def test_config5_pattern_four_ranks_gloo():
    _run(4, _config5_worker, 200_000)


def _multi_domain_worker(rank, world, case, grouping):
    import ghex_amd
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    d = case["domains"]
    mine = [DomainDescriptor(i, d[str(i)]["gids"], d[str(i)]["halo_lids"]) for i in grouping[rank]]
    pc = make_pattern(ghex_amd.make_context(), HaloGenerator(), mine)
    odoms = [[orc.UnstructuredDomain(i, d[str(i)]["gids"], d[str(i)]["halo_lids"]) for i in g]
             for g in grouping]
    opats = orc.unstructured_make_pattern(odoms)
    for li in range(len(grouping[rank])):
        for direction, key in ((0, "send"), (1, "recv")):
            got = [(rr, tag, rid, lids) for rid, rr, tag, lids in pc.halos(li, direction)]
            exp = [(rr, tag, rid, lids) for (rr, tag), (rid, lids) in opats[rank][li][key].items()]
            assert got == exp, (li, key, got, exp)


def test_unstructured_multi_domain_ranks_gloo(golden_dir):
    """Two gloo ranks with two domains each (the known-answer case): the setup's
    point-to-point gid lists include messages a rank sends itself (between its two domains),
    which Context.exchange_arrays keeps local; patterns equal the oracle's."""
    import json
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    _run(2, _multi_domain_worker, case, [[0, 1], [2, 3]])


def _certificate_worker(rank, world):
    import types

    import torch

    import bench
    plan = types.SimpleNamespace(
        send=[{"rank": 1 - rank, "size": 100}, {"rank": rank, "size": 7},
              {"rank": 1 - rank, "size": 20}],
        recv=[{"rank": 1 - rank, "size": 60}, {"rank": rank, "size": 7}])
    cert = bench.transport_certificate(torch, dist, torch.device("cuda", 0), plan, rank, world,
                                       "gloo")
    assert cert["world_size"] == 2 and cert["backend"] == "gloo" and cert["rccl_ranks"] is None
    assert cert["devices"] == [0, 0]
    peer = cert["peers"][str(1 - rank)]
    assert peer["bytes_sent_per_step"] == 120 and peer["bytes_received_per_step"] == 60
    assert peer.get("same_device") is True  # both ranks name device 0
    assert cert["certified"] is False and "gloo" in cert["why_not"]
    assert str(rank) not in cert["peers"]  # self messages are not a transport


def test_transport_certificate_gloo_two_ranks():
    """bench.transport_certificate over gloo on CPU: the world size and backend,
    per-peer bytes from the plan's buffers (self messages excluded), and a line that is NOT
    certified as an RCCL N-GPU run (gloo, shared device). The RCCL rank count is exercised by
    the driver's N>1 runs."""
    _run(2, _certificate_worker)


def _collision_worker(rank, world):
    import ghex_amd
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    ranks = [[(1, list(range(0, 10)), []), (2, list(range(10, 20)), [])],
             [(8, list(range(20, 30)) + [10], [10]), (0, list(range(30, 40)) + [11], [10])]]
    ctx = ghex_amd.make_context()
    try:
        make_pattern(ctx, HaloGenerator(), [DomainDescriptor(i, g, o) for i, g, o in ranks[rank]])
    except Exception as e:
        assert "share tag 8" in str(e), e
        return
    raise AssertionError("make_pattern returned despite a tag collision")


def test_unstructured_setup_error_reaches_every_rank_gloo():
    """a rank whose make_pattern<unstructured> fails mid-setup (here: a tag
    collision found while resolving the reduced halos of the ring) must not leave its peers
    waiting in the ring or a later collective; over gloo both ranks raise (the error names the
    collision on the rank that saw it and on its peer)."""
    _run(2, _collision_worker)
