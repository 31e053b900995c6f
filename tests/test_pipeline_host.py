"""Host logic of the per-peer pipeline (no GPU): the global round order every rank issues its
peers in, per-buffer plan bookkeeping through the C ABI, and the RCCL loader's error path."""
import ctypes
import itertools

import pytest

from ghex_amd.communication_object import peer_order, round_of


@pytest.mark.parametrize("world", range(1, 17))
def test_round_robin_schedule(world):
    """Every pair meets in exactly one round; no rank plays twice in a round; at most world-1
    rounds (world even) / world rounds (odd)."""
    rounds = {}
    for a, b in itertools.combinations(range(world), 2):
        r = round_of(a, b, world)
        assert r == round_of(b, a, world)
        rounds.setdefault(r, []).append((a, b))
    m = world + world % 2
    assert all(0 <= r < max(1, m - 1) for r in rounds)
    for r, pairs in rounds.items():
        seen = [x for p in pairs for x in p]
        assert len(seen) == len(set(seen)), (r, pairs)
    assert sum(len(p) for p in rounds.values()) == world * (world - 1) // 2


def test_peer_order_is_consistent_across_ranks():
    """If rank a issues b before c, no rank issues a pair of a later round first: the k-th peer
    of every rank plays in a non-decreasing sequence of rounds, the same round on both sides."""
    world = 8
    for me in range(world):
        order = peer_order(me, [p for p in range(world) if p != me], world)
        rs = [round_of(me, p, world) for p in order]
        assert rs == sorted(rs)
        for p in order:
            assert round_of(p, me, world) == round_of(me, p, world)


def _one_rank_exchange():
    from ghex_amd import _ghx
    from ghex_amd.communication_object import _ExchangePlan
    from tests import helpers as H
    from tests.test_host import _regular_pattern_abi
    N, Hw = 8, 2
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    pc = _regular_pattern_abi(ranks, gf, gl, (Hw,) * 6, (1, 1, 1), 0)
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
    it.pattern, it.local_index, it.kind, it.field = pc.handle, 0, 0, fd
    it.align, it.tag_offset = 8, 0
    plan = _ExchangePlan([it])
    plan._keep = pc
    return plan, _ghx


def test_split_and_buffer_index_errors():
    plan, _ghx = _one_rank_exchange()
    L = _ghx.lib()
    z = _ghx.ptr_array([1])
    # not split yet
    assert L.ghx_exchange_pack_buffer(plan.h, 0, z, 1, z, 1, None) == -1
    assert b"split" in L.ghx_last_error()
    _ghx.call("ghx_exchange_split", plan.h)
    assert L.ghx_exchange_pack_buffer(plan.h, 5, z, 1, z, 1, None) == -1
    assert b"out of range" in L.ghx_last_error()
    # in range, but no device in this container: a HIP error, not a crash
    assert L.ghx_exchange_unpack_buffer(plan.h, 0, z, 1, z, 1, None) == -2


def test_rccl_loader_reports_missing_library():
    from ghex_amd import _ghx
    L = _ghx.lib()
    assert L.ghx_rccl_open(b"/nonexistent/librccl.so") == -1
    assert b"dlopen" in L.ghx_last_error()
    buf = (ctypes.c_ubyte * 128)()
    # not loaded: refused with a message
    assert L.ghx_rccl_unique_id(buf) == -1
    assert b"RCCL not loaded" in L.ghx_last_error()


def _rank_plan(ranks, gf, gl, Hw, my_rank, n_fields=2):
    """Exchange plan of `my_rank` over every local domain (n_fields fields per domain, two
    pattern containers so that one pair of ranks carries messages of several tags)."""
    from ghex_amd import _ghx
    from ghex_amd.communication_object import _ExchangePlan
    from tests.test_host import _regular_pattern_abi
    pcs = [_regular_pattern_abi(ranks, gf, gl, (Hw,) * 6, (1, 1, 1), my_rank),
           _regular_pattern_abi(ranks, gf, gl, (1,) * 6, (1, 1, 1), my_rank)]
    d0 = ranks[0][0]
    E = [d0.last[d] - d0.first[d] + 1 + 2 * Hw for d in range(3)]
    items, off = [], 0
    for c, pc in enumerate(pcs):
        for li in range(len(ranks[my_rank])):
            for k in range(n_fields):
                fd = _ghx.FieldDesc()
                fd.dim, fd.elem_size = 3, 8 if k % 2 == 0 else 4
                for d in range(3):
                    fd.layout[d] = 2 - d
                    fd.offsets[d] = Hw
                    fd.extents[d] = E[d]
                es = fd.elem_size
                fd.byte_strides[0], fd.byte_strides[1] = es, es * E[0]
                fd.byte_strides[2] = es * E[0] * E[1]
                fd.num_components, fd.has_components = 1, 0
                it = _ghx.ExchangeItem()
                it.pattern, it.local_index, it.kind, it.field = pc.handle, li, 0, fd
                it.align, it.tag_offset = es, off
                items.append(it)
        off += pc.max_tag() + 1
    plan = _ExchangePlan(items)
    plan._keep = pcs
    return plan


@pytest.mark.parametrize("parts,doms", [((2, 1, 1), 2), ((2, 2, 1), 2), ((2, 2, 2), 1)])
def test_pair_messages_match_in_pipeline_order(parts, doms):
    """the per-peer pipeline issues the messages of one rank pair in (tag, domain
    pair) order on both ends (ghx_pipeline.cpp, ghx_pipeline_create: the `order` comparator;
    RCCL matches a pair's sends and receives by issue order). For every ordered pair of ranks,
    rank a's sends to b sorted that way must line up one to one with rank b's receives from a
    sorted that way: same domain pair, same tag, same size. Several domains per rank and two
    pattern containers give several messages (and tags) per pair."""
    from tests import helpers as H
    N, Hw = 6, 2
    ranks1, gf, gl = H.cube_domains(N, parts)
    # `doms` domains per rank along x: split each rank's box in x
    ranks = []
    from oracle import oracle as orc
    nid = 0
    for r, (d,) in enumerate(ranks1):
        w = N // doms
        sub = []
        for k in range(doms):
            f = (d.first[0] + k * w,) + d.first[1:]
            l = (d.first[0] + (k + 1) * w - 1,) + d.last[1:]
            sub.append(orc.RegularDomain(nid, f, l))
            nid += 1
        ranks.append(sub)
    world = len(ranks)
    plans = [_rank_plan(ranks, gf, gl, min(Hw, N // doms), r) for r in range(world)]
    key = lambda x: (x["tag"], x["pair"][0], x["pair"][1])  # noqa: E731
    checked = 0
    for a in range(world):
        for b in range(world):
            if a == b:
                continue
            sends = sorted((x for x in plans[a].send if x["rank"] == b), key=key)
            recvs = sorted((x for x in plans[b].recv if x["rank"] == a), key=key)
            assert len(sends) == len(recvs)
            for s, r in zip(sends, recvs):
                assert (s["tag"], s["pair"], s["size"]) == (r["tag"], r["pair"], r["size"])
                checked += 1
    assert checked > 0


def test_rccl_self_requires_device_buffers():
    """the host-staged pipeline keeps self messages on the device (recv aliases
    send), so routing them through RCCL (rccl_self) is refused there instead of unpacking a
    never-filled recv buffer."""
    import ghex_amd
    from ghex_amd.communication_object import CommunicationObject
    ctx = ghex_amd.make_context()
    with pytest.raises(ValueError, match="rccl_self"):
        CommunicationObject(ctx, staging="host", pipelined=True, rccl_self=True)
    CommunicationObject(ctx, staging=None, pipelined=True, rccl_self=True)


def test_failed_enqueue_leaves_object_usable(monkeypatch):
    """an exception while posting an exchange (an RCCL or gloo error) must not leave
    the object marked as having an exchange in flight."""
    import ghex_amd
    from ghex_amd.communication_object import CommunicationObject

    class BI:
        class field:
            device = None
    co = CommunicationObject(ghex_amd.make_context())
    monkeypatch.setattr(co, "plan", lambda bis: (_ for _ in ()).throw(RuntimeError("boom")))
    for _ in range(2):
        with pytest.raises(RuntimeError, match="boom"):
            co._start([BI], None)
        assert not co._valid
    # the same through the enqueue step itself
    monkeypatch.setattr(co, "plan", lambda bis: type("P", (), {"send": [], "recv": []})())
    monkeypatch.setattr(co, "buffers", lambda plan, dev: ([], []))
    monkeypatch.setattr(co, "_enqueue", lambda *a: (_ for _ in ()).throw(RuntimeError("rccl")))
    BI.field.data_ptr = staticmethod(lambda: 0)
    with pytest.raises(RuntimeError, match="rccl"):
        co._start([BI], None)
    assert not co._valid
