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
