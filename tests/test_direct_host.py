"""CPU: the direct exchange's message matching (ghex_amd.communication_object.direct_matches) —
which receiver buffer each peer send buffer of a plan is packed into. Messages of one rank pair
match k-th to k-th in tag order on both sides, as route() matches them for RCCL/gloo; counts,
tags and sizes must agree. (The exchange itself runs in tests/test_gpu_multiproc.py.)"""
import pytest

from ghex_amd.communication_object import direct_matches


def _send(*msgs):
    return [dict(rank=r, tag=t, size=s, pair=(0, 0)) for r, t, s in msgs]


def test_matches_in_tag_order_and_skips_self_and_others():
    send = _send((1, 5, 16), (0, 9, 64), (1, 3, 32), (2, 5, 8))
    recv_of = {1: [(0, 3, 32, "b3"), (2, 5, 8, "x"), (0, 5, 16, "b5")],  # rank 2's entry: not ours
               2: [(0, 5, 8, "c5")]}
    got = {i: e[3] for i, e in direct_matches(0, send, recv_of)}
    assert got == {0: "b5", 2: "b3", 3: "c5"}  # index 1 is a self message: never exported


def test_equal_tags_keep_plan_order():
    """Two domain pairs between the same ranks with the same tag: the plan orders of sender and
    receiver decide, on both sides stably (the same assumption route() makes)."""
    send = _send((1, 7, 8), (1, 7, 24))
    recv_of = {1: [(0, 7, 8, "first"), (0, 7, 24, "second")]}
    assert [(i, e[3]) for i, e in direct_matches(0, send, recv_of)] == [(0, "first"), (1, "second")]


@pytest.mark.parametrize("recv,msg", [([(0, 7, 8, "a")], "expects 1 messages"),
                                      ([(0, 7, 8, "a"), (0, 8, 16, "b")], "mismatch"),
                                      ([(0, 7, 9, "a"), (0, 7, 24, "b")], "mismatch")])
def test_disagreements_raise(recv, msg):
    with pytest.raises(RuntimeError, match=msg):
        direct_matches(0, _send((1, 7, 8), (1, 7, 24)), {1: recv})


def test_no_peers_no_matches():
    assert direct_matches(3, _send((3, 1, 8), (3, 2, 8)), {}) == []


def test_epochs_group_is_node_local_beyond_64_ranks():
    """the epochs' flag block is per host and indexed by node-local position, so a
    job of 9 hosts x 8 ranks (72 > the 64-rank block limit) maps every rank to [0, 8)."""
    from ghex_amd.bulk_communication_object import node_local_group
    hosts = [f"node{r // 8}" for r in range(72)]
    for me in range(72):
        local, idx = node_local_group(hosts, me)
        assert local == list(range(8 * (me // 8), 8 * (me // 8) + 8))
        assert idx == me % 8 and len(local) <= 64
    # hosts interleaved by rank: positions follow ascending global rank on each host
    hosts = [f"h{r % 3}" for r in range(10)]
    assert node_local_group(hosts, 7) == ([1, 4, 7], 2)
    assert node_local_group(hosts, 9) == ([0, 3, 6, 9], 3)


def test_epoch_error_codes_decode():
    """ghx_epochs_status codes as the Python objects report them (the host side of the device
    epochs; the codes themselves are set by ghx_epochs.hip)."""
    import ctypes
    from ghex_amd import bulk_communication_object as B
    from ghex_amd import _ghx
    orig = _ghx.call

    def fake(code):
        def call(name, ep, err, epoch):
            assert name == "ghx_epochs_status"
            err._obj.value = code
        return call
    hosts = ["a", "b", "a", "a"]
    try:
        for code, text in ((0, None), (1, "open phase timed out"), (2, "close phase timed out"),
                           (3, "every XCD"), (4 | (1 << 8), "rank 2 failed an epoch wait")):
            _ghx.call = fake(code)
            got = B.epochs_error(ctypes.c_void_p(1), hosts, 0)
            assert (got is None) if text is None else (text in got), (code, got)
    finally:
        _ghx.call = orig
