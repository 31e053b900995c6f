"""Plan pairings at the BASELINE sizes (CPU: host-side planning only, no GPU needed).

A fused launch pairs a primary plan with a companion plan segment by segment: the zero-copy put
(source pack plan + target unpack plan, ghx_put_create), the fused self exchange (pack + unpack
of the same buffers, ghx_exchange_self_fusable) and the mixed self/peer pack
(ghx_exchange_mixed). Short-row tiles are sized per field from that field's short-row count
(ghx_plan.cpp build_tiles), and the two sides of a pairing count different fields' rows: one
source field against one target field per peer, or a field's self messages against all of its
messages. Round 5 compared the tilings and so refused every 512^3 put with more than one peer
(ghx_put_create "source and target iteration spaces do not describe the same
message bytes"). The suite's small fields all sit at the 512-row minimum, where the tilings agree;
these cases are sized so that the short-row rule leaves its minimum (>= 131k short rows per
field: N=256 H=2 and up), as every planner change must be re-tested."""
import ctypes
from types import SimpleNamespace

import pytest

from tests import helpers as H


def _desc(N, Hw, elem=8):
    from ghex_amd import _ghx
    E = N + 2 * Hw
    d = _ghx.FieldDesc()
    d.dim, d.elem_size = 3, elem
    st = (elem, elem * E, elem * E * E)  # x fastest: layout map (2, 1, 0)
    for k in range(3):
        d.layout[k] = 2 - k
        d.byte_strides[k] = st[k]
        d.offsets[k] = Hw
        d.extents[k] = E
    d.num_components, d.has_components = 1, 0
    return d


def _patterns(parts, N, Hw):
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    out = []
    for r in range(nr):
        dd = R.DomainDescriptor(ranks[r][0].id, ranks[r][0].first, ranks[r][0].last)
        out.append(R.make_pattern(FakeContext(r, nr, table),
                                  R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd]))
    return out


def _short_rows(pc, direction, N, Hw):
    """Short-row count (16-B-or-shorter x rows) of one field's halos in one direction."""
    halos = pc.send_halos(0) if direction == 0 else pc.recv_halos(0)
    n = 0
    for _, _, _, spaces in halos:
        for sp in spaces:
            lf, ll = sp[0], sp[1]
            if ll[0] - lf[0] + 1 < N:  # rows shorter than the domain: the x-face pieces
                n += (ll[1] - lf[1] + 1) * (ll[2] - lf[2] + 1)
    return n


CASES = [((2, 2, 1), 256, 2), ((2, 2, 1), 512, 2), ((2, 2, 2), 512, 2), ((2, 2, 2), 512, 3),
         ((2, 1, 1), 512, 1), ((2, 2, 2), 384, 1)]


@pytest.mark.parametrize("parts,N,Hw", CASES)
def test_put_plans_pair_at_baseline_sizes(parts, N, Hw):
    """Every rank's put plans — built by the bulk object's own message / chunk / entry code —
    are accepted by ghx_put_create and carry exactly the bytes of its node-local send halos."""
    from ghex_amd import _ghx
    from ghex_amd.bulk_communication_object import put_chunks, put_entries, put_messages
    L = _ghx.lib()
    pcs = _patterns(parts, N, Hw)
    desc = _desc(N, Hw)
    assert _short_rows(pcs[0], 0, N, Hw) >= 131072  # beyond the short-row rule's minimum
    allr = []
    for pc in pcs:
        recv = [(rid, tag, [(sp[0], sp[1]) for sp in spaces])
                for rid, rr, tag, spaces in pc.recv_halos(0)]
        allr.append({"host": "h", "fields": [{"domain": pc.domains[0].domain_id(), "j": 0,
                                              "desc": bytes(desc), "recv": recv}]})
    local = list(range(len(pcs)))
    for me, pc in enumerate(pcs):
        bi = SimpleNamespace(pattern_container=pc, local_index=0)
        msgs = put_messages([bi], [(pc.domains[0].domain_id(), 0)], allr, local)
        want = sum(8 * (sp[1][0] - sp[0][0] + 1) * (sp[1][1] - sp[0][1] + 1) *
                   (sp[1][2] - sp[0][2] + 1) for _, _, _, sps in pc.send_halos(0) for sp in sps)
        got = 0
        for chunk, srcs, dsts in put_chunks(msgs):
            src, dst, keep = put_entries(chunk, srcs, dsts, [desc], allr)
            h = ctypes.c_void_p()
            rc = L.ghx_put_create(src, len(chunk), dst, len(chunk), ctypes.byref(h))
            assert rc == 0, (me, L.ghx_last_error())
            nb = ctypes.c_uint64()
            assert L.ghx_put_info(h, ctypes.byref(nb), None) == 0
            got += nb.value
            assert L.ghx_put_destroy(h) == 0
        assert got == want


def _exchange(pc, desc):
    from ghex_amd import _ghx
    it = _ghx.ExchangeItem()
    it.pattern = pc.handle
    it.local_index = 0
    it.kind = 0
    it.field = desc
    it.align = desc.elem_size
    it.tag_offset = 0
    arr = (_ghx.ExchangeItem * 1)(it)
    h = ctypes.c_void_p()
    _ghx.call("ghx_exchange_create", arr, 1, ctypes.byref(h))
    return h


def _flag(name, h):
    from ghex_amd import _ghx
    f = ctypes.c_int32()
    _ghx.call(name, h, ctypes.byref(f))
    return f.value


@pytest.mark.parametrize("N,Hw", [(256, 2), (384, 1), (512, 1), (512, 2), (512, 3), (640, 2)])
def test_self_exchange_fuses_at_every_size(N, Hw):
    """One rank, periodic: every message is a self message, so the exchange is fusable (k_self)
    whatever tile sizes the two directions' plans chose."""
    from ghex_amd import _ghx
    pc, = _patterns((1, 1, 1), N, Hw)
    h = _exchange(pc, _desc(N, Hw))
    try:
        assert _flag("ghx_exchange_self_fusable", h) == 1
    finally:
        _ghx.lib().ghx_exchange_destroy(h)


@pytest.mark.parametrize("parts,N,Hw", [((1, 1, 2), 512, 2), ((1, 2, 2), 512, 2),
                                        ((1, 1, 2), 256, 2), ((1, 2, 1), 384, 1),
                                        ((1, 2, 2), 640, 3)])
def test_mixed_pack_self_kept_at_every_size(parts, N, Hw):
    """Decompositions whose x wrap stays on the rank (self messages with short x rows next to
    peer messages) take the mixed pack-self launch on every rank: the companion plan of the self
    messages alone counts fewer short rows than the pack plan of all messages, and that must not
    drop the fused form."""
    from ghex_amd import _ghx
    for pc in _patterns(parts, N, Hw):
        h = _exchange(pc, _desc(N, Hw))
        try:
            assert _flag("ghx_exchange_mixed", h) == 1, (parts, N, Hw)
        finally:
            _ghx.lib().ghx_exchange_destroy(h)
