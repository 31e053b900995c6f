"""CPU tests of the product's host side (no GPU): the C-ABI library loads and exports every
declared symbol; patterns and exchange buffer plans computed by libghx equal the oracle's
(which is pinned to the reference, tests/test_oracle.py)."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from oracle import oracle as orc
from tests import helpers as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ghx():
    from ghex_amd import _ghx
    return _ghx


def test_library_exports_every_declared_symbol(ghx):
    L = ghx.lib()
    with open(os.path.join(ROOT, "include", "ghx.h")) as fh:
        decl = set(re.findall(r"^(?:int|const char\*)\s+(ghx_\w+)\s*\(", fh.read(), re.M))
    assert len(decl) >= 25
    missing = [n for n in decl if not hasattr(L, n)]
    assert not missing, missing
    assert set(ghx.EXPORTED) == decl, set(ghx.EXPORTED) ^ decl
    assert b"gfx950" in L.ghx_version()


def test_library_is_built_for_gfx950():
    so = os.path.join(ROOT, "ghex_amd", "lib", "libghx.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data
    assert b"oracle" not in data.lower().replace(b"ghex_amd", b"")  # product never links the oracle


def test_errors_are_reported_not_thrown(ghx):
    h = ctypes.c_void_p()
    rc = ghx.lib().ghx_regular_pattern_create(7, None, 0, None, None, None, None, 0,
                                              ctypes.byref(h))
    assert rc == -1
    assert b"null" in ghx.lib().ghx_last_error() or b"dim" in ghx.lib().ghx_last_error()


@pytest.mark.parametrize("key,good,bad", [("fast_addr", [0, 1], [-1, 2]),
                                           ("pack_tile_rows", [0, 64, 65536], [-1, 63, 65537]),
                                           ("unpack_tile_rows", [0, 512], [32, 1 << 20]),
                                           ("tile_records", [0, 1], [2])])
def test_tuning_knobs_validate_their_range(ghx, key, good, bad):
    """ghx_tune accepts each knob's documented range and refuses the rest with a message naming
    the knob (unknown keys too); `reset` restores the defaults."""
    L = ghx.lib()
    try:
        for v in good:
            assert L.ghx_tune(key.encode(), v) == 0, (key, v, L.ghx_last_error())
        for v in bad:
            assert L.ghx_tune(key.encode(), v) != 0, (key, v)
            assert key.encode() in L.ghx_last_error()
        assert L.ghx_tune(b"no_such_knob", 1) != 0
    finally:
        assert L.ghx_tune(b"reset", 0) == 0


def test_halo_boxes_via_abi_match_reference(golden_dir):
    from ghex_amd.structured.regular import DomainDescriptor, HaloGenerator
    with open(os.path.join(golden_dir, "ref_halo_boxes.json")) as fh:
        cfgs = json.load(fh)["configs"]
    for c in cfgs:
        hg = HaloGenerator(c["gfirst"], c["glast"], c["halos"], c["periodic"])
        got = hg(DomainDescriptor(0, c["dom"][0], c["dom"][1]))
        exp = c["boxes"]
        assert [list(a) + list(b) + list(g) + list(h) for a, b, g, h in got] == exp


def _regular_pattern_abi(ranks, gf, gl, halos, periodic, my_rank):
    from ghex_amd.structured.regular import DomainDescriptor, HaloGenerator, make_pattern

    class FakeCtx:
        def __init__(self, r, n):
            self.r, self.n = r, n

        def rank(self):
            return self.r

        def size(self):
            return self.n

        def all_gather_object(self, obj):
            return [[(d.id, d.first, d.last) for d in doms] for doms in ranks]

    hg = HaloGenerator(gf, gl, halos, periodic)
    mine = [DomainDescriptor(d.id, d.first, d.last) for d in ranks[my_rank]]
    return make_pattern(FakeCtx(my_rank, len(ranks)), hg, mine)


def _cmp_regular(pc, opats, D):
    assert len(pc) == len(opats)
    for li, op in enumerate(opats):
        for direction, omap in ((0, op.send_items()), (1, op.recv_items())):
            got = pc.halos(li, direction)
            assert len(got) == len(omap)
            for (rid, rr, tag, spaces), ((oid, otag), (orank, lst)) in zip(got, omap):
                assert (rid, tag, rr) == (oid, otag, orank)
                assert [(a, b, c, d) for a, b, c, d in spaces] == \
                    [(isp.lf, isp.ll, isp.gf, isp.gl) for isp in lst]
        assert pc.max_tag() == op.max_tag


@pytest.mark.parametrize("halos", [H.HALOS_1, H.HALOS_2])
def test_regular_pattern_reference_geometry(halos):
    ranks, gf, gl = H.regular_test_domains(4)
    opat = orc.regular_make_pattern(ranks, gf, gl, halos, (1, 1, 1))
    for r in range(4):
        pc = _regular_pattern_abi(ranks, gf, gl, halos, (1, 1, 1), r)
        _cmp_regular(pc, opat[r], 3)


@pytest.mark.parametrize("parts", [(1, 1, 1), (2, 1, 1), (2, 2, 1), (2, 2, 2), (3, 2, 1)])
@pytest.mark.parametrize("halos,periodic", [((1,) * 6, (1, 1, 1)), ((2, 1, 1, 2, 0, 3), (1, 1, 1)),
                                            ((2,) * 6, (0, 1, 0))])
def test_regular_pattern_cubes(parts, halos, periodic):
    ranks, gf, gl = H.cube_domains(6, parts)
    opat = orc.regular_make_pattern(ranks, gf, gl, halos, periodic)
    for r in range(len(ranks)):
        pc = _regular_pattern_abi(ranks, gf, gl, halos, periodic, r)
        _cmp_regular(pc, opat[r], 3)


def _unstructured_abi(doms_ranks, halo_gids):
    """Every rank's make_pattern<unstructured>, run as threads of this process (LoopbackWorld):
    each rank passes only its own domains; returns the pattern containers in rank order."""
    from ghex_amd.context import LoopbackWorld
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern

    def rank_fn(ctx):
        r = ctx.rank()
        mine = [DomainDescriptor(d.id, d.gids, d.outer_lids) for d in doms_ranks[r]]
        hg = HaloGenerator(None if halo_gids is None else halo_gids[r][0])
        return make_pattern(ctx, hg, mine)

    return LoopbackWorld(len(doms_ranks)).run(rank_fn)


class _UD:
    def __init__(self, id_, gids, outer_lids):
        self.id, self.gids, self.outer_lids = id_, gids, outer_lids


def test_unstructured_pattern_known_answer(golden_dir):
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    doms = [[_UD(int(k), v["gids"], v["halo_lids"])] for k, v in sorted(case["domains"].items())]
    for r, pc in enumerate(_unstructured_abi(doms, None)):
        sends = {str(rid): lids for rid, rr, tag, lids in pc.send_halos(0)}
        recvs = {str(rid): lids for rid, rr, tag, lids in pc.recv_halos(0)}
        assert sends == case["send_maps"][str(r)]
        assert recvs == case["recv_maps"][str(r)]


def test_unstructured_pattern_matches_oracle_with_repeats(golden_dir):
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        fx = json.load(fh)["python_fixture"]
    items = sorted(fx["domains"].items())
    doms = [[_UD(int(k), v["all"], v["outer_lids"])] for k, v in items]
    hg = [[v["outer"]] for k, v in items]
    odoms = [[orc.UnstructuredDomain(int(k), v["all"], v["outer_lids"])] for k, v in items]
    opats = orc.unstructured_make_pattern(odoms, hg)
    for r, pc in enumerate(_unstructured_abi(doms, hg)):
        for direction, key in ((0, "send"), (1, "recv")):
            got = [(rr, tag, rid, lids) for rid, rr, tag, lids in pc.halos(0, direction)]
            exp = [(rr, tag, rid, lids) for (rr, tag), (rid, lids) in opats[r][0][key].items()]
            assert got == exp
        assert pc.max_tag() == 0 or pc.max_tag() > 0


def test_exchange_buffer_plan_matches_oracle():
    """communication_object::allocate: buffers per domain pair, fields in argument order with
    alignof padding, tag offsets per pattern container — mixed f64/f32 fields (config 4 shape)."""
    from ghex_amd import _ghx
    ranks, gf, gl = H.cube_domains(5, (2, 2, 2))
    types = [(8, 8), (4, 4), (8, 8), (4, 4), (8, 8)]
    Hw = 3
    for r in (0, 5):
        pc = _regular_pattern_abi(ranks, gf, gl, (Hw,) * 6, (1, 1, 1), r)
        opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
        items, oitems = [], []
        E = 5 + 2 * Hw
        for k, (elem, align) in enumerate(types):
            fd = _ghx.FieldDesc()
            fd.dim, fd.elem_size = 3, elem
            for d in range(3):
                fd.layout[d] = 2 - d
                fd.offsets[d] = Hw
                fd.extents[d] = E
            fd.byte_strides[0], fd.byte_strides[1], fd.byte_strides[2] = elem, elem * E, elem * E * E
            fd.num_components, fd.has_components = 1, 0
            it = _ghx.ExchangeItem()
            it.pattern, it.local_index, it.kind, it.field = pc.handle, 0, 0, fd
            it.align, it.tag_offset = align, 0
            items.append(it)
            oitems.append((k, r, opat[r][0], elem, align, 1, 0))
        from ghex_amd.communication_object import _ExchangePlan
        plan = _ExchangePlan(items)
        for direction, receive in ((plan.send, False), (plan.recv, True)):
            ob = orc.plan_buffers(oitems, receive)
            assert [(b["pair"], b["rank"], b["tag"], b["size"]) for b in direction] == \
                [(pair, b.rank, b.tag, b.size) for pair, b in ob.items()]
        # 4-byte fields after 8-byte ones: the padding rule produced odd offsets somewhere?
        sizes = [b["size"] for b in plan.send]
        assert len(sizes) == 7


def _put_entries(lasts, strides=(8, 96, 1152)):
    import ctypes
    from ghex_amd import _ghx
    out = []
    for last in lasts:
        d = _ghx.FieldDesc()
        d.dim, d.elem_size = 3, 8
        for k in range(3):
            d.layout[k] = 2 - k
            d.byte_strides[k] = strides[k]
            d.offsets[k] = 2
            d.extents[k] = 12
        d.num_components, d.has_components = 1, 0
        arr = (_ghx.Box * 1)()
        for k in range(3):
            arr[0].first[k], arr[0].last[k] = 0, last[k]
        e = _ghx.PackEntry()
        e.field, e.field_slot, e.buffer_slot, e.buffer_offset = d, 0, 0, 0
        e.boxes, e.n_boxes = ctypes.cast(arr, ctypes.POINTER(_ghx.Box)), 1
        out.append((e, arr))
    return out


def test_put_plan_pairs_matching_sides_and_refuses_mismatch():
    """ghx_put_create (zero-copy put, host-side planning only here): same message bytes on both
    sides -> a plan; different shapes -> GHX_ERR_INVALID with a message."""
    import ctypes
    from ghex_amd import _ghx
    L = _ghx.lib()
    (a, ka), (b, kb) = _put_entries([(3, 1, 1), (3, 1, 1)])
    h = ctypes.c_void_p()
    assert L.ghx_put_create(ctypes.byref(a), 1, ctypes.byref(b), 1, ctypes.byref(h)) == 0
    nb = ctypes.c_uint64()
    assert L.ghx_put_info(h, ctypes.byref(nb), None) == 0 and nb.value == 4 * 2 * 2 * 8
    assert L.ghx_put_destroy(h) == 0
    (a, ka), (b, kb) = _put_entries([(3, 1, 1), (1, 3, 1)])
    assert L.ghx_put_create(ctypes.byref(a), 1, ctypes.byref(b), 1, ctypes.byref(h)) == -1
    assert b"same message bytes" in L.ghx_last_error()


def test_plans_beyond_64_slots_are_cut_into_launch_groups():
    """A launch carries at most 64 field and 64 buffer pointers; a plan whose entries use more
    slots (many fields in one exchange, many domain-pair buffers) is planned in launch groups of
    <= 64 slots each: every slot accepted, every tile kept (the sum over entries planned alone).
    Host-side planning only here; tests/test_gpu_fuzz.py runs such exchanges on the device."""
    import ctypes
    from ghex_amd import _ghx
    L = _ghx.lib()
    ents = _put_entries([(3 + k % 5, 1 + k % 3, k % 2) for k in range(150)])
    singles = 0
    for k, (e, _) in enumerate(ents):
        e.field_slot, e.buffer_slot = k, 149 - k  # 150 distinct slots on both sides
        h = ctypes.c_void_p()
        assert L.ghx_plan_create(ctypes.byref(e), 1, 0, ctypes.byref(h)) == 0
        nt = ctypes.c_int32()
        assert L.ghx_plan_info(h, None, None, ctypes.byref(nt)) == 0
        singles += nt.value
        assert L.ghx_plan_destroy(h) == 0
    arr = (_ghx.PackEntry * len(ents))(*[e for e, _ in ents])
    h = ctypes.c_void_p()
    assert L.ghx_plan_create(arr, len(ents), 0, ctypes.byref(h)) == 0, L.ghx_last_error()
    nb, ns, nt = ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_int32()
    assert L.ghx_plan_info(h, ctypes.byref(nb), ctypes.byref(ns), ctypes.byref(nt)) == 0
    assert nt.value == singles and ns.value >= 150
    assert L.ghx_plan_destroy(h) == 0
    e, _ = ents[0]
    e.field_slot = -1
    assert L.ghx_plan_create(ctypes.byref(e), 1, 0, ctypes.byref(h)) == -1
    assert b"negative slot" in L.ghx_last_error()


def test_unstructured_lists_beyond_one_segment_are_split():
    """A segment addresses its message with 32-bit offsets: an index list of more than 1 GiB is
    planned as several segments — index ranges, or level by level for levels-last data — and
    the plan's byte count is unchanged (host-side planning; the device check is in
    tests/test_gpu_large.py)."""
    import ctypes
    import numpy as np
    from ghex_amd import _ghx
    L = _ghx.lib()
    for levels, first, n, want in ((1, 1, 1 << 21, 2), (2, 0, 1 << 20, 2), (3, 1, 1 << 19, 2),
                                   (1, 1, 1000, 1)):
        lids = np.arange(n, dtype=np.int64)[::-1].copy()
        e = _ghx.UPackEntry()
        e.data.elem_size, e.data.levels, e.data.levels_first = 1024, levels, first
        e.data.index_stride = levels if first else 1
        e.data.level_stride = 1 if first else n
        e.field_slot, e.buffer_slot, e.buffer_offset = 0, 0, 0
        e.lids = lids.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        e.n_lids = n
        h = ctypes.c_void_p()
        assert L.ghx_uplan_create(ctypes.byref(e), 1, 0, ctypes.byref(h)) == 0, L.ghx_last_error()
        nb, ns = ctypes.c_uint64(), ctypes.c_int32()
        assert L.ghx_uplan_info(h, ctypes.byref(nb), ctypes.byref(ns), None) == 0
        assert nb.value == n * levels * 1024 and ns.value >= want, (levels, first, ns.value)
        assert L.ghx_uplan_destroy(h) == 0


def test_epochs_flag_block_argument_checks_and_cleanup(ghx):
    """ghx_epochs_* (device-side access epochs of the bulk exchange) without a GPU: bad names,
    world/rank and timeouts are refused; a creating rank that cannot register the block (no
    device here) leaves no shared-memory segment behind; attaching to a missing block fails."""
    import ctypes
    import os
    L = ghx.lib()
    h = ctypes.c_void_p()
    assert L.ghx_epochs_create(b"no-slash", 1, 2, 0, 1.0, ctypes.byref(h)) == -1
    assert L.ghx_epochs_create(b"/a/b", 1, 2, 0, 1.0, ctypes.byref(h)) == -1
    assert L.ghx_epochs_create(b"/ghx_t", 1, 65, 0, 1.0, ctypes.byref(h)) == -1
    assert L.ghx_epochs_create(b"/ghx_t", 1, 2, 2, 1.0, ctypes.byref(h)) == -1
    assert L.ghx_epochs_create(b"/ghx_t", 1, 2, 0, 0.0, ctypes.byref(h)) == -1
    name = f"/ghx_test_{os.getpid()}"
    rc = L.ghx_epochs_create(name.encode(), 1, 2, 0, 1.0, ctypes.byref(h))
    if rc == 0:  # a GPU is present: clean up and stop here
        L.ghx_epochs_unlink(name.encode())
        L.ghx_epochs_destroy(h)
        return
    assert rc == -2 and b"hipHostRegister" in L.ghx_last_error()
    assert not os.path.exists("/dev/shm" + name)
    assert L.ghx_epochs_create(name.encode(), 0, 2, 1, 1.0, ctypes.byref(h)) == -1
    assert b"shm_open" in L.ghx_last_error()
    assert L.ghx_epochs_unlink(name.encode()) == -1
    assert L.ghx_epochs_peers(None, None, 0, None, 0) == -1
    assert L.ghx_epochs_enqueue(None, 0, None) == -1


def test_pattern_filter_splits_local_and_remote_halos():
    """ghx_pattern_filter (the bulk exchange's local / remote pattern split): keep=True keeps
    exactly the halos to/from the given ranks, keep=False the others, both in map order, tags
    and spaces unchanged; the two parts together are the whole pattern."""
    from tests import helpers as H
    ranks, gf, gl = H.cube_domains(6, (2, 2, 1))
    pc = _regular_pattern_abi(ranks, gf, gl, (2,) * 6, (1, 1, 1), 0)
    for sel in ([1], [1, 2], [0], [3], []):
        a = pc.filtered(sel, keep=True)
        b = pc.filtered(sel, keep=False)
        assert a.max_tag() == b.max_tag() == pc.max_tag()
        for direction in (0, 1):
            whole = pc.halos(0, direction)
            ka, kb = a.halos(0, direction), b.halos(0, direction)
            assert ka == [h for h in whole if h[1] in sel]
            assert kb == [h for h in whole if h[1] not in sel]
            assert sorted(ka + kb) == sorted(whole)


@pytest.mark.parametrize("world,cells,halo", [(2, 3000, 150), (3, 2000, 100), (8, 500, 25)])
def test_unstructured_pattern_config5_domains_match_oracle(world, cells, halo):
    """The reduced-halo make_pattern (every rank passes only its own domain; LoopbackWorld
    threads) against the oracle's all-ranks restatement of unstructured/pattern.hpp:187-370, on
    BASELINE config 5's domain generation (tools/config5_gen.cpp) at small sizes."""
    from tools import config5 as C5
    doms = [C5.generate(r, world, cells, halo) for r in range(world)]
    odoms = [[orc.UnstructuredDomain(r, g.tolist(), o.tolist())] for r, (g, o) in enumerate(doms)]
    opats = orc.unstructured_make_pattern(odoms)
    pcs = _unstructured_abi([[_UD(r, g, o)] for r, (g, o) in enumerate(doms)], None)
    for r, pc in enumerate(pcs):
        for direction, key in ((0, "send"), (1, "recv")):
            got = [(rr, tag, rid, list(lids)) for rid, rr, tag, lids in pc.halos(0, direction)]
            exp = [(rr, tag, rid, lids) for (rr, tag), (rid, lids) in opats[r][0][key].items()]
            assert got == exp
        assert sum(len(l) for *_, l in pc.recv_halos(0)) == halo


def test_unstructured_domain_errors_match_reference():
    """domain_descriptor's constructor and make_outer_lids errors (user_concepts.hpp:88-175)."""
    from ghex_amd import _ghx
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator
    with pytest.raises(_ghx.GhxError, match="repeated outer"):
        DomainDescriptor(0, [1, 2, 3], [1, 1])
    with pytest.raises(_ghx.GhxError, match="repeated inner"):
        DomainDescriptor(0, [1, 2, 1], [1])
    d = DomainDescriptor(0, [5, 7, 7, 9], [1, 2])  # gid 7 held by two outer cells
    assert d.inner_size() == 2 and d.size() == 4
    assert list(d.halo_gids(HaloGenerator())) == [7, 7]
    assert list(d.halo_gids(HaloGenerator([9, 7, 7]))) == [7, 7]  # 9 is inner: skipped
    with pytest.raises(_ghx.GhxError, match="not often enough"):
        d.halo_gids(HaloGenerator([7]))
    with pytest.raises(_ghx.GhxError, match="associated lid"):
        d.halo_gids(HaloGenerator([7, 7, 7]))


@pytest.mark.parametrize("grouping", [[[0, 1], [2, 3]], [[3], [0, 2], [1]], [[0, 1, 2, 3]]])
def test_unstructured_pattern_multi_domain_ranks_match_oracle(golden_dir, grouping):
    """Several domains per rank (the reference's tag layout shifts the source domain's local
    index by num_bits(max domains per rank), unstructured/pattern.hpp:230-233; self messages
    between two domains of one rank): the 4-domain known-answer case grouped onto 1-3 ranks,
    product (LoopbackWorld ranks, own domains only) vs the oracle."""
    with open(os.path.join(golden_dir, "unstructured_case.json")) as fh:
        case = json.load(fh)
    d = case["domains"]
    doms = [[_UD(i, d[str(i)]["gids"], d[str(i)]["halo_lids"]) for i in g] for g in grouping]
    odoms = [[orc.UnstructuredDomain(x.id, x.gids, x.outer_lids) for x in g] for g in doms]
    opats = orc.unstructured_make_pattern(odoms)
    from ghex_amd.context import LoopbackWorld
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern

    def rank_fn(ctx):
        mine = [DomainDescriptor(x.id, x.gids, x.outer_lids) for x in doms[ctx.rank()]]
        return make_pattern(ctx, HaloGenerator(), mine)

    for r, pc in enumerate(LoopbackWorld(len(grouping)).run(rank_fn)):
        assert len(pc) == len(grouping[r])
        for li in range(len(pc)):
            for direction, key in ((0, "send"), (1, "recv")):
                got = [(rr, tag, rid, lids) for rid, rr, tag, lids in pc.halos(li, direction)]
                exp = [(rr, tag, rid, lids)
                       for (rr, tag), (rid, lids) in opats[r][li][key].items()]
                assert got == exp, (r, li, key)


@pytest.mark.parametrize("block", range(8))
def test_unstructured_pattern_random_meshes_match_oracle(block):
    """200 seeded random meshes (tests/test_gpu_fuzz.py::draw_unstructured: 1-4 ranks with 1-2
    domains each, repeated halo gids, random storage orders), half with an explicit halo
    generator per rank (a random subset of its outer gids plus gids it does not hold, which
    halo_generator skips, user_concepts.hpp:251-255): the product's reduced-halo make_pattern
    (LoopbackWorld ranks) equals the oracle's all-ranks restatement, key for key."""
    from tests.test_gpu_fuzz import draw_unstructured
    from ghex_amd.context import LoopbackWorld
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    for seed in range(block * 25, block * 25 + 25):
        case = draw_unstructured(seed)
        nr = case["nr"]
        by_rank = [[d for d in case["doms"] if d["rank"] == r] for r in range(nr)]
        rng = np.random.default_rng(seed + 991)
        hg = None
        if seed % 2:
            hg = []
            for r in range(nr):
                mult = {}  # each outer gid as often as the rank's first domain holding it has it
                for d in by_rank[r]:
                    cnt = {}
                    for l in d["outer"]:
                        cnt[d["gids"][l]] = cnt.get(d["gids"][l], 0) + 1
                    for g, c in cnt.items():
                        mult.setdefault(g, c)
                pick = [g for g in sorted(mult) if rng.random() < 0.6 for _ in range(mult[g])]
                pick += [7, 10 ** 6 + seed]
                hg.append([int(x) for x in rng.permutation(pick)])
        odoms = [[orc.UnstructuredDomain(d["id"], d["gids"], d["outer"]) for d in ds]
                 for ds in by_rank]
        try:
            opats = orc.unstructured_make_pattern(
                odoms, None if hg is None else [[hg[r]] * len(ds) for r, ds in enumerate(by_rank)])
        except RuntimeError as e:  # e.g. a repeated gid only partly named: both must refuse
            with pytest.raises(Exception, match=str(e)[:20]):
                LoopbackWorld(nr).run(lambda ctx: make_pattern(
                    ctx, HaloGenerator(hg[ctx.rank()]),
                    [DomainDescriptor(d["id"], d["gids"], d["outer"]) for d in by_rank[ctx.rank()]]))
            continue

        def rank_fn(ctx):
            r = ctx.rank()
            mine = [DomainDescriptor(d["id"], d["gids"], d["outer"]) for d in by_rank[r]]
            return make_pattern(ctx, HaloGenerator(None if hg is None else hg[r]), mine)

        for r, pc in enumerate(LoopbackWorld(nr).run(rank_fn)):
            for li in range(len(pc)):
                for direction, key in ((0, "send"), (1, "recv")):
                    got = [(rr, tag, rid, lids) for rid, rr, tag, lids in pc.halos(li, direction)]
                    exp = [(rr, tag, rid, lids)
                           for (rr, tag), (rid, lids) in opats[r][li][key].items()]
                    assert got == exp, (seed, r, li, key)


def test_unstructured_pattern_edge_cases():
    """A domain without outer cells, an explicit empty halo generator and a rank without any
    halo: the reduced-halo make_pattern agrees with the oracle (empty maps where the reference
    has none)."""
    from ghex_amd.context import LoopbackWorld
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    ranks = [[(0, [10, 11, 12, 20, 21], [3, 4])],  # holds 20, 21 of rank 1 as outer cells
             [(1, [20, 21, 22], [])]]              # no outer cells at all
    for hgs in (None, [[21], []], [[], []]):
        odoms = [[orc.UnstructuredDomain(i, g, o) for i, g, o in rs] for rs in ranks]
        opats = orc.unstructured_make_pattern(
            odoms, None if hgs is None else [[h] for h in hgs])

        def rank_fn(ctx):
            r = ctx.rank()
            mine = [DomainDescriptor(i, g, o) for i, g, o in ranks[r]]
            return make_pattern(ctx, HaloGenerator(None if hgs is None else hgs[r]), mine)

        for r, pc in enumerate(LoopbackWorld(2).run(rank_fn)):
            for direction, key in ((0, "send"), (1, "recv")):
                got = [(rr, tag, rid, lids) for rid, rr, tag, lids in pc.halos(0, direction)]
                exp = [(rr, tag, rid, lids) for (rr, tag), (rid, lids) in opats[r][0][key].items()]
                assert got == exp, (hgs, r, key)


def test_loopback_world_reusable_after_failure():
    """A rank that raises aborts the run (the others leave their barrier) and its error is
    re-raised; the same LoopbackWorld then runs again with a fresh rendezvous."""
    from ghex_amd.context import LoopbackWorld
    w = LoopbackWorld(3)

    def bad(ctx):
        if ctx.rank() == 1:
            raise ValueError("rank 1 failed")
        return ctx.all_gather_object(ctx.rank())

    with pytest.raises(ValueError, match="rank 1 failed"):
        w.run(bad)

    def good(ctx):
        got = ctx.exchange_arrays([((ctx.rank() + 1) % 3, [ctx.rank()] * 2)],
                                  [((ctx.rank() - 1) % 3, 2)])
        return ctx.all_gather_object(ctx.rank()), [int(x) for x in got[0]]

    assert w.run(good) == [([0, 1, 2], [2, 2]), ([0, 1, 2], [0, 0]), ([0, 1, 2], [1, 1])]


@pytest.mark.parametrize("thread_safe", [True, False])
def test_context_and_config_like_the_reference(thread_safe, capsys):
    """test/bindings/python/test_context.py: the module's version and configuration, and a
    context over one process (here: no torch.distributed group = the single rank)."""
    import ghex_amd
    from ghex_amd.context import make_context
    assert ghex_amd.__version__ and ghex_amd.__config__["gpu"] is True
    assert ghex_amd.config() == ghex_amd.__config__ and ghex_amd.config() is not ghex_amd.__config__
    ghex_amd.print_config()
    assert "transport" in capsys.readouterr().out
    ctx = make_context(None, thread_safe)
    assert ctx.size() == 1 and ctx.rank() == 0


def test_stream_argument_forms_refused_like_the_reference():
    """as_stream refuses what the reference binding's extract_cuda_stream refuses
    (bindings/python/src/_pyghex/unstructured/communication_object.cpp:39-85)."""
    from ghex_amd.communication_object import as_stream

    class Bad:
        pass

    class V1:
        def __cuda_stream__(self):
            return 1, 0

    class Short:
        def __cuda_stream__(self):
            return (0,)
    with pytest.raises(TypeError, match="Failed to convert"):
        as_stream(Bad())
    with pytest.raises(TypeError, match="version 0"):
        as_stream(V1())
    with pytest.raises(TypeError, match="length 2"):
        as_stream(Short())


def test_unstructured_tag_collision_fails_on_every_rank():
    """with several domains per rank the reference's tag layout
    (src_local << num_bits(max domains per rank)) | dst_id (unstructured/pattern.hpp:230-232)
    repeats a tag once a domain id needs more bits: here shift = num_bits(2) = 3, and rank 0's
    second domain (local index 1) sends to rank 1's domains 8 and 0 under tag
    (1 << 3) | 8 == (1 << 3) | 0 == 8.
    The reference's map keeps one of the two halos and the exchange hangs or moves wrong data;
    here setup fails, on every rank (the others do not wait in the ring or a later collective)."""
    from ghex_amd.context import LoopbackWorld
    from ghex_amd.unstructured import DomainDescriptor, HaloGenerator, make_pattern
    ranks = [[(1, list(range(0, 10)), []), (2, list(range(10, 20)), [])],
             [(8, list(range(20, 30)) + [10], [10]), (0, list(range(30, 40)) + [11], [10])]]
    errs = []

    def rank_fn(ctx):
        try:
            make_pattern(ctx, HaloGenerator(), [DomainDescriptor(i, g, o) for i, g, o in ranks[ctx.rank()]])
        except Exception as e:
            errs.append((ctx.rank(), str(e)))
            return "raised"
        return "returned"

    assert LoopbackWorld(2).run(rank_fn) == ["raised", "raised"]
    assert any("share tag 8" in e for _, e in errs), errs
    # the same halos with domain ids below 1 << shift are fine
    ranks[1][0] = (3,) + ranks[1][0][1:]
    assert LoopbackWorld(2).run(rank_fn) == ["returned", "returned"]
