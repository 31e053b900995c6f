"""Seeded random structured exchanges, device path against the oracle.

Each case draws a non-cubic periodic-or-not global grid, an uneven decomposition into boxes, 1-3
domains per rank (ranks emulated in one process), two pattern containers with independent
asymmetric halos (0-3 cells per side, wider than a domain at times), and 1-3 fields of mixed
element types (1, 2, 4 and 8 bytes) with random layout maps and extra allocation padding
(offsets larger than the halo, extents larger than domain + halos). Every cell of every field
after the exchange — halos, interior and padding — equals the oracle's exchange, and every
packed send buffer equals the oracle's bytes (alignment pads masked: the reference never writes
them either, communication_object.hpp:1059-1065). The oracle follows
include/ghex/structured/pattern.hpp:214-571 (patterns) and pack_kernels.hpp:62-158 (bytes)."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.int16, np.float32, np.int32, np.float64, np.int64]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def _split(n, parts, rng):
    """n cells into `parts` non-empty intervals of random sizes: [(first, last)]."""
    cuts = sorted(rng.choice(np.arange(1, n), size=parts - 1, replace=False)) if parts > 1 else []
    b = [0] + [int(c) for c in cuts] + [n]
    return [(b[i], b[i + 1] - 1) for i in range(parts)]


def draw_case(seed):
    rng = np.random.default_rng(seed)
    G = [int(rng.integers(3, 15)) for _ in range(3)]
    parts = [int(rng.integers(1, min(3, G[d]) + 1)) for d in range(3)]
    ivals = [_split(G[d], parts[d], rng) for d in range(3)]
    boxes = [((ivals[0][i][0], ivals[1][j][0], ivals[2][k][0]),
              (ivals[0][i][1], ivals[1][j][1], ivals[2][k][1]))
             for k in range(parts[2]) for j in range(parts[1]) for i in range(parts[0])]
    nd = len(boxes)
    nr = int(rng.integers(1, min(4, nd) + 1))
    owner = [r for r in range(nr)] + [int(rng.integers(0, nr)) for _ in range(nd - nr)]
    owner = [owner[i] for i in rng.permutation(nd)]
    ids = [int(x) for x in rng.permutation(nd) + 10]
    ranks = [[] for _ in range(nr)]
    for b, (f, l) in enumerate(boxes):
        ranks[owner[b]].append(orc.RegularDomain(ids[b], f, l))
    halos = {pc: tuple(int(h) for h in rng.integers(0, 4, size=6)) for pc in (1, 2)}
    periodic = tuple(int(p) for p in rng.integers(0, 2, size=3))
    nf = int(rng.integers(1, 4))
    fields = []
    for _ in range(nf):
        fields.append({"dtype": DTYPES[int(rng.integers(0, len(DTYPES)))],
                       "layout": tuple(int(x) for x in rng.permutation(3)),
                       "pc": int(rng.integers(1, 3)),
                       "pad": [(int(rng.integers(0, 3)), int(rng.integers(0, 3))) for _ in range(3)]})
    return {"G": G, "ranks": ranks, "halos": halos, "periodic": periodic, "fields": fields,
            "mixed": bool(rng.integers(0, 2)), "seed": seed}


def _alloc(dom, f, halos_max, rng):
    """Random-valued field storage for `dom` (memory order by the layout map) + its FieldSpec."""
    dt = np.dtype(f["dtype"])
    offs, exts = [], []
    for d in range(3):
        n = dom.last[d] - dom.first[d] + 1
        lo, hi = halos_max[2 * d] + f["pad"][d][0], halos_max[2 * d + 1] + f["pad"][d][1]
        offs.append(lo)
        exts.append(max(2, lo + n + hi))  # extent 1 would tie two strides (layout ambiguity)
    order = sorted(range(3), key=lambda d: f["layout"][d])  # slowest ... fastest
    shape = tuple(exts[d] for d in order)
    raw = rng.integers(0, 256, size=int(np.prod(shape)) * dt.itemsize, dtype=np.uint8)
    a = raw.view(dt).reshape(shape).copy()
    return a, orc.FieldSpec(a, dt.itemsize, f["layout"], tuple(offs), tuple(exts))


def _setup_case(case):
    """Device fields, communication objects and buffer infos of every emulated rank, and the
    oracle's exchange of the same fields (its packed buffers; its field arrays are updated in
    place to the post-exchange state)."""
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field
    ranks, nr = case["ranks"], len(case["ranks"])
    gf, gl = (0, 0, 0), tuple(g - 1 for g in case["G"])
    per = case["periodic"]
    hmax = tuple(max(case["halos"][1][i], case["halos"][2][i]) for i in range(6))
    pat_o = {pc: orc.regular_make_pattern(ranks, gf, gl, case["halos"][pc], per) for pc in (1, 2)}
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    rng = np.random.default_rng(case["seed"] + 1000)
    cos, bis_all, pairs, ranks_fields = [], [], [], []
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        dds = [R.DomainDescriptor(d.id, d.first, d.last) for d in ranks[r]]
        pcs = {pc: R.make_pattern(ctx, R.HaloGenerator(gf, gl, case["halos"][pc], per), dds)
               for pc in (1, 2)}
        bis, rf = [], []
        for f in case["fields"]:  # exchange() argument order: field-major, then domains
            for li, dom in enumerate(ranks[r]):
                a, spec = _alloc(dom, f, hmax, rng)
                base, logical = device_field(a.copy(), f["layout"])
                fd = R.make_field_descriptor(dds[li], logical, spec.offsets, spec.extents)
                assert fd.layout == f["layout"]
                bis.append(pcs[f["pc"]](fd))
                pairs.append((base, a))
                rf.append((spec, dom.id, li, f["pc"]))
        cos.append(R.make_communication_object(ctx))
        bis_all.append(bis)
        ranks_fields.append(rf)
    obufs = orc.regular_exchange(ranks_fields, pat_o, nr)
    return dict(nr=nr, pat_o=pat_o, cos=cos, bis_all=bis_all, pairs=pairs,
                ranks_fields=ranks_fields, obufs=obufs)


def _check_buffer(st, r, x, got):
    """A packed message (uint8 device tensor) against the oracle's bytes, pads masked."""
    ob = st["obufs"][(r, x["pair"])]
    assert ob.size == x["size"]
    rf = st["ranks_fields"][r]
    items = [(k, f[1], st["pat_o"][f[3]][r][f[2]], f[0].elem, f[0].data.dtype.alignment, 1, 0)
             for k, f in enumerate(rf)]
    b = orc.plan_buffers(items, receive=False)[x["pair"]]
    m = np.zeros(b.size, dtype=bool)
    for pf in b.fields:
        elem = rf[pf.field_index][0].elem
        n = sum(isp.size() for isp in pf.boxes) * elem
        m[pf.offset:pf.offset + n] = True
    np.testing.assert_array_equal(got[:x["size"]].cpu().numpy()[m], ob[m])


def run_case(case):
    from ghex_amd import _ghx
    from tests.gpu_util import emulated_exchange
    st = _setup_case(case)
    _ghx.call("ghx_tune", b"mixed_always", 1 if case["mixed"] else 0)
    try:
        plans, bufs = emulated_exchange(st["cos"], st["bis_all"], mixed=case["mixed"])
    finally:
        _ghx.call("ghx_tune", b"reset", 0)
    for base, a in st["pairs"]:
        np.testing.assert_array_equal(base.cpu().numpy(), a)
    for r in range(st["nr"]):
        for i, x in enumerate(plans[r].send):
            _check_buffer(st, r, x, bufs[r][0][i])


def run_case_direct(case):
    """The same random case as the direct exchange runs it between processes
    (tests.gpu_util.EmulatedDirect: packs into the receivers' double-buffered buffers, the copy
    chosen on the device). Exchange e = 1 and e = 2 (both copies), each from the pre-exchange
    fields: every cell equals the oracle's exchange, every packed message equals the oracle's
    bytes in copy e&1, and copy 0 is untouched by exchange 1. Returns the peer messages checked."""
    from ghex_amd import _ghx
    from tests.gpu_util import EmulatedDirect
    st = _setup_case(case)
    before = [base.clone() for base, _ in st["pairs"]]
    _ghx.call("ghx_tune", b"mixed_always", 1 if case["mixed"] else 0)
    try:
        dx = EmulatedDirect(st["cos"], st["bis_all"], mixed=case["mixed"])
        msgs = dx.peer_messages()
        for e in (1, 2):
            for (base, _), b0 in zip(st["pairs"], before):
                base.copy_(b0)
            dx.exchange(e)
            for base, a in st["pairs"]:
                np.testing.assert_array_equal(base.cpu().numpy(), a)
            for r, i, q, x, d in msgs:
                _check_buffer(st, q, x, dx.recv[r][i][d * (e & 1):])
                if e == 1:  # copy 0 not yet written
                    assert bool((dx.recv[r][i][:x["size"]] == 0xA5).all())
    finally:
        _ghx.call("ghx_tune", b"reset", 0)
    return len(msgs)


@pytest.mark.parametrize("seed", range(60))
def test_random_structured_exchange(seed):
    run_case(draw_case(seed))


@pytest.mark.parametrize("seed", range(200, 230))
def test_random_direct_double_buffered_exchange(seed):
    """The seeded random cases through the direct exchange's launches: packs into the receivers'
    double-buffered buffers, copies chosen on the device (run_case_direct)."""
    run_case_direct(draw_case(seed))


def test_more_slots_than_one_launch_holds():
    """One rank with 8 domains of a periodic 6^3 grid and 70 fields: 560 exchange items (field
    slots) over 56 domain-pair buffers, far beyond the 64 field pointers one launch carries —
    the plans run as launch groups (ghx_plan.cpp partition_slots), bit-exact as ever. (Random
    seed 7 above has 178 buffers: the buffer side of the same limit.)"""
    rng = np.random.default_rng(64)
    doms = [orc.RegularDomain(100 + i, (3 * (i % 2), 3 * (i // 2 % 2), 3 * (i // 4)),
                              (3 * (i % 2) + 2, 3 * (i // 2 % 2) + 2, 3 * (i // 4) + 2))
            for i in range(8)]
    fields = [{"dtype": DTYPES[k % len(DTYPES)], "layout": tuple(int(x) for x in rng.permutation(3)),
               "pc": 1 + k % 2, "pad": [(k % 2, k % 3), (0, 1), (1, 0)]} for k in range(70)]
    run_case({"G": [6, 6, 6], "ranks": [doms], "halos": {1: (1,) * 6, 2: (2, 1, 0, 2, 1, 1)},
              "periodic": (1, 1, 1), "fields": fields, "mixed": False, "seed": 64})


def test_receive_only_field_slot_in_mixed_exchange():
    """Seed 249 (found by the soak, tools/fuzz_soak.py): 2 ranks x 12-15 thin domains, a y- halo
    only and no y periodicity, so the highest field slot of a rank belongs to a domain that only
    receives. The mixed launch (ghx_exchange_pack_self) writes that domain's self-message halos
    from the pack registers; it must fill the field slots its companion unpack segments name,
    not only the pack segments' (round-3 regression: a null field pointer in the kernel)."""
    from tests.gpu_util import emulated_exchange
    run_case(draw_case(249))
    assert emulated_exchange.mixed_ranks >= 1


# ---------------------------------------------------------------------------------------------
# unstructured: random meshes, the reference tests' halo property
# ---------------------------------------------------------------------------------------------
UDTYPES = [np.float64, np.float32, np.int32, np.int64, np.int16]


def draw_unstructured(seed):
    """Ranks (1-4) holding 1-2 domains each; every domain owns 5-60 cells with globally unique
    gids and holds a halo of gids owned by other domains (repeats allowed: a gid may be the halo
    of one domain twice, unstructured/user_concepts.hpp:88-113), all in a random storage order."""
    rng = np.random.default_rng(seed)
    nr = int(rng.integers(1, 5))
    doms = []  # (rank, id, inner gids)
    next_gid, did = 1000, 0
    for r in range(nr):
        for _ in range(int(rng.integers(1, 3))):
            n = int(rng.integers(5, 61))
            doms.append([r, did, list(range(next_gid, next_gid + n))])
            next_gid += n + int(rng.integers(0, 50))
            did += 1
    out = []
    for k, (r, i, inner) in enumerate(doms):
        others = [g for kk, d in enumerate(doms) if kk != k for g in d[2]]
        nh = int(rng.integers(0, min(len(others), 30) + 1)) if others else 0
        halo = [int(g) for g in rng.choice(others, size=nh, replace=False)] if nh else []
        if halo and rng.random() < 0.3:
            halo.append(halo[0])  # a repeated halo gid: two outer cells of one gid
        gids = inner + halo
        perm = rng.permutation(len(gids))
        gids = [gids[p] for p in perm]
        outer = sorted(int(np.where(perm == len(inner) + h)[0][0]) for h in range(len(halo)))
        out.append({"rank": r, "id": i, "gids": gids, "outer": outer})
    fields = []
    for _ in range(int(rng.integers(1, 3))):
        fields.append({"dtype": UDTYPES[int(rng.integers(0, len(UDTYPES)))],
                       "levels": int(rng.integers(1, 5)), "first": bool(rng.integers(0, 2)),
                       "pad": int(rng.integers(0, 3))})
    return {"nr": nr, "doms": out, "fields": fields, "seed": seed}


def _ufield(torch, n, f, rng):
    """Device tensor (n, levels) in the field's layout: levels_first rows padded by `pad`
    values (outer stride levels + pad), or levels_last (level-major, stride n); random bytes."""
    dt, L = np.dtype(f["dtype"]), f["levels"]
    if f["first"]:
        shape, cols = (n, L + f["pad"]), slice(0, L)
    else:
        shape = (L, n)
    raw = rng.integers(0, 256, size=int(np.prod(shape)) * dt.itemsize, dtype=np.uint8)
    a = raw.view(dt).reshape(shape).copy()
    t = torch.from_numpy(a).cuda()
    view = t[:, cols] if f["first"] else t.t()
    if L == 1 and f["first"] and f["pad"] == 0:
        view = t[:, 0]  # the 1-D form
    return t, view, a


def _setup_unstructured(case):
    import torch
    from ghex_amd import unstructured as U
    from tests.gpu_util import FakeContext, unstructured_patterns
    nr = case["nr"]
    table = {r: [] for r in range(nr)}
    rng = np.random.default_rng(case["seed"] + 7)
    cos, bis_all, recs = [], [], []
    pats = unstructured_patterns([[(d["id"], d["gids"], d["outer"]) for d in case["doms"]
                                   if d["rank"] == r] for r in range(nr)])
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        mine = [d for d in case["doms"] if d["rank"] == r]
        dds, pc = pats[r]
        bis = []
        for f in case["fields"]:
            for dd, d in zip(dds, mine):
                t, view, a = _ufield(torch, len(d["gids"]), f, rng)
                bis.append(pc(U.make_field_descriptor(dd, view)))
                recs.append((f, d, t, a))
        cos.append(U.make_communication_object(ctx))
        bis_all.append(bis)
    return cos, bis_all, recs


def _check_unstructured(case, recs):
    """Every outer cell holds, on every level, the value of the cell that owns its gid."""
    for f in case["fields"]:
        owner = {}
        for (ff, d, t, a) in recs:
            if ff is not f:
                continue
            outer = set(d["outer"])
            for lid, g in enumerate(d["gids"]):
                if lid not in outer:
                    owner[g] = a[lid, :f["levels"]] if f["first"] else a[:, lid]
        for (ff, d, t, a) in recs:
            if ff is not f:
                continue
            got = t.cpu().numpy()
            exp = a.copy()
            for lid in d["outer"]:
                v = owner[d["gids"][lid]]
                if f["first"]:
                    exp[lid, :f["levels"]] = v
                else:
                    exp[:, lid] = v
            np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


def run_unstructured(case):
    from tests.gpu_util import emulated_exchange
    cos, bis_all, recs = _setup_unstructured(case)
    emulated_exchange(cos, bis_all)
    _check_unstructured(case, recs)


def run_unstructured_direct(case):
    """A random unstructured case through the direct exchange's double-buffered launches
    (tests.gpu_util.EmulatedDirect; index-list and run-path kernels alike): exchanges 1 and 2,
    each from the pre-exchange fields, every field byte checked, copy 0 untouched by exchange 1.
    Returns the peer messages checked."""
    from tests.gpu_util import EmulatedDirect
    cos, bis_all, recs = _setup_unstructured(case)
    before = [t.clone() for (_, _, t, _) in recs]
    dx = EmulatedDirect(cos, bis_all)
    msgs = dx.peer_messages()
    for e in (1, 2):
        for (_, _, t, _), b0 in zip(recs, before):
            t.copy_(b0)
        dx.exchange(e)
        _check_unstructured(case, recs)
        if e == 1:
            for r, i, q, x, d in msgs:
                assert bool((dx.recv[r][i][:x["size"]] == 0xA5).all())
    return len(msgs)


@pytest.mark.parametrize("seed", range(40))
def test_random_unstructured_exchange(seed):
    run_unstructured(draw_unstructured(seed))


@pytest.mark.parametrize("seed", range(100, 120))
def test_random_unstructured_direct_double_buffered_exchange(seed):
    """The seeded random unstructured cases through the direct exchange's launches
    (run_unstructured_direct)."""
    run_unstructured_direct(draw_unstructured(seed))


def test_unstructured_more_buffers_than_one_launch_holds():
    """2 ranks x 40 domains, each domain's halo drawn from 12 other domains: ~960 domain-pair
    buffers and 80 field slots per rank, unpacked through launch groups of <= 64 slots."""
    rng = np.random.default_rng(99)
    doms, gid = [], 5000
    for k in range(80):
        doms.append({"rank": k // 40, "id": k, "inner": list(range(gid, gid + 6))})
        gid += 6
    out = []
    for k, d in enumerate(doms):
        src = [int(x) for x in rng.choice([j for j in range(80) if j != k], size=12, replace=False)]
        halo = [doms[j]["inner"][int(rng.integers(0, 6))] for j in src]
        gids = d["inner"] + halo
        out.append({"rank": d["rank"], "id": d["id"], "gids": gids,
                    "outer": list(range(6, 6 + len(halo)))})
    run_unstructured({"nr": 2, "doms": out, "seed": 99,
                      "fields": [{"dtype": np.float64, "levels": 2, "first": True, "pad": 1}]})


@pytest.mark.parametrize("knobs", [{"u_tile_bytes": 1024}, {"u_tile_bytes": 65536},
                                   {"u_tile_rows": 3, "urun": 0},
                                   {"small_row_bytes": 4096, "u_tile_rows": 5}])
def test_unstructured_tuning_variants_stay_bit_exact(knobs):
    """The unstructured general path (copy_tile_u: positions past a tile's end clamped to its
    last vector) under tile sizes that leave partial and tiny tiles: the seeded random meshes
    stay bit-exact."""
    from ghex_amd import _ghx
    try:
        for k, v in knobs.items():
            _ghx.call("ghx_tune", k.encode(), v)
        for seed in range(12):
            run_unstructured(draw_unstructured(seed))
    finally:
        _ghx.call("ghx_tune", b"reset", 0)
