"""GPU parity: the HIP path (through the C ABI) against the oracle on the same inputs.

Bit-exact on every byte: packed send buffers (pad bytes excluded, they are never written by the
reference either — communication_object.hpp:1059-1065) and the fields after unpack.
"""
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
    import ghex_amd
    ghex_amd.native_library()  # must load: no fallback


def _single_rank_ctx():
    from ghex_amd import make_context
    return make_context()


def _oracle_exchange_single(spec_list, pattern):
    rf = [[(s, 0, 0, 0) for s in spec_list]]
    return orc.regular_exchange(rf, {0: pattern}, 1)


def _mask_for(plan_buffers_entry, fields_elem_nc):
    b = plan_buffers_entry
    m = np.zeros(b.size, dtype=bool)
    for pf in b.fields:
        elem, nc = fields_elem_nc[pf.field_index]
        n = sum(isp.size() for isp in pf.boxes) * nc * elem
        m[pf.offset:pf.offset + n] = True
    return m


LAYOUTS = [(2, 1, 0), (0, 1, 2), (1, 2, 0), (2, 0, 1), (1, 0, 2), (0, 2, 1)]


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("Hw", [1, 2, 3])
@pytest.mark.parametrize("N", [8, 13])
def test_single_domain_periodic_fp64(layout, Hw, N):
    import torch
    from ghex_amd.structured import regular as R
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, spec = H.linear_index_field(dom, N, Hw, gl, layout=layout)
    a0 = a.copy()
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    obufs = _oracle_exchange_single([spec], opat)
    ctx = _single_rank_ctx()
    hg = R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3)
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, hg, [dd])
    base, logical = __import__("tests.gpu_util", fromlist=["x"]).device_field(a0, layout)
    E = N + 2 * Hw
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    assert fd.layout == tuple(layout)
    co = R.make_communication_object(ctx)
    plan, send, recv = co.pack_only([pc(fd)])
    torch.cuda.synchronize()
    (key, ob), = obufs.items()
    assert len(plan.send) == 1 and plan.send[0]["size"] == ob.size
    got = send[0][:ob.size].cpu().numpy()
    np.testing.assert_array_equal(got, ob)
    co.unpack_only([pc(fd)])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(base.cpu().numpy(), a)
    np.testing.assert_array_equal(a, H.expected_linear_halo(a, dom, N, Hw, gl, layout=layout))


@pytest.mark.parametrize("dtype", [np.float32, np.int32, np.int64, np.uint8, np.int16])
def test_dtypes_exchange(dtype):
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 9, 2
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, spec = H.linear_index_field(dom, N, Hw, gl, dtype=dtype, seed=7)
    a0 = a.copy()
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    obufs = _oracle_exchange_single([spec], opat)
    ctx = _single_rank_ctx()
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3),
                        [R.DomainDescriptor(0, dom.first, dom.last)])
    base, logical = device_field(a0, (2, 1, 0))
    fd = R.make_field_descriptor(pc.domains[0], logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
    co = R.make_communication_object(ctx)
    h = co.exchange([pc(fd)])
    h.wait()
    np.testing.assert_array_equal(base.cpu().numpy(), a)
    (key, ob), = obufs.items()
    np.testing.assert_array_equal(co.buffers(co.plan([pc(fd)]), fd.device)[0][0][:ob.size]
                                  .cpu().numpy(), ob)


@pytest.mark.parametrize("mixed", [False, True])
@pytest.mark.parametrize("types", [(np.float64, np.float32, np.int32),
                                   (np.float64, np.float64, np.float64)])
def test_reference_geometry_4ranks_emulated(types, mixed):
    """test_regular_domain.cpp: 4 ranks x 2 domains, 3 fields of array<T,3>, 2 patterns;
    emulated in one process on one GPU; every byte vs the oracle exchange. mixed: the messages
    between a rank's own two domains are completed in the pack launch (ghx_exchange_pack_self)
    and only the peer messages unpacked."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field, emulated_exchange
    ranks, gf, gl = H.regular_test_domains(4)
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(4)}
    pat_o = {1: orc.regular_make_pattern(ranks, gf, gl, H.HALOS_1, (1, 1, 1)),
             2: orc.regular_make_pattern(ranks, gf, gl, H.HALOS_2, (1, 1, 1))}
    cos, bis_all, bases, oracle_arrays, ranks_fields = [], [], [], [], []
    for r in range(4):
        ctx = FakeContext(r, 4, table)
        dds = [R.DomainDescriptor(d.id, d.first, d.last) for d in ranks[r]]
        pcs = {1: R.make_pattern(ctx, R.HaloGenerator(gf, gl, H.HALOS_1, (1, 1, 1)), dds),
               2: R.make_pattern(ctx, R.HaloGenerator(gf, gl, H.HALOS_2, (1, 1, 1)), dds)}
        bis, rf = [], []
        for fi, (T, pcn) in enumerate(zip(types, (1, 2, 1))):
            for li in range(2):
                dom = ranks[r][li]
                a = H.coord_field(dom, T)
                base, logical = device_field(a.copy(), (2, 1, 0, 3), has_components=True)
                # array<T,3> values: the component axis is the value type, not a GHEX component
                # dim -> view the 3 components as one element of 3*sizeof(T) bytes
                ext = (a.shape[2], a.shape[1], a.shape[0])
                fd = R.make_field_descriptor(dds[li], logical, H.OFFSET, ext)
                fd_elem = _as_struct_elem(fd, a.itemsize * 3)
                bis.append(pcs[pcn](fd_elem))
                bases.append(base)
                oracle_arrays.append(a)
                rf.append((H.coord_fieldspec(a), dom.id, li, pcn))
        ranks_fields.append(rf)
        cos.append(R.make_communication_object(ctx))
        bis_all.append(bis)
    obufs = orc.regular_exchange(ranks_fields, pat_o, 4)
    from ghex_amd import _ghx
    _ghx.call("ghx_tune", b"mixed_always", 1 if mixed else 0)
    try:
        plans, bufs = emulated_exchange(cos, bis_all, mixed=mixed)
    finally:
        _ghx.call("ghx_tune", b"reset", 0)
    if mixed:
        assert emulated_exchange.mixed_ranks > 0
    for b, a in zip(bases, oracle_arrays):
        np.testing.assert_array_equal(b.cpu().numpy(), a)
    # byte parity of every send buffer (pads masked)
    for r in range(4):
        for i, x in enumerate(plans[r].send):
            ob = obufs[(r, x["pair"])]
            assert ob.size == x["size"]
            got = bufs[r][0][i][:x["size"]].cpu().numpy()
            items = [(k, f[1], pat_o[f[3]][r][f[2]], f[0].elem, f[0].data.dtype.alignment, 1, 0)
                     for k, f in enumerate(ranks_fields[r])]
            pbe = orc.plan_buffers(items, receive=False)[x["pair"]]
            m = _mask_for(pbe, {k: (f[0].elem, 1) for k, f in enumerate(ranks_fields[r])})
            np.testing.assert_array_equal(got[m], ob[m])


def _as_struct_elem(fd, elem):
    """Re-describe a (x,y,z,c=3) field of T as a 3-D field of array<T,3> values (sizeof 3*T)."""
    from ghex_amd import _ghx
    d = _ghx.FieldDesc()
    d.dim, d.elem_size = 3, elem
    for k in range(3):
        d.layout[k] = fd.layout[k] - 1 if fd.layout[k] > 0 else fd.layout[k]
        d.byte_strides[k] = fd.desc.byte_strides[k]
        d.offsets[k] = fd.desc.offsets[k]
        d.extents[k] = fd.desc.extents[k]
    # layout of (x,y,z) = (2,1,0) for these fields
    d.layout[0], d.layout[1], d.layout[2] = 2, 1, 0
    d.num_components, d.has_components = 1, 0
    fd.desc = d
    fd.has_components = False
    fd.align = elem // 3
    return fd


@pytest.mark.parametrize("parts,always", [((1, 1, 2), 0), ((1, 2, 2), 0), ((1, 2, 1), 0),
                                          ((2, 1, 1), 1), ((2, 2, 1), 1)])
def test_cube_multi_rank_emulated_mixed(parts, always):
    """Decompositions whose ranks have self AND peer messages: the pack launch completes the
    self messages (register forwarding), the unpack launch only the peer ones. x-local
    decompositions get the mixed plans by default (their self messages hold the short x rows);
    for (2,1,1) / (2,2,1) they are forced with the knob mixed_always."""
    from ghex_amd import _ghx
    from tests.gpu_util import emulated_exchange
    _ghx.call("ghx_tune", b"mixed_always", always)
    try:
        test_cube_multi_rank_emulated(parts, mixed=True)
    finally:
        _ghx.call("ghx_tune", b"reset", 0)
    assert emulated_exchange.mixed_ranks == parts[0] * parts[1] * parts[2]


@pytest.mark.parametrize("parts", [(2, 1, 1), (2, 2, 2), (3, 2, 1)])
def test_cube_multi_rank_emulated(parts, mixed=False):
    _cube_multi_rank(parts, 10, 2, mixed)


@pytest.mark.parametrize("parts,N,Hw", [((4, 2, 2), 2, 3), ((3, 3, 3), 1, 2), ((4, 1, 1), 2, 3),
                                        ((5, 2, 1), 1, 2)])
def test_halo_wider_than_neighbour_domains(parts, N, Hw):
    """Halos wider than a domain: a halo box reaches through its neighbour into the next
    domain(s), and boxes that straddle the periodic boundary are wrapped but not split
    (halo_generator.hpp:133-145), so the reference leaves their far cells untouched. Bytes and
    fields equal the oracle's, untouched cells included."""
    _cube_multi_rank(parts, N, Hw, full=False)


def test_config1_full_size_two_emulated_ranks():
    """BASELINE config 1 (128^3 fp64 per rank, H=1, periodic, (2,1,1)) on the device path: both
    ranks' packed buffers routed, unpacked, every cell equal to the oracle's exchange."""
    _cube_multi_rank((2, 1, 1), 128, 1)


def _cube_multi_rank(parts, N, Hw, mixed=False, full=True):
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field, emulated_exchange
    ranks, gf, gl = H.cube_domains(N, parts)
    nr = len(ranks)
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    cos, bis, bases, arrs, rf = [], [], [], [], []
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        dd = R.DomainDescriptor(ranks[r][0].id, ranks[r][0].first, ranks[r][0].last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)), [dd])
        a, spec = H.linear_index_field(ranks[r][0], N, Hw, gl)
        base, logical = device_field(a.copy(), (2, 1, 0))
        fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
        cos.append(R.make_communication_object(ctx))
        bis.append([pc(fd)])
        bases.append(base)
        arrs.append(a)
        rf.append([(spec, ranks[r][0].id, 0, 0)])
    before = [a.copy() for a in arrs]
    orc.regular_exchange(rf, {0: opat}, nr)
    emulated_exchange(cos, bis, mixed=mixed)
    for b, a, doms in zip(bases, arrs, ranks):
        np.testing.assert_array_equal(b.cpu().numpy(), a)
        if full:
            np.testing.assert_array_equal(a, H.expected_linear_halo(a, doms[0], N, Hw, gl))
    if not full:  # the exchange did fill halo cells beyond the nearest neighbour
        assert any((a != a0).sum() > 0 for a, a0 in zip(arrs, before))


def test_mixed_five_fields_config4_shape():
    """Config 4 shape (scaled): 5 fields [f64,f32,f64,f32,f64], H=3, one exchange, pads."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import FakeContext, device_field, emulated_exchange
    N, Hw = 7, 3
    ranks, gf, gl = H.cube_domains(N, (2, 2, 2))
    nr = 8
    table = {r: [(d.id, d.first, d.last) for d in ranks[r]] for r in range(nr)}
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    types = [np.float64, np.float32, np.float64, np.float32, np.float64]
    cos, bis, pairs, rf = [], [], [], []
    for r in range(nr):
        ctx = FakeContext(r, nr, table)
        dd = R.DomainDescriptor(r, ranks[r][0].first, ranks[r][0].last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (1, 1, 1)), [dd])
        bl, fl = [], []
        for k, T in enumerate(types):
            a, spec = H.linear_index_field(ranks[r][0], N, Hw, gl, dtype=T, seed=k)
            base, logical = device_field(a.copy(), (2, 1, 0))
            fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
            bl.append(pc(fd))
            pairs.append((base, a))
            fl.append((spec, r, 0, 0))
        cos.append(R.make_communication_object(ctx))
        bis.append(bl)
        rf.append(fl)
    obufs = orc.regular_exchange(rf, {0: opat}, nr)
    plans, bufs = emulated_exchange(cos, bis)
    for base, a in pairs:
        np.testing.assert_array_equal(base.cpu().numpy(), a)
    for r in range(nr):
        items = [(k, r, opat[r][0], f[0].elem, f[0].data.dtype.alignment, 1, 0)
                 for k, f in enumerate(rf[r])]
        pb = orc.plan_buffers(items, receive=False)
        for i, x in enumerate(plans[r].send):
            ob = obufs[(r, x["pair"])]
            m = _mask_for(pb[x["pair"]], {k: (f[0].elem, 1) for k, f in enumerate(rf[r])})
            np.testing.assert_array_equal(bufs[r][0][i][:x["size"]].cpu().numpy()[m], ob[m])


def test_field_descriptor_pack_unpack_api_unaligned_and_components():
    """field.pack(buffer, spaces, stream) / unpack — the concept's member functions — on a
    vector field (component axis) at a misaligned base (vector-width downgrade)."""
    import torch
    from ghex_amd.structured import regular as R
    N, Hw, nc = 6, 2, 3
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    rng = np.random.default_rng(3)
    # memory (z, y, x, c) float32, plus a 1-element shift to misalign the base by 4 bytes
    flat = rng.integers(0, 1 << 20, size=E * E * E * nc + 1).astype(np.float32)
    a_mem = flat[1:].reshape(E, E, E, nc)
    spec = orc.FieldSpec(a_mem, 4, (2, 1, 0, 3), (Hw,) * 3 + (0,), (E,) * 3 + (nc,),
                         num_components=nc, has_components=True)
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    lst = list(opat[0][0].send.values())[0][1]
    n = sum(b.size() for b in lst) * nc * 4
    ob = np.zeros(n, np.uint8)
    orc.structured_pack(spec, ob, lst)
    dflat = torch.from_numpy(flat).cuda()
    logical = dflat[1:].view(E, E, E, nc).permute(2, 1, 0, 3)
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    assert fd.has_components and fd.num_components == nc
    buf = torch.zeros(n + 4, dtype=torch.uint8, device="cuda")
    spaces = [(b.lf, b.ll) for b in lst]
    fd.pack(buf[4:], spaces)  # buffer misaligned by 4 too
    torch.cuda.synchronize()
    np.testing.assert_array_equal(buf[4:].cpu().numpy(), ob)
    # unpack into the halo of a fresh copy and compare with the oracle's unpack
    rl = list(opat[0][0].recv.values())[0][1]
    a2 = a_mem.copy()
    spec2 = orc.FieldSpec(a2, 4, (2, 1, 0, 3), (Hw,) * 3 + (0,), (E,) * 3 + (nc,),
                          num_components=nc, has_components=True)
    orc.structured_unpack(spec2, ob, rl)
    fd.unpack(buf[4:], [(b.lf, b.ll) for b in rl])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dflat[1:].cpu().numpy().reshape(E, E, E, nc), a2)


def test_strided_fastest_dim_elementwise():
    """A field whose fastest dim is not unit-stride (a sliced view): element-wise semantics of the
    GPU reference (pack_kernels.hpp:161-183), checked against the oracle's element-wise mode."""
    import torch
    from ghex_amd.structured import regular as R
    N, Hw = 6, 1
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    big = np.arange(E * E * 2 * E, dtype=np.float64).reshape(E, E, 2 * E)
    view = big[:, :, ::2]  # x stride 16 B
    spec = orc.FieldSpec(view, 8, (2, 1, 0), (Hw,) * 3, (E,) * 3,
                         byte_strides=(16, 16 * E, 16 * E * E))
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    lst = list(opat[0][0].send.values())[0][1]
    n = sum(b.size() for b in lst) * 8
    ob = np.zeros(n, np.uint8)
    orc.lib()
    orc.structured_pack(spec, ob, lst, elementwise=True)
    dbig = torch.from_numpy(big).cuda()
    logical = dbig[:, :, ::2].permute(2, 1, 0)
    fd = R.make_field_descriptor(R.DomainDescriptor(0, dom.first, dom.last), logical,
                                 (Hw,) * 3, (E,) * 3)
    buf = torch.zeros(n, dtype=torch.uint8, device="cuda")
    fd.pack(buf, [(b.lf, b.ll) for b in lst])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(buf.cpu().numpy(), ob)


def test_full_size_512_h2_checksum():
    """BASELINE config 2 at full size: 512^3 fp64, H=2, one periodic domain. Packed buffer
    checksum (FNV-1a 64) and the unpacked field equal the oracle's; halo property holds."""
    import torch
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 512, 2
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, spec = H.linear_index_field(dom, N, Hw, gl)
    base, logical = device_field(a, (2, 1, 0))
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    obufs = _oracle_exchange_single([spec], opat)  # packs + unpacks `a` in place
    (key, ob), = obufs.items()
    assert ob.size == 101451776 // 4  # n(512,2) * 8 B
    ctx = _single_rank_ctx()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx)
    co.exchange([pc(fd)]).wait()
    send = co.buffers(co.plan([pc(fd)]), fd.device)[0][0]
    got = send[:ob.size].cpu().numpy()
    assert orc.fnv1a64(got) == orc.fnv1a64(ob)
    out = base.cpu().numpy()
    assert np.array_equal(out, a)
    # size-independent property on the halo shell: every cell = wrapped global linear index
    G = N
    for sl in (np.s_[:Hw], np.s_[-Hw:]):
        z = out[sl]  # z halo planes
        zz, yy, xx = np.meshgrid(np.arange(z.shape[0]), np.arange(E), np.arange(E), indexing="ij")
        zi = zz if sl == np.s_[:Hw] else zz + E - Hw
        exp = ((xx - Hw) % G) + G * (((yy - Hw) % G) + G * ((zi - Hw) % G))
        assert np.array_equal(z, exp.astype(np.float64))
    del base, logical
    torch.cuda.empty_cache()


@pytest.mark.parametrize("knobs", [{"order": 0, "small_tile_rows": 100},
                                   {"order": 0, "tile_bytes": 1024},
                                   {"small_tile_rows": 64}, {"small_tile_rows": 512},
                                   {"grid_cap": 7}, {"grid_cap": 300, "xcd_pair": 0},
                                   {"short_pol": 3}, {"short_pol": 1, "small_row_bytes": 4096},
                                   {"short_pol": 2, "small_tile_rows": 64},
                                   {"tile_bytes": 65536, "small_row_bytes": 8},
                                   {"short_pol": 3, "tile_bytes": 4096},
                                   {"tile_records": 0}, {"tile_records": 0, "grid_cap": 7},
                                   {"unpack_tile_bytes": 32768},
                                   {"unpack_tile_bytes": 16384, "tile_records": 0},
                                   {"fast_addr": 0}, {"fast_addr": 0, "tile_records": 0},
                                   {"pack_tile_rows": 64}, {"unpack_tile_rows": 64},
                                   {"pack_tile_rows": 4096, "unpack_tile_rows": 128}],
                         ids=lambda d: "-".join(f"{k}={v}" for k, v in d.items()))
@pytest.mark.parametrize("Hw", [1, 2, 3])
def test_tuning_variants_stay_bit_exact(knobs, Hw):
    """Every launch/planning setting of the remaining ghx_tune knobs produces the same bytes."""
    from ghex_amd import _ghx
    try:
        for k, v in knobs.items():
            _ghx.call("ghx_tune", k.encode(), v)
        test_single_domain_periodic_fp64((2, 1, 0), Hw, 11)
        test_single_domain_periodic_fp64((2, 1, 0), Hw, 16)  # 16-B aligned x-face rows
        test_cube_multi_rank_emulated((2, 2, 2))
    finally:
        _ghx.call("ghx_tune", b"reset", 0)
