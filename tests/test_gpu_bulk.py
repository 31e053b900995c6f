"""Zero-copy bulk exchange (BulkCommunicationObject, libghx ghx_put_*): every send region is
copied straight into the receiving field's halo. Checked against the oracle's exchange and the
reference tests' halo properties; one process here (self puts, several domains per rank), real
multi-process IPC puts in tests/test_gpu_multiproc.py."""
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
    ghex_amd.native_library()


@pytest.mark.parametrize("Hw", [1, 2, 3])
@pytest.mark.parametrize("layout", [(2, 1, 0), (0, 2, 1), (1, 0, 2)])
def test_bulk_single_periodic_domain(layout, Hw):
    from ghex_amd import make_context, make_bulk_communication_object
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N = 20
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, spec = H.linear_index_field(dom, N, Hw, gl, layout=layout)
    base, logical = device_field(a.copy(), layout)
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    bco = make_bulk_communication_object(ctx)
    bco.add_field(pc(fd))
    bco.init()
    assert bco.bytes_per_exchange() == (E ** 3 - N ** 3) * 8
    for _ in range(2):
        bco.exchange().wait()
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    orc.regular_exchange([[(spec, 0, 0, 0)]], {0: opat}, 1)
    got = base.cpu().numpy()
    np.testing.assert_array_equal(got, a)
    np.testing.assert_array_equal(got, H.expected_linear_halo(a, dom, N, Hw, gl, layout=layout))


@pytest.mark.parametrize("types", [(np.float64, np.float32, np.int32)])
def test_bulk_one_rank_eight_domains_two_patterns(types):
    """The reference test geometry (test_regular_domain.cpp) with all 8 domains on one rank,
    3 fields x 8 domains of array<T,3>, 2 pattern containers: every domain pair is a put."""
    from ghex_amd import make_context, make_bulk_communication_object
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    from tests.test_gpu_parity import _as_struct_elem
    ranks4, gf, gl = H.regular_test_domains(4)
    doms = [d for r in ranks4 for d in r]
    ctx = make_context()
    dds = [R.DomainDescriptor(d.id, d.first, d.last) for d in doms]
    pcs = {1: R.make_pattern(ctx, R.HaloGenerator(gf, gl, H.HALOS_1, (1, 1, 1)), dds),
           2: R.make_pattern(ctx, R.HaloGenerator(gf, gl, H.HALOS_2, (1, 1, 1)), dds)}
    pat_o = {1: orc.regular_make_pattern([doms], gf, gl, H.HALOS_1, (1, 1, 1)),
             2: orc.regular_make_pattern([doms], gf, gl, H.HALOS_2, (1, 1, 1))}
    bco = make_bulk_communication_object(ctx)
    bases, arrays, rf = [], [], []
    for T, pcn in zip(types, (1, 2, 1)):
        for li, dom in enumerate(doms):
            a = H.coord_field(dom, T)
            base, logical = device_field(a.copy(), (2, 1, 0, 3), has_components=True)
            ext = (a.shape[2], a.shape[1], a.shape[0])
            fd = _as_struct_elem(R.make_field_descriptor(dds[li], logical, H.OFFSET, ext),
                                 a.itemsize * 3)
            bco.add_field(pcs[pcn](fd))
            bases.append(base)
            arrays.append(a)
            rf.append((H.coord_fieldspec(a), dom.id, li, pcn))
    bco.exchange().wait()
    orc.regular_exchange([rf], pat_o, 1)
    for b, a in zip(bases, arrays):
        np.testing.assert_array_equal(b.cpu().numpy(), a)


def test_put_rejects_mismatched_sides():
    """Source and target spaces of different shapes are refused (GHX_ERR_INVALID)."""
    import ctypes
    import torch
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    t = torch.zeros((12, 12, 12), dtype=torch.float64, device="cuda")
    fd = R.make_field_descriptor(R.DomainDescriptor(0, (0, 0, 0), (7, 7, 7)), t, (2, 2, 2),
                                 (12, 12, 12))
    entries = []
    for last in ((3, 1, 1), (1, 3, 1)):
        arr = (_ghx.Box * 1)()
        arr[0].first[0], arr[0].first[1], arr[0].first[2] = 0, 0, 0
        arr[0].last[0], arr[0].last[1], arr[0].last[2] = last
        e = _ghx.PackEntry()
        e.field, e.field_slot, e.buffer_slot, e.buffer_offset = fd.desc, 0, 0, 0
        e.boxes, e.n_boxes = ctypes.cast(arr, ctypes.POINTER(_ghx.Box)), 1
        entries.append((e, arr))
    h = ctypes.c_void_p()
    rc = _ghx.lib().ghx_put_create(ctypes.byref(entries[0][0]), 1, ctypes.byref(entries[1][0]),
                                   1, ctypes.byref(h))
    assert rc == -1 and b"same message bytes" in _ghx.lib().ghx_last_error()


def test_bulk_more_fields_than_one_launch_holds():
    """70 fields of one periodic domain in one bulk object: the puts are planned in launches of
    <= 64 source and <= 64 target fields (ghx_put_create takes one launch's worth), every halo
    equal to the oracle's exchange."""
    from ghex_amd import make_context, make_bulk_communication_object
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 6, 1
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    opat = orc.regular_make_pattern(ranks, gf, gl, (Hw,) * 6, (1, 1, 1))
    bco = make_bulk_communication_object(ctx)
    pairs, rf = [], []
    for k in range(70):
        a, spec = H.linear_index_field(dom, N, Hw, gl, seed=k)
        base, logical = device_field(a.copy(), (2, 1, 0))
        bco.add_field(pc(R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)))
        pairs.append((base, a))
        rf.append((spec, 0, 0, 0))
    bco.init()
    assert bco.bytes_per_exchange() == 70 * (E ** 3 - N ** 3) * 8
    bco.exchange().wait()
    orc.regular_exchange([rf], {0: opat}, 1)
    for base, a in pairs:
        np.testing.assert_array_equal(base.cpu().numpy(), a)
