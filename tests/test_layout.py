"""ghex_amd.structured.layout: padded-row allocation (host logic on CPU) and the device-timed
choice of the row width, with an exchange on the padded field checked cell by cell."""
import numpy as np
import pytest

import tests.helpers as H


def test_allocate_pads_rows_only():
    import torch
    from ghex_amd.structured.layout import allocate
    f = allocate((10, 7, 5), torch.float64, x_alloc=14, device="cpu", fill=3.0)
    assert tuple(f.shape) == (10, 7, 5)
    assert f.stride() == (1, 14, 14 * 7)
    assert bool((f == 3.0).all())
    g = allocate((10, 7, 5), torch.float32, device="cpu")
    assert g.stride() == (1, 10, 70)
    with pytest.raises(ValueError):
        allocate((10, 7, 5), torch.float64, x_alloc=9, device="cpu")


@pytest.mark.gpu
def test_suggested_layout_exchanges_bit_exact():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    from ghex_amd.structured import regular as R
    from ghex_amd.structured.layout import allocate, suggest_x_alloc
    N, Hw = 24, 2
    E = N + 2 * Hw
    xa = suggest_x_alloc((E, E, E), Hw, reps=5)
    assert E <= xa <= E + 16
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, _ = H.linear_index_field(dom, N, Hw, gl)  # memory order (z, y, x)
    f = allocate((E, E, E), torch.float64, x_alloc=xa, fill=7.0)
    f.copy_(torch.from_numpy(a).permute(2, 1, 0))
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    co = R.make_communication_object(ctx)
    co.exchange([pc(R.make_field_descriptor(dd, f, (Hw,) * 3, (E,) * 3))]).wait()
    got = f.permute(2, 1, 0).cpu().numpy()
    np.testing.assert_array_equal(got, H.expected_linear_halo(a, dom, N, Hw, gl))
    pad = f.permute(2, 1, 0).as_strided((E, E, xa - E), (xa * E, xa, 1), E)
    assert bool((pad == 7.0).all())  # the exchange never touches the pad
