"""schedule_exchange / schedule_wait / has_scheduled_exchange (communication_object.hpp:287-330,
832-968; the reference's Python test test_unstructured_domain_descriptor.py:300-377): the
exchange is ordered after earlier work on the given stream, later work on the stream passed to
schedule_wait is ordered after the unpack, and the host never blocks until wait()."""
import numpy as np
import pytest

from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


@pytest.mark.parametrize("fuse_self", [True, False])
def test_schedule_exchange_on_side_stream(fuse_self):
    import torch
    from ghex_amd import make_context
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 24, 2
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    expect = H.expected_linear_halo(a, dom, N, Hw, gl)
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    src = torch.from_numpy(a).cuda()
    base, logical = device_field(np.full_like(a, -7.0), (2, 1, 0))
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx, fuse_self=fuse_self)
    s = torch.cuda.Stream()
    for it in range(3):
        with torch.cuda.stream(s):
            torch.cuda._sleep(2_000_000)  # keep the stream busy: ordering, not luck
            base.copy_(src)               # the field is only valid in stream order
        h = co.schedule_exchange(s, [pc(fd)])
        assert not co.has_scheduled_exchange()
        h.schedule_wait(s)
        assert co.has_scheduled_exchange()
        with torch.cuda.stream(s):
            got = base.clone()  # ordered after the unpack by schedule_wait
        assert co.has_scheduled_exchange()
        if it < 2:
            h.wait()
            assert not co.has_scheduled_exchange()
        else:
            # the next exchange completes the scheduled one by itself (:950-968)
            co.exchange([pc(fd)]).wait()
            assert not co.has_scheduled_exchange()
        s.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), expect)


def test_is_ready_after_schedule_wait():
    import torch
    from ghex_amd import make_context
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 16, 1
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    base, logical = device_field(a, (2, 1, 0))
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
    co = R.make_communication_object(ctx)
    h = co.schedule_exchange(None, pc(fd))
    h.schedule_wait(None)
    torch.cuda.synchronize()
    assert h.is_ready()
    assert not co.has_scheduled_exchange()
    np.testing.assert_array_equal(base.cpu().numpy(), H.expected_linear_halo(a, dom, N, Hw, gl))


class _ProtocolStream:
    """An object with the CUDA stream protocol (as the reference test's CUDAStreamProtocolMock)."""

    def __init__(self, s):
        self._s = s

    def __cuda_stream__(self):
        return 0, self._s.cuda_stream


class _PtrStream:
    """A CuPy-style stream: the handle in `.ptr`."""

    def __init__(self, s):
        self.ptr = s.cuda_stream


@pytest.mark.parametrize("kind", ["torch", "protocol", "ptr", "none"])
def test_schedule_exchange_stream_types(kind):
    """The stream forms the reference binding accepts (test_unstructured_domain_descriptor.py
    STREAM_TYPES_TO_TEST: None, a CuPy stream, a __cuda_stream__ object): the exchange is
    ordered after the stream's earlier work and schedule_wait orders later work after it."""
    import torch
    from ghex_amd import make_context
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    N, Hw = 16, 1
    E = N + 2 * Hw
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    expect = H.expected_linear_halo(a, dom, N, Hw, gl)
    ctx = make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    src = torch.from_numpy(a).cuda()
    base, logical = device_field(np.full_like(a, -7.0), (2, 1, 0))
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx)
    s = torch.cuda.Stream() if kind != "none" else torch.cuda.current_stream()
    arg = {"torch": s, "protocol": _ProtocolStream(s), "ptr": _PtrStream(s), "none": None}[kind]
    with torch.cuda.stream(s):
        torch.cuda._sleep(2_000_000)
        base.copy_(src)
    h = co.schedule_exchange(arg, [pc(fd)])
    h.schedule_wait(arg)
    with torch.cuda.stream(s):
        got = base.clone()
    h.wait()
    s.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), expect)
