"""hipGraph capture of the C ABI's executions (include/ghx.h ABI rules: executions are
stream-ordered, never allocate and never synchronise, so a caller may capture them): the
exchange-plan pack/unpack and the cached convenience entry point, captured once and replayed
after the field changed — the replays must read the field's current contents and write the
oracle's bytes."""
import ctypes

import numpy as np
import pytest

import tests.helpers as H
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def _capture(torch, fn):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn(side.cuda_stream)  # warm: plans and caches built outside the capture
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn(torch.cuda.current_stream().cuda_stream)
    return g


@pytest.mark.parametrize("N,Hw", [(12, 2), (9, 3)])
def test_exchange_pack_unpack_replayed_from_a_graph(N, Hw):
    import torch
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    from tests.gpu_util import device_field
    ranks, gf, gl = H.cube_domains(N, (1, 1, 1))
    dom = ranks[0][0]
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    base, logical = device_field(a.copy(), (2, 1, 0))
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
    co = R.make_communication_object(ctx)
    bis = [pc(fd)]
    plan = co.plan(bis)
    send, recv = co.buffers(plan, base.device)
    L = _ghx.lib()
    fp = _ghx.ptr_array([fd.data_ptr()])
    sp = _ghx.ptr_array([t.data_ptr() for t in send])
    rp = _ghx.ptr_array([t.data_ptr() for t in recv])

    def step(s):
        _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")
        _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, rp, len(recv), s), "unpack")
    g = _capture(torch, step)
    for scale in (3.0, -7.0):
        # new owned values, stale halos: the replay must move the current contents
        b = a.copy()
        owned = b != -1
        b[owned] = b[owned] * scale
        base.copy_(torch.from_numpy(b))
        g.replay()
        torch.cuda.synchronize()
        exp = H.expected_linear_halo(b, dom, N, Hw, gl) * scale
        np.testing.assert_array_equal(base.cpu().numpy(), exp)


def test_cached_structured_pack_replayed_from_a_graph():
    import torch
    from ghex_amd import _ghx
    N, Hw = 10, 2
    E = N + 2 * Hw
    f = torch.arange(E ** 3, dtype=torch.float64, device="cuda").view(E, E, E)
    d = _ghx.FieldDesc()
    d.dim, d.elem_size, d.num_components = 3, 8, 1
    for k in range(3):
        d.layout[k] = 2 - k
        d.offsets[k] = Hw
        d.extents[k] = E
    d.byte_strides[0], d.byte_strides[1], d.byte_strides[2] = 8, 8 * E, 8 * E * E
    boxes = (_ghx.Box * 2)()
    for b, (x0, x1) in enumerate(((0, Hw - 1), (N - Hw, N - 1))):
        boxes[b].first[0], boxes[b].last[0] = x0, x1
        boxes[b].first[1], boxes[b].last[1] = 0, N - 1
        boxes[b].first[2], boxes[b].last[2] = 0, N - 1
    buf = torch.empty(2 * Hw * N * N, dtype=torch.float64, device="cuda")
    bp = ctypes.cast(boxes, ctypes.POINTER(_ghx.Box))

    def pack(s):
        _ghx.check(_ghx.lib().ghx_structured_pack(ctypes.byref(d), f.data_ptr(), buf.data_ptr(),
                                                   bp, 2, s), "structured_pack")
    g = _capture(torch, pack)
    for k in (1.0, 5.0):
        f.mul_(k)
        buf.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        a = f.cpu().numpy()
        spec = orc.FieldSpec(np.ascontiguousarray(a), 8, (2, 1, 0), (Hw,) * 3, (E,) * 3)
        exp = np.zeros(buf.numel() * 8, dtype=np.uint8)
        orc.structured_pack(spec, exp, [orc.ISPair((x0, 0, 0), (x1, N - 1, N - 1),
                                                   (x0, 0, 0), (x1, N - 1, N - 1))
                                        for x0, x1 in ((0, Hw - 1), (N - Hw, N - 1))])
        np.testing.assert_array_equal(buf.cpu().numpy().view(np.uint8), exp)


def test_cached_plan_used_on_two_streams_survives_eviction():
    """a cached plan executed on stream A (held back by a long kernel) and then on
    stream B, then evicted from the 256-entry cache: it may be freed only once BOTH streams have
    passed their use, so A's pack still reads valid device tables and writes the right bytes."""
    import torch
    from ghex_amd import _ghx
    N, Hw = 12, 2
    E = N + 2 * Hw
    f = torch.arange(E ** 3, dtype=torch.float64, device="cuda").view(E, E, E)
    d = _ghx.FieldDesc()
    d.dim, d.elem_size, d.num_components = 3, 8, 1
    for k in range(3):
        d.layout[k] = 2 - k
        d.offsets[k] = Hw
        d.extents[k] = E
    d.byte_strides[0], d.byte_strides[1], d.byte_strides[2] = 8, 8 * E, 8 * E * E

    def boxes_of(y1):
        bx = (_ghx.Box * 2)()
        for b, (x0, x1) in enumerate(((0, Hw - 1), (N - Hw, N - 1))):
            bx[b].first[0], bx[b].last[0] = x0, x1
            bx[b].first[1], bx[b].last[1] = 0, y1
            bx[b].first[2], bx[b].last[2] = 0, N - 1
        return bx
    main = boxes_of(N - 1)
    buf_a = torch.full((2 * Hw * N * N,), -1.0, dtype=torch.float64, device="cuda")
    buf_b = torch.full_like(buf_a, -1.0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    L = _ghx.lib()
    bp = ctypes.cast(main, ctypes.POINTER(_ghx.Box))
    with torch.cuda.stream(sa):
        torch.cuda._sleep(200_000_000)  # hold stream A back while the host evicts the plan
    _ghx.check(L.ghx_structured_pack(ctypes.byref(d), f.data_ptr(), buf_a.data_ptr(), bp, 2,
                                     sa.cuda_stream), "pack A")
    _ghx.check(L.ghx_structured_pack(ctypes.byref(d), f.data_ptr(), buf_b.data_ptr(), bp, 2,
                                     sb.cuda_stream), "pack B")
    sb.synchronize()
    # 300 other keys (other box shapes and halo offsets) push the plan out of the cache and
    # trigger the reaping of retired plans while stream A has not yet run its pack
    scratch = torch.empty_like(buf_a)
    for i in range(300):
        d2 = _ghx.FieldDesc()
        ctypes.memmove(ctypes.byref(d2), ctypes.byref(d), ctypes.sizeof(d))
        d2.offsets[0] = Hw - (i % 2)
        bx = boxes_of(i % (N - 1))
        _ghx.check(L.ghx_structured_pack(ctypes.byref(d2), f.data_ptr(), scratch.data_ptr(),
                                         ctypes.cast(bx, ctypes.POINTER(_ghx.Box)), 2,
                                         sb.cuda_stream), "evicting pack")
    sb.synchronize()
    sa.synchronize()
    a = f.cpu().numpy()
    spec = orc.FieldSpec(np.ascontiguousarray(a), 8, (2, 1, 0), (Hw,) * 3, (E,) * 3)
    exp = np.zeros(buf_a.numel() * 8, dtype=np.uint8)
    orc.structured_pack(spec, exp, [orc.ISPair((x0, 0, 0), (x1, N - 1, N - 1),
                                               (x0, 0, 0), (x1, N - 1, N - 1))
                                    for x0, x1 in ((0, Hw - 1), (N - Hw, N - 1))])
    np.testing.assert_array_equal(buf_b.cpu().numpy().view(np.uint8), exp)
    np.testing.assert_array_equal(buf_a.cpu().numpy().view(np.uint8), exp)
