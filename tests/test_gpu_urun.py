"""Unstructured run path (copy_runs in ghx_kernels.hip): rows of 4 or 8 bytes whose lids form
runs move as 16-B field accesses, the rest row by row inside the same 16-B lane chunk.

Bit-exact against the oracle's restatement of data_descriptor get/set
(include/ghex/unstructured/user_concepts.hpp:385-440) on index lists built to reach every
branch: runs of 1..96 lids at odd and even starts (16-B and 8-B aligned 16-B field accesses),
runs interleaved with isolated lids, list lengths whose byte size is not a multiple of 16
(segment tails), int32 and int64 lid tables, plus the cases that must fall back to the
one-row-per-lane path (index stride != row length, a 4-B misaligned field pointer, a buffer
offset that is not a multiple of 16, urun off)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def _run_lists(rng, ncells, n_lists, per_list, maxrun):
    """Disjoint lid lists (unique lids: scatters are order-independent): runs of random length
    inside disjoint blocks, run order shuffled, some isolated lids mixed in."""
    block = max(4, 2 * maxrun)
    blocks = rng.permutation(ncells // block)
    out, bi = [], 0
    for _ in range(n_lists):
        runs, total = [], 0
        while total < per_list:
            b = int(blocks[bi]) * block
            bi += 1
            ln = int(rng.integers(1, maxrun + 1)) if rng.random() < 0.8 else 1
            st = b + int(rng.integers(0, block - ln + 1))
            runs.append(np.arange(st, st + ln))
            total += ln
        rng.shuffle(runs)
        out.append(np.concatenate(runs)[:per_list + int(rng.integers(0, 3))])
    return out


def _exchange(elem, levels, index_stride, lists, lid_bias=0, field_shift=0, buf_off=0):
    """Pack every list into its buffer, then unpack fresh buffer bytes; return (packed, field)
    from the device and the oracle. lid_bias > 0 offsets every lid (forcing int64 lid tables)
    and the field pointer by the opposite amount, so the same memory is addressed."""
    import torch
    from ghex_amd import _ghx
    rng = np.random.default_rng(7)
    ncells = max(int(l.max()) for l in lists) + 1
    nbytes = ncells * index_stride * elem
    host = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
    dev_raw = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
    base = 16 + field_shift
    dev_raw[base:base + nbytes] = torch.from_numpy(host).cuda()
    fptr = dev_raw.data_ptr() + base - lid_bias * index_stride * elem

    def plan(direction):
        ents, keep = [], []
        for k, l in enumerate(lists):
            e = _ghx.UPackEntry()
            e.data.elem_size, e.data.levels, e.data.levels_first = elem, levels, 1
            e.data.index_stride, e.data.level_stride = index_stride, 1
            e.field_slot, e.buffer_slot, e.buffer_offset = 0, k, buf_off
            arr = np.ascontiguousarray(l + lid_bias, dtype=np.int64)
            keep.append(arr)
            e.lids = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            e.n_lids = len(arr)
            ents.append(e)
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", (_ghx.UPackEntry * len(ents))(*ents), len(ents),
                  direction, ctypes.byref(h))
        return h

    sizes = [len(l) * levels * elem for l in lists]
    bufs = [torch.zeros(buf_off + s, dtype=torch.uint8, device="cuda") for s in sizes]
    s = torch.cuda.current_stream().cuda_stream
    hp = plan(0)
    _ghx.call("ghx_uplan_execute", hp, _ghx.ptr_array([fptr]), 1,
              _ghx.ptr_array([b.data_ptr() for b in bufs]), len(bufs), s)
    torch.cuda.synchronize()
    for l, b, sz in zip(lists, bufs, sizes):
        ob = np.zeros(sz, np.uint8)
        orc.unstructured_get(host, ob, elem, l, levels, True, index_stride, 1)
        got = b.cpu().numpy()
        assert not got[:buf_off].any(), "bytes before the buffer offset were written"
        assert np.array_equal(got[buf_off:], ob)
    hu = plan(1)
    fresh = [rng.integers(0, 256, size=buf_off + sz, dtype=np.uint8) for sz in sizes]
    rbufs = [torch.from_numpy(f).cuda() for f in fresh]
    _ghx.call("ghx_uplan_execute", hu, _ghx.ptr_array([fptr]), 1,
              _ghx.ptr_array([b.data_ptr() for b in rbufs]), len(rbufs), s)
    torch.cuda.synchronize()
    exp = host.copy()
    for l, f in zip(lists, fresh):
        orc.unstructured_set(exp, f, elem, l, levels, True, index_stride, 1, byte_offset=buf_off)
    got = dev_raw.cpu().numpy()
    assert np.array_equal(got[base:base + nbytes], exp)
    assert not got[:base].any() and not got[base + nbytes:].any(), "wrote outside the field"
    _ghx.lib().ghx_uplan_destroy(hp)
    _ghx.lib().ghx_uplan_destroy(hu)


@pytest.mark.parametrize("elem,levels,index_stride", [(8, 1, 1), (4, 1, 1), (4, 2, 2),
                                                      (2, 4, 4), (4, 1, 2), (8, 2, 2)])
@pytest.mark.parametrize("maxrun", [1, 3, 96])
@pytest.mark.parametrize("urun", [1, 0])
def test_run_lists_bit_exact(elem, levels, index_stride, maxrun, urun):
    """(8,1,1) fp64 / (4,1,1) fp32 / (4,2,2) / (2,4,4): 8-B and 4-B rows on the run path;
    (4,1,2): index stride != row length and (8,2,2): 16-B rows -> the one-row-per-lane path."""
    from ghex_amd import _ghx
    rng = np.random.default_rng(1000 * elem + 10 * levels + maxrun)
    lists = _run_lists(rng, 400_000, 3, 20_011, maxrun)
    _ghx.call("ghx_tune", b"urun", urun)
    try:
        _exchange(elem, levels, index_stride, lists)
    finally:
        _ghx.call("ghx_tune", b"reset", 0)


@pytest.mark.parametrize("elem", [8, 4])
def test_run_lists_int64_lids(elem):
    """lids >= 2^31 (int64 lid table) on the run path: every lid biased by 2^31 + 5, the field
    pointer by the opposite amount."""
    rng = np.random.default_rng(5)
    lists = _run_lists(rng, 200_000, 2, 10_007, 64)
    _exchange(elem, 1, 1, lists, lid_bias=(1 << 31) + 5)


@pytest.mark.parametrize("field_shift,buf_off", [(4, 0), (0, 8), (8, 0)])
def test_run_lists_alignment_fallbacks(field_shift, buf_off):
    """fp64 rows with a field pointer 4-B misaligned (fallback), buffer offset 8 (the planner
    keeps the one-row path), field pointer 8-B aligned only (run path, 8-B aligned accesses)."""
    rng = np.random.default_rng(11)
    lists = _run_lists(rng, 100_000, 2, 5_003, 48)
    _exchange(8, 1, 1, lists, field_shift=field_shift, buf_off=buf_off)


def test_config5_shape_with_and_without_runs():
    """BASELINE config 5's random lists (no runs) through the run path and the row path."""
    from ghex_amd import _ghx
    rng = np.random.default_rng(20260715)
    lists = np.split(rng.choice(2_000_000, size=100_000, replace=False), [10_000, 45_000, 70_001])
    for urun in (1, 0):
        _ghx.call("ghx_tune", b"urun", urun)
        try:
            _exchange(8, 1, 1, lists)
        finally:
            _ghx.call("ghx_tune", b"reset", 0)
