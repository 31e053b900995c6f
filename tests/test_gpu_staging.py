"""Host staging copies on measured SDMA engines (ghex_amd.staging.Copier, libghx ghx_copier_*):
engine choice, byte-exact round trips of odd sizes and offsets, a dependent H2D started by the
copy engine behind its D2H, and the L2 acquire that makes H2D-written bytes visible to kernels
queued after it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ghex_amd
    ghex_amd.native_library()


def test_engines_are_probed_and_distinct():
    from ghex_amd.staging import Copier
    info = Copier.for_device(0).info()
    assert 0 <= info["d2h_engine"] < 4 and 0 <= info["h2d_engine"] < 4
    assert info["d2h_engine"] != info["h2d_engine"]
    assert info["d2h_GBps"] > 1 and info["h2d_GBps"] > 1 and info["both_GBps"] > 1


@pytest.mark.parametrize("n,off", [(1, 0), (17, 3), (4096, 0), (1 << 20, 8), (25362944, 0),
                                   (3_000_001, 5)])
def test_round_trip_bytes(n, off):
    import torch
    from ghex_amd.staging import Copier
    cp = Copier.for_device(0)
    rng = np.random.default_rng(n)
    src = torch.from_numpy(rng.integers(0, 256, size=n + off, dtype=np.uint8)).cuda()
    host = torch.zeros(n + off, dtype=torch.uint8, pin_memory=True)
    dst = torch.zeros(n + off, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t = cp.d2h(host.data_ptr() + off, src.data_ptr() + off, n)
    u = cp.h2d(dst.data_ptr() + off, host.data_ptr() + off, n, after=t)  # engine-side dependency
    cp.wait(u)
    cp.wait(t)
    s = torch.cuda.current_stream()
    cp.acquire(s)
    got = dst.cpu().numpy()
    np.testing.assert_array_equal(host.numpy()[off:], src.cpu().numpy()[off:])
    np.testing.assert_array_equal(got[off:], src.cpu().numpy()[off:])
    assert not got[:off].any()


def test_acquire_makes_copied_bytes_visible_to_later_kernels():
    """A kernel reads a device buffer (its lines in L2), an H2D copy replaces the bytes behind
    the caches, and after acquire() a kernel on the same stream sees the new bytes — repeated
    with changing contents."""
    import torch
    from ghex_amd.staging import Copier
    cp = Copier.for_device(0)
    n = 1 << 16
    dev = torch.zeros(n, dtype=torch.int64, device="cuda")
    host = torch.zeros(n, dtype=torch.int64, pin_memory=True)
    s = torch.cuda.current_stream()
    for k in range(1, 6):
        warm = dev.sum()  # bring the old lines into L2
        torch.cuda.synchronize()
        host.fill_(k)
        cp.wait(cp.h2d(dev.data_ptr(), host.data_ptr(), n * 8))
        cp.acquire(s)
        assert int(dev.sum().item()) == k * n, (k, int(warm.item()))
