"""bench.py's contract on the GPU box, at a small size: one JSON line with the metric's fields, the
roofline / cpu-free extras, a verified exchange; and the N>1 path through bench.py's own rank
spawning (`--gpus 2 --rehearse`: both ranks on the one GPU, gloo + host staging, the pipelined
exchange included). Each run is a child process bounded by a timeout."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bench(*args, timeout=150):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_n1_small():
    d = _bench("--N", "64", "--steps", "12", "--warmup", "3", "--no-cpu-baseline")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["verified"] is True and d["n_gpus"] == 1 and d["steps"] == 12 and d["warmup"] == 3
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["launch_us"] > 0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["algorithmic_bytes_per_launch"] == 2 * (68 ** 3 - 64 ** 3) * 8
    assert "cold_clean_launch_us" in r and "cold_clean_step_us" in r and "fused_self" in d
    # the dominant launch's share of the step comes from the kernels' own start/stop events
    assert r["pack_kernel_us"] > 0 and r["unpack_kernel_us"] > 0
    assert r["launch_us"] <= r["step_device_us"]
    assert d["fused_self"]["bytes_moved"] == 3 * (68 ** 3 - 64 ** 3) * 8
    assert "extras_error" not in d, d.get("extras_error")
    # `verified` is the timed graph (k_copy pack + unpack) replayed on reset halos and buffers;
    # the fused first exchange is reported separately
    assert d["verified_fused"] is True and "timed hipGraph" in d["verified_what"]
    for h, x in d["halo_widths"].items():
        assert x["verified"] is True and x["verified_fused"] is True, h
    c = r["cold_clean_kernel_events_us"]
    assert c["pack"] > 0 and c["unpack"] > 0 and c["step_pack"] > 0 and c["step_unpack"] > 0
    # the other BASELINE configs: each verifies the launches it times
    ex = d["extra_configs"]
    c4 = ex["config4_5fields_256^3_h3_f64f32"]
    assert c4["verified"] is True and c4["verified_fused"] is True and "timed hipGraph" in \
        c4["verified_what"]
    fl = c4["floor"]  # the five-field floor probe beside the two launches
    assert "error" not in fl, fl
    assert fl["pack_floor_over_kernel"] > 0 and fl["unpack_floor_over_kernel"] > 0
    assert fl["halo_bytes"] * 4 == c4["bytes_per_exchange"]
    for lv in (1, 8):
        c5 = ex[f"config5_unstructured_10M_5pct_levels{lv}"]
        assert c5["verified"] is True and c5["halo_cells"] == 500_000 and c5["peers"] == 7, c5
        assert "cpu_baseline" not in c5  # --no-cpu-baseline
        assert "error" not in c5["index_floor"] and c5["index_floor"]["gather_us"] > 0, c5
    assert ex["config5_pattern_setup"]["ranks"] == 8


def test_bench_spawns_two_ranks_rehearsal():
    d = _bench("--gpus", "2", "--rehearse", "--N", "64", "--steps", "10", "--warmup", "2",
               "--no-cold", timeout=240)
    assert d["n_gpus"] == 2 and d["verified"] is True and d["verified_fused"] is True
    assert "transported into the receive buffers" in d["verified_what"]
    for h, x in d["halo_widths"].items():
        assert x["verified"] is True, h
    assert d["config"]["decomposition"] == [2, 1, 1] and d["config"]["world_size"] == 2
    assert d["exchange_pipelined"]["verified"] is True
    u = d["unstructured_exchange"]
    assert u.get("verified") is True and u["cells_per_rank"] == 10_000_000, u
    assert u["halo_cells_per_rank"] == 500_000 and u["setup_s"] < 60, u
    assert "extras_error" not in d, d.get("extras_error")


def test_launch_timing_records_each_kernel():
    """ghx_launch_timing: one start/stop pair per kernel launch of this thread, durations > 0,
    nothing recorded once disabled."""
    import ctypes
    import torch
    from ghex_amd import _ghx
    L = _ghx.lib()
    t = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    b = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    d = _ghx.FieldDesc()
    d.dim, d.elem_size, d.num_components = 1, 1, 1
    d.layout[0], d.offsets[0], d.extents[0], d.byte_strides[0] = 0, 0, t.numel(), 1
    box = _ghx.Box()
    box.first[0], box.last[0] = 4096, 4096 + b.numel() - 1
    s = torch.cuda.current_stream().cuda_stream
    ms = (ctypes.c_float * 8)()
    n = ctypes.c_int32()
    _ghx.call("ghx_launch_timing", 1)
    try:
        for _ in range(3):
            _ghx.call("ghx_structured_pack", ctypes.byref(d), t.data_ptr(), b.data_ptr(),
                      ctypes.byref(box), 1, s)
        _ghx.call("ghx_launch_timing_read", ms, 8, ctypes.byref(n))
        assert n.value == 3 and all(0 < ms[i] < 100 for i in range(3))
        _ghx.call("ghx_launch_timing_read", ms, 8, ctypes.byref(n))
        assert n.value == 0
    finally:
        _ghx.call("ghx_launch_timing", 0)
    _ghx.call("ghx_structured_pack", ctypes.byref(d), t.data_ptr(), b.data_ptr(),
              ctypes.byref(box), 1, s)
    _ghx.call("ghx_launch_timing_read", ms, 8, ctypes.byref(n))
    assert n.value == 0
    torch.cuda.synchronize()
    assert torch.equal(b, t[4096:4096 + b.numel()])
