"""bench.py's host side without a GPU: argument contract and the rank-spawning parent's failure
path (a rank that dies takes the others down and the parent exits non-zero instead of waiting
forever). The GPU legs are in tests/test_gpu_bench.py."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_spawned_ranks_fail_fast_without_a_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("this checks the failure path; a GPU would run the bench")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0", "--N", "8"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode != 0
    # no measurement: at most rank 0's line with value null and the failing stage's error
    import json
    for l in [l for l in p.stdout.splitlines() if l.startswith("{")]:
        d = json.loads(l)
        assert d["value"] is None and d["verified"] is False and "failed" in d["error"], d


def test_a_failing_stage_prints_a_null_line():
    """Single rank without a GPU: the first stage raises; the line still comes out (value null,
    the stage and its error) and the process fails."""
    import json
    import torch
    if torch.cuda.is_available():
        pytest.skip("this checks the failure path; a GPU would run the bench")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1",
                        "--warmup", "0", "--no-extras"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode != 0
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] is None and d["stage"] == "init_process_group" and "HIP" in d["error"]


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stdout + p.stderr)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_init_timeout_prints_unverified_line_and_exits_nonzero():
    """rank 0 of a 2-rank job whose peer never starts hangs in the process
    group's rendezvous; the stage guard prints the line with verified=false and an error naming
    the stage, and exits non-zero (no retry, no re-exec)."""
    import json
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--rehearse", "--init-timeout", "6"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    o = json.loads(lines[0])
    assert o["verified"] is False and o["value"] is None
    assert o["stage"] == "init_process_group" and "init_process_group" in o["error"]
    assert o["n_gpus"] == 2 and o["metric"].startswith("device-resident halo pack+unpack")


@pytest.mark.parametrize("rank", [0, 1])
def test_exchange_timeout_prints_unverified_line_and_exits_nonzero(rank):
    """The same guard around the verified full exchange (the first RCCL traffic between GPUs):
    a stage that never finishes ends the process with status 3; rank 0 prints the line on
    stdout, other ranks report on stderr only."""
    import json
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "g = bench.StageGuard({'metric': bench.METRIC, 'n_gpus': 8}, %d); "
            "c = g.stage('verified_exchange', 2); c.__enter__(); time.sleep(60)") % (ROOT, rank)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 3
    out = [l for l in p.stdout.splitlines() if l.startswith("{")]
    err = [l for l in p.stderr.splitlines() if l.startswith("{")]
    o = json.loads((out if rank == 0 else err)[0])
    assert (len(out), len(err)) == ((1, 0) if rank == 0 else (0, 1))
    assert o["verified"] is False and o["stage"] == "verified_exchange"
    assert "verified_exchange" in o["error"] and f"rank {rank}" in o["error"]


def test_stage_guard_is_silent_when_the_stage_finishes():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "g = bench.StageGuard({'metric': bench.METRIC}, 0)\n"
            "with g.stage('init_process_group', 1.5): time.sleep(0.1)\n"
            "time.sleep(3); print('survived')") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout.strip() == "survived"


def test_read_floor_probe_reports_instead_of_failing_without_a_gpu():
    """roofline.read_floor (tools/lib/libpackfloor.so) is a developer measurement: without a
    device (or without the library) it reports an error entry, never an exception. Runs in a
    child process (the probe's HIP runtime stays out of the test runner)."""
    code = ("import sys, json; sys.path.insert(0, %r); import bench; "
            "print(json.dumps(bench.pack_read_floor(8, 1, {'pack_kernel_us': 1.0})))") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-500:]
    out = __import__("json").loads(p.stdout.strip().splitlines()[-1])
    assert "error" in out


def test_isolated_bulk_leg_reports_a_failed_child():
    """bench.py's zero-copy leg at N>1 runs in child processes: a child that fails (here: no GPU)
    becomes an error entry in the line; the rank itself carries on."""
    code = ("import sys, json, types; sys.path.insert(0, %r); import bench\n"
            "a = types.SimpleNamespace(steps=5, N=8, halo=1, bulk_timeout=60.0)\n"
            "print(json.dumps(bench.bulk_isolated(a, 0, 2, 0, 29517, 60.0)))") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-500:]
    out = __import__("json").loads(p.stdout.strip().splitlines()[-1])
    assert out["isolated"] and "error" in out


def _bench():
    import importlib
    import sys as _s
    if ROOT not in _s.path:
        _s.path.insert(0, ROOT)
    return importlib.import_module("bench")


def test_cpu_rank_count_caps_and_reasons():
    """cpu_baseline.ranks: one rank per core of the affinity set, capped by the CPU quota, the
    box's declared CPU share (OMP_NUM_THREADS) and host memory; the binding cap is named."""
    b = _bench()
    share = list(range(256))
    per = 1_100_000_000
    n, why = b.cpu_rank_count(share, per, env={}, quota=None, avail=None)
    assert n == b.CPU_RANKS_MEM_BUDGET // per and "host memory" in why[0]
    n, why = b.cpu_rank_count(share, per, env={"OMP_NUM_THREADS": "16"}, quota=None,
                              avail=1 << 40)
    assert n == 16 and "OMP_NUM_THREADS=16" in why[0]
    n, why = b.cpu_rank_count(share, per, env={"OMP_NUM_THREADS": "16"}, quota=8, avail=None)
    assert n == 8 and why == ["cgroup CPU quota 8 cores"]
    n, why = b.cpu_rank_count(list(range(4)), 1000, env={}, quota=None, avail=1 << 40)
    assert n == 4 and why == ["affinity set 4 cores"]
    # available memory halves the budget when it is the smaller
    n, _ = b.cpu_rank_count(share, per, env={}, quota=None, avail=10 * per)
    assert n == 5


def test_median_of_25_drops_the_first_five():
    b = _bench()
    times = [100.0] * 5 + [float(i) for i in range(1, 21)] + [1000.0] * 7
    assert b._median_of_25(times) == 11.0  # of 1..20 (sorted, upper median)


def test_verify_replay_resets_before_the_timed_replay():
    """`verified` counts cells after the TIMED kernels alone: halos reset and every buffer byte
    set to 0xFF before the replay, then the optional delivery (N>1), then the check."""
    import types

    import torch
    b = _bench()
    calls = []
    send = [torch.zeros(8, dtype=torch.uint8), torch.zeros(4, dtype=torch.uint8)]
    recv = [send[0], torch.zeros(6, dtype=torch.uint8)]

    def replay():
        assert all(int(t.min()) == 255 for t in send + recv)
        calls.append("replay")

    fake = types.SimpleNamespace(cuda=types.SimpleNamespace(
        synchronize=lambda dev: calls.append("sync")))
    bad = b.verify_replay(fake, None, replay, lambda: calls.append("clear"),
                          lambda: calls.append("check") or 7, send, recv,
                          lambda: calls.append("deliver"))
    assert bad == 7
    # N>1: the timed graph is replayed again after the transport, so the peer halos are
    # written by its own unpack launch
    assert calls == ["clear", "replay", "deliver", "replay", "sync", "check"]
    calls.clear()
    assert b.verify_replay(fake, None, replay, lambda: calls.append("clear"),
                           lambda: calls.append("check") or 0, send, recv) == 0
    assert calls == ["clear", "replay", "sync", "check"]


def test_read_floor_keys_say_floor_over_kernel():
    """The floor ratios are floor time / kernel time and are named so."""
    import ctypes
    import types
    b = _bench()

    def probe(N, H, reps, us, c):
        for i in range(10):
            us[i] = 10.0 + i
        for i in range(3):
            c[i] = 100 + i
        return 0
    fake = types.SimpleNamespace(ghx_probe_pack_floor=probe, ghx_probe_unpack_floor=probe)
    orig = b._floor_lib
    b._floor_lib = lambda: fake
    try:
        out = b.pack_read_floor(8, 1, {"pack_kernel_us": 8.0, "unpack_kernel_us": 32.0})
    finally:
        b._floor_lib = orig
    assert out["floor_over_kernel"] == round(16.0 / 8.0, 3)
    # the unpack floor is its write set alone (us[4]); the reads-included probes beside it
    assert out["write_floor"]["floor_over_kernel"] == round(14.0 / 32.0, 3)
    assert out["write_floor"]["floor_us"] == 14.0
    assert out["write_floor"]["writes_reads_us"] == 16.0
    assert out["write_floor"]["writes_reads_interleaved_us"] == 18.0
    assert not any("vs_floor" in k for k in list(out) + list(out["write_floor"]))
    del ctypes


def test_cold_launch_durations_flush_precedes_every_timed_step():
    """roofline.cold_clean_kernel_events_us: each eager step is flush, then the timed launches;
    medians of the kernels' own events per launch."""
    import types
    b = _bench()
    order = []

    class G:
        @staticmethod
        def call(name, *a):
            order.append(name)
            if name == "ghx_launch_timing_read":
                ms, n, got = a
                for i in range(n):
                    ms[i] = 1.0 if i % 2 == 0 else 3.0
                got._obj.value = n
    fake = types.SimpleNamespace(cuda=types.SimpleNamespace(synchronize=lambda d: None))
    stream = types.SimpleNamespace(cuda_stream=0)
    p, u = b.cold_launch_durations(fake, None, stream, G, [lambda s: order.append("pack"),
                                                           lambda s: order.append("unpack")],
                                   lambda s: order.append("flush"), reps=3)
    assert (p, u) == (1e-3, 3e-3)
    timed = order[order.index("ghx_launch_timing"):]
    assert timed[1:10] == ["flush", "pack", "unpack"] * 3


def test_bulk_only_mode_reports_failed_children():
    """`bench.py --bulk-only N` spawns N isolated zero-copy children (no headline ranks); here
    (no GPU) they fail: the parent prints rank 0's line with the errors and exits 1."""
    import json
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--bulk-only", "2",
                        "--N", "8", "--halo", "1", "--bulk-timeout", "90"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 1, p.stderr[-800:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    o = json.loads(lines[0])
    assert o["mode"] == "bulk-only" and o["n_procs"] == 2 and "error" in o


def test_config5_patterns_small_and_cpu_baseline_keys():
    """config5_patterns (8 ranks' product make_pattern as threads) at a small size: every peer's
    send list to rank 0 carries rank 0's receive gids; cpu_baseline_config5's keys, and its
    bit-exact check against (here: numpy-computed) GPU buffers, including a detected mismatch."""
    import numpy as np
    import bench
    pats, t_all, t_rank = bench.config5_patterns(world=8, cells=4000)
    gids, outer, sends, recvs = pats[0]
    assert len(sends) == 7 and len(recvs) == 7 and sum(len(l) for *_, l in recvs) == 200
    for rid, rr, tag, lids in recvs:
        pg, _, psend, _ = pats[rr]
        plids = next(l for (i, q, tg, l) in psend if q == 0 and tg == tag)
        assert np.array_equal(pg[plids], gids[lids])
    levels = 8
    host = gids.astype(np.float64)[:, None] * 100.0 + np.arange(levels)[None, :]
    peer = [np.ascontiguousarray(host[l]).view(np.uint8).reshape(-1) for *_, l in recvs]
    gpu = [np.ascontiguousarray(host[l]).view(np.uint8).reshape(-1) for *_, l in sends]
    r = bench.cpu_baseline_config5(0.05, host, sends, recvs, peer, gpu, levels)
    for k in ("value", "unit", "cores", "kind", "sample", "matches_gpu", "median_of_25_GBps"):
        assert k in r, k
    assert r["matches_gpu"] is True and r["cores"] == 1 and r["kind"] == "port"
    gpu[3] = gpu[3].copy()
    gpu[3][5] ^= 1
    assert bench.cpu_baseline_config5(0.01, host, sends, recvs, peer, gpu, levels)["matches_gpu"] \
        is False


def test_cpu_baseline_config4_keys_and_parity_check():
    """cpu_baseline_config4 on the full config-4 exchange: keys, and its field-byte comparison
    with a packed message (here the oracle's own: equal; one flipped byte: detected)."""
    import numpy as np
    import bench
    from oracle import oracle as orc
    N, H = 256, 3
    E = N + 2 * H
    dom = orc.RegularDomain(0, (0, 0, 0), (N - 1,) * 3)
    pat = orc.regular_make_pattern([[dom]], (0, 0, 0), (N - 1,) * 3, (H,) * 6, (1, 1, 1))[0][0]
    val = np.arange(N ** 3, dtype=np.float64).reshape(N, N, N)
    specs = []
    for k, t in enumerate(bench.CONFIG4_TYPES):
        dt = np.float64 if t == "f64" else np.float32
        a = np.full((E, E, E), -1, dtype=dt)
        a[H:H + N, H:H + N, H:H + N] = ((val + k) % (1 << 23)).astype(dt)
        specs.append(orc.FieldSpec(a, a.itemsize, (2, 1, 0), (H,) * 3, (E,) * 3))
    items = [(k, 0, pat, sp.elem, sp.elem, 1, 0) for k, sp in enumerate(specs)]
    (sb,) = orc.plan_buffers(items, receive=False).values()
    buf = np.zeros(sb.size, np.uint8)
    for pf in sb.fields:
        orc.structured_pack(specs[pf.field_index], buf, pf.boxes, pf.offset)
    r = bench.cpu_baseline_config4(0.05, buf)
    for k in ("value", "unit", "cores", "kind", "sample", "matches_gpu", "median_of_25_GBps"):
        assert k in r, k
    assert r["matches_gpu"] is True and r["value"] > 0
    buf[sb.fields[2].offset + 11] ^= 1
    assert bench.cpu_baseline_config4(0.01, buf)["matches_gpu"] is False


def record_errors(o, path=""):
    """Every key of a bench record that reports a failure ("error" or "*_error", non-empty),
    with its path: a rehearsal leg that errored must never be summarised as verified (VERDICT
    r05 #2). Skipped legs say "skipped", not "error"."""
    out = []
    if isinstance(o, dict):
        for k, v in o.items():
            p = f"{path}.{k}" if path else k
            if (k == "error" or k.endswith("_error")) and v:
                out.append((p, str(v)[:200]))
            out += record_errors(v, p)
    elif isinstance(o, list):
        for i, v in enumerate(o):
            out += record_errors(v, f"{path}[{i}]")
    return out


def _record_line(path):
    import json
    lines = [l for l in open(path) if l.startswith("{")]
    assert lines, path
    return json.loads(lines[-1])


def test_record_errors_finds_nested_errors():
    rec = {"value": 1, "bulk": {"isolated": True, "error": "exit 1: ghx_put_create failed"},
           "extras": [{"transport_error": "x"}, {"skipped": "budget"}], "ok": {"error": ""}}
    assert [p for p, _ in record_errors(rec)] == ["bulk.error", "extras[0].transport_error"]


def test_latest_rehearsal_records_carry_no_error():
    """The committed rehearsal records of the latest round (profiles/rNN*_rehearse_n*.json and
    the isolated zero-copy legs rNN*_bulk_n*.json): no leg errored, and the zero-copy legs (puts
    and the direct exchange) verified at N = 4 and 8 — the check that would have caught round
    5's refused 512^3 put plans (profiles/r05h_rehearse_n4.json)."""
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_rehearse_n*.json")) + \
        glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_bulk_n*.json"))
    rnd = max(re.match(r"r(\d\d)", os.path.basename(f)).group(1) for f in files)
    latest = [f for f in files if os.path.basename(f).startswith(f"r{rnd}")]
    bulk_ok = set()
    for f in latest:
        rec = _record_line(f)
        assert record_errors(rec) == [], (os.path.basename(f), record_errors(rec))
        b = rec.get("bulk", rec if rec.get("mode") == "bulk-only" else None)
        if b and b.get("verified") and b.get("direct", {}).get("verified"):
            bulk_ok.add(rec.get("n_procs", rec.get("n_gpus")))
    assert {4, 8} <= bulk_ok, (rnd, sorted(bulk_ok))
    rec5 = _record_line(os.path.join(ROOT, "profiles", "r05h_rehearse_n4.json"))
    assert [p for p, _ in record_errors(rec5)] == ["bulk.error"]  # the check sees round 5's
