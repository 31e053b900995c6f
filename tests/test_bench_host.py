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
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


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
