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
