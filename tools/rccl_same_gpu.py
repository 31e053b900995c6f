#!/usr/bin/env python3
"""Developer probe: can two RCCL ranks share one GPU (the 1-GPU test box)? Spawns `--world`
child processes (torch.distributed "nccl" backend, every rank on cuda:0) that all-reduce and
exchange one send/recv pair, and prints one JSON line per rank with what happened. A rank that
fails prints the error; the parent bounds the whole run with --timeout and kills the children's
process group when it expires.

usage: python tools/rccl_same_gpu.py [--world 2] [--timeout 60]"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    out = {"rank": rank}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        world = dist.get_world_size()
        t = torch.full((1024,), float(rank + 1), device="cuda")
        dist.all_reduce(t)
        out["all_reduce"] = float(t[0].item())
        out["all_reduce_ok"] = out["all_reduce"] == world * (world + 1) / 2
        s = torch.full((4096,), float(rank), device="cuda")
        r = torch.empty_like(s)
        ops = [dist.P2POp(dist.isend, s, (rank + 1) % world),
               dist.P2POp(dist.irecv, r, (rank - 1) % world)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize()
        out["p2p_ok"] = bool((r == float((rank - 1) % world)).all().item())
        dist.destroy_process_group()
    except Exception as e:  # report, never hang on the error path
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    print(json.dumps(out), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--world", type=int, default=2)
    p.add_argument("--timeout", type=float, default=60)
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        return child()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(a.world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child"],
                                      env=env, start_new_session=True))
    rc = 0
    for pr in procs:
        try:
            rc |= pr.wait(timeout=a.timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    os.killpg(q.pid, signal.SIGKILL)
            print(json.dumps({"timeout": a.timeout}), flush=True)
            return 124
    return rc


if __name__ == "__main__":
    sys.exit(main())
