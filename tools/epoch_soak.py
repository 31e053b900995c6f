#!/usr/bin/env python3
"""Developer soak (GPU box): the device-epoch protocols of the zero-copy exchanges under skew.
Runs tests/mp_exchange_worker.py's race / graph modes (every exchange ordered on the stream
only, halos rewritten and checked on the device between exchanges, factors cycling with period
5 so a value of another exchange is caught) with many exchanges per run and GHX_SOAK_JITTER=1
(each rank queues 0-3 seeded busy kernels before every exchange, so the ranks drift apart and
only the epochs keep them in step). Modes: directrace / directgraph (the one-launch close with
double-buffered receive buffers), directmany (70 fields, launch groups), bulkrace / bulkgraph
(open + close around the puts); and a negative control, directnoepoch (the direct race loop with
the epoch launch left out), which must report bad cells. All processes on the one GPU (at most 8, within the box's
process bound). One progress line per case on stderr, one JSON summary on stdout.
usage: python tools/epoch_soak.py --reps 150 --seconds 500"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "mp_exchange_worker.py")

CASES = [
    ((2, 1, 1), 16, 2, "directrace"),
    ((2, 2, 1), 12, 3, "directrace"),
    ((2, 2, 1), 12, 3, "directgraph"),
    ((2, 2, 2), 8, 2, "directrace"),
    ((2, 2, 2), 8, 1, "directgraph"),
    ((2, 1, 1), 6, 1, "directmany"),
    ((2, 2, 1), 12, 3, "bulkrace"),
    ((2, 2, 1), 12, 2, "bulkgraph"),
    ((2, 2, 2), 8, 2, "bulkrace"),
]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_case(parts, N, Hw, mode, reps, timeout):
    world = parts[0] * parts[1] * parts[2]
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK="0", GHX_SOAK_JITTER="1")
        procs.append(subprocess.Popen(
            [sys.executable, WORKER, *map(str, parts), str(N), str(Hw), str(reps), mode],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs, codes = [], []
    t0 = time.time()
    for p in procs:
        try:
            out, _ = p.communicate(timeout=max(1.0, timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            for q in procs:
                q.wait()
            return {"ok": False, "error": "timeout"}
        outs.append(out)
        codes.append(p.returncode)
    ok = codes == [0] * world and "bad cells 0" in outs[0]
    rec = {"ok": ok, "seconds": round(time.time() - t0, 1)}
    import re
    m = re.search(r"bad cells (\d+)", outs[0])
    rec["bad_cells"] = int(m.group(1)) if m else None
    if not ok:
        rec["codes"] = codes
        rec["tail"] = [o[-600:] for o in outs]
    return rec


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=150)
    p.add_argument("--seconds", type=float, default=500)
    p.add_argument("--case-timeout", type=float, default=240)
    a = p.parse_args()
    t0 = time.time()
    out = {"reps": a.reps, "jitter": "0-3 seeded busy kernels per rank per exchange", "cases": []}
    for parts, N, Hw, mode in CASES:
        if time.time() - t0 > a.seconds:
            break
        # exchanges per run: the worker's loops run 4*reps (race), 3*reps (graph) or 2*reps
        # (directmany) exchanges for each of its two field layouts
        per = {"directmany": 2, "bulkgraph": 3, "directgraph": 4}.get(mode, 4)
        rec = run_case(parts, N, Hw, mode, a.reps if mode != "directmany" else max(1, a.reps // 10),
                       a.case_timeout)
        rec.update(parts=list(parts), N=N, H=Hw, mode=mode,
                   exchanges=2 * per * (a.reps if mode != "directmany" else max(1, a.reps // 10)))
        out["cases"].append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
        if rec.get("error") == "timeout":
            break  # a hung GPU step: start nothing more
    out["all_ok"] = all(c["ok"] for c in out["cases"])
    if time.time() - t0 < a.seconds and out["all_ok"]:
        neg = run_case((2, 2, 1), 12, 3, "directnoepoch", a.reps, a.case_timeout)
        out["negative_control"] = {"mode": "directnoepoch", "parts": [2, 2, 1], "N": 12, "H": 3,
                                   "bad_cells": neg.get("bad_cells"),
                                   "detected": bool(neg.get("bad_cells"))}
        print(json.dumps(out["negative_control"]), file=sys.stderr, flush=True)
    out["seconds"] = round(time.time() - t0, 1)
    print(json.dumps(out), flush=True)
    return 0 if out["all_ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
