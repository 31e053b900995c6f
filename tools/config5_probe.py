#!/usr/bin/env python3
"""Developer measurement (not product): BASELINE config 5's shape on one GPU (10M cells, 5 %
halo = 500k lids, 7 peers, random lids, seed 20260715, levels_first fp64) as plain eager
launches — the fused gather (pack) and fused scatter (unpack) of all index lists — so that a
rocprofv3 --pmc pass attributes counters per dispatch (tools/config5_pmc.sh). --time prints the
per-launch durations (libghx launch events, medians). Same inputs as bench.py bench_config5."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--levels", type=int, default=1)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--time", action="store_true")
    p.add_argument("--sorted", action="store_true", help="lids ascending within each list")
    a = p.parse_args()
    import numpy as np
    import torch
    from ghex_amd import _ghx
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(20260715)
    n, levels = 10_000_000, a.levels
    nh = n // 20
    send = rng.choice(n, size=nh, replace=False)
    recv = rng.permutation(n)[:nh]
    cuts = np.sort(rng.choice(np.arange(1, nh), size=6, replace=False))
    sl, rl = np.split(send, cuts), np.split(recv, cuts)
    if a.sorted:
        sl, rl = [np.sort(x) for x in sl], [np.sort(x) for x in rl]
    vals = torch.randn(n * levels, dtype=torch.float64, device=dev)

    def plan(lists, direction):
        ents, keep = [], []
        for k, l in enumerate(lists):
            e = _ghx.UPackEntry()
            e.data.elem_size, e.data.levels, e.data.levels_first = 8, levels, 1
            e.data.index_stride, e.data.level_stride = levels, 1
            e.field_slot, e.buffer_slot, e.buffer_offset = 0, k, 0
            arr = np.ascontiguousarray(l, dtype=np.int64)
            keep.append(arr)
            e.lids = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            e.n_lids = len(arr)
            ents.append(e)
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", (_ghx.UPackEntry * len(ents))(*ents), len(ents), direction,
                  ctypes.byref(h))
        return h

    hp, hu = plan(sl, 0), plan(rl, 1)
    bufs = [torch.empty(len(x) * levels * 8, dtype=torch.uint8, device=dev) for x in sl]
    fp = _ghx.ptr_array([vals.data_ptr()])
    bp = _ghx.ptr_array([b.data_ptr() for b in bufs])
    L = _ghx.lib()
    s = torch.cuda.current_stream(dev).cuda_stream

    def step():
        _ghx.check(L.ghx_uplan_execute(hp, fp, 1, bp, len(bufs), s), "pack")
        _ghx.check(L.ghx_uplan_execute(hu, fp, 1, bp, len(bufs), s), "unpack")
    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    if not a.time:
        for _ in range(a.iters):
            step()
        torch.cuda.synchronize(dev)
        return
    nk = 2 * a.iters
    ms = (ctypes.c_float * nk)()
    got = ctypes.c_int32()
    _ghx.call("ghx_launch_timing", 1)
    for _ in range(a.iters):
        step()
    _ghx.call("ghx_launch_timing_read", ms, nk, ctypes.byref(got))
    _ghx.call("ghx_launch_timing", 0)
    pk = sorted(ms[0:got.value:2])
    up = sorted(ms[1:got.value:2])
    print(json.dumps({"levels": levels, "lids_per_direction": nh, "sorted": a.sorted,
                      "pack_us": round(pk[len(pk) // 2] * 1e3, 2),
                      "unpack_us": round(up[len(up) // 2] * 1e3, 2),
                      "value_bytes_per_launch": 2 * nh * levels * 8}), flush=True)


if __name__ == "__main__":
    main()
