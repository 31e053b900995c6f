#!/usr/bin/env python3
"""Developer micro-benchmark: does the unstructured index-list gather/scatter need a wave-level
ballot/prefix run detection (contiguous lid runs -> wider per-lane vectors)?

The product kernel (k_copy<seg_u>, one lane per 8-B row at levels=1 fp64) is timed on one index
list shape per line — pack (gather into a buffer) + unpack (scatter back) of n indices of a
10M-cell fp64 field, hipGraph-replayed — next to a plain device copy of the same bytes (argv:
ghx_tune settings "key=v,key=v", one pass over the shapes each):
  random    : n distinct random lids (BASELINE config 5's shape)
  sorted    : the same lids ascending (field side in address order)
  runs64    : runs of 64 consecutive lids at random run starts
  contig    : lids = offset + arange(n) (one run)
If `contig` and `runs64` already run at the streaming copy rate, the texture addresser has merged
the adjacent lanes' 8-B accesses into full-line requests and a ballot-based run detection could
only save instructions, not memory requests.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from ghex_amd import _ghx
    ncells = 10_000_000
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(20260715)
    field = torch.randn(ncells, dtype=torch.float64, device=dev)
    L = _ghx.lib()

    def plan(lids, direction):
        e = _ghx.UPackEntry()
        e.data.elem_size, e.data.levels, e.data.levels_first = 8, 1, 1
        e.data.index_stride, e.data.level_stride = 1, 1
        e.field_slot, e.buffer_slot, e.buffer_offset = 0, 0, 0
        arr = np.ascontiguousarray(lids, dtype=np.int64)
        e.lids = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        e.n_lids = len(arr)
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", ctypes.byref(e), 1, direction, ctypes.byref(h))
        return h

    def graph_time(fn, per=10, reps=30):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            fn(s.cuda_stream)
        torch.cuda.current_stream(dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(per):
                fn(torch.cuda.current_stream(dev).cuda_stream)
        g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / (reps * per)

    tunes = sys.argv[1:] or [""]
    for n in (500_000, 4_000_000):
        shapes = {}
        r = rng.choice(ncells, size=n, replace=False)
        shapes["random"] = r
        shapes["sorted"] = np.sort(r)
        starts = rng.choice(ncells // 64, size=n // 64, replace=False) * 64
        shapes["runs64"] = (starts[:, None] + np.arange(64)[None, :]).reshape(-1)
        shapes["contig"] = 1234 + np.arange(n)
        buf = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        fp = _ghx.ptr_array([field.data_ptr()])
        bp = _ghx.ptr_array([buf.data_ptr()])
        # streaming reference: the same bytes as one device copy each way
        src = torch.empty(n, dtype=torch.float64, device=dev)
        dst = torch.empty_like(src)
        t_copy = graph_time(lambda s: (dst.copy_(src), src.copy_(dst)))
        ref = 4 * n * 8 / t_copy / 1e9
        for tune, (name, lids) in ((t, x) for t in tunes for x in shapes.items()):
            _ghx.call("ghx_tune", b"reset", 0)
            for kv in filter(None, tune.split(",")):
                k, v = kv.split("=")
                _ghx.call("ghx_tune", k.encode(), int(v))
            hp, hu = plan(lids, 0), plan(lids, 1)

            def step(s):
                L.ghx_uplan_execute(hp, fp, 1, bp, 1, s)
                L.ghx_uplan_execute(hu, fp, 1, bp, 1, s)
            t = graph_time(step)
            L.ghx_uplan_destroy(hp)
            L.ghx_uplan_destroy(hu)
            lines = len(np.unique(np.asarray(lids) * 8 // 128))
            print(json.dumps({"tune": tune, "n": n, "lids": name, "us": round(t * 1e6, 2),
                              "GBps": round(4 * n * 8 / t / 1e9, 1),
                              "copy_GBps_same_bytes": round(ref, 1),
                              "field_lines": lines}), flush=True)


if __name__ == "__main__":
    main()
