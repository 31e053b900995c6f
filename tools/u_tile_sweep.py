#!/usr/bin/env python3
"""Developer measurement (not product): the config-5 gather / scatter launches (rank 0 of 8,
lists from the product pattern, tools/config5_gen.cpp) under plan-shaping ghx_tune settings, by
the kernels' own events (ghx_launch_timing, medians of 41), beside the index-list floor probe
(tools/pack_floor.hip ghx_probe_index_floor). One JSON line per (levels, setting).
usage: python tools/u_tile_sweep.py [levels ...]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (round 5 also swept a per-lane unroll of 1/2/4 vectors, then removed: 4 was best at levels 8,
# profiles/r05_u_tile_sweep.jsonl)
SETTINGS = [{}] + [{"u_tile_bytes": tb} for tb in (8192, 16384, 32768, 65536)]


def main():
    import numpy as np
    import torch
    import bench
    from ghex_amd import _ghx
    L = _ghx.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    pats, _, _ = bench.config5_patterns()
    gids, outer, sends, recvs = pats[0]
    n = gids.size
    for levels in [int(x) for x in sys.argv[1:]] or [1, 8]:
        vals = torch.zeros(n * levels, dtype=torch.float64, device=dev)
        sb = [torch.empty(len(l) * levels * 8, dtype=torch.uint8, device=dev) for *_, l in sends]
        rb = [torch.zeros(len(l) * levels * 8, dtype=torch.uint8, device=dev) for *_, l in recvs]
        fp = _ghx.ptr_array([vals.data_ptr()])
        sp = _ghx.ptr_array([b.data_ptr() for b in sb])
        rp = _ghx.ptr_array([b.data_ptr() for b in rb])
        floor = bench.index_floor(int(n), levels, sends, recvs, 0, 0)
        for st in SETTINGS:
            _ghx.call("ghx_tune", b"reset", 0)
            for k, v in st.items():
                _ghx.call("ghx_tune", k.encode(), v)

            def plan(lists, direction):
                ents, keep = [], []
                for k, (_, _, _, l) in enumerate(lists):
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
                _ghx.call("ghx_uplan_create", (_ghx.UPackEntry * len(ents))(*ents), len(ents),
                          direction, ctypes.byref(h))
                return h
            hp, hu = plan(sends, 0), plan(recvs, 1)
            tiles = ctypes.c_int32()
            _ghx.call("ghx_uplan_info", hu, None, None, ctypes.byref(tiles))

            def g(s):
                _ghx.check(L.ghx_uplan_execute(hp, fp, 1, sp, len(sb), s), "pack")

            def sc(s):
                _ghx.check(L.ghx_uplan_execute(hu, fp, 1, rp, len(rb), s), "unpack")
            kg, ks = bench.launch_durations(torch, dev, stream, _ghx, [g, sc])
            print(json.dumps({"levels": levels, "tune": st, "unpack_tiles": tiles.value,
                              "gather_us": round(kg * 1e6, 2), "scatter_us": round(ks * 1e6, 2),
                              "floor_gather_us": floor.get("gather_us"),
                              "floor_scatter_us": floor.get("scatter_us")}), flush=True)
            L.ghx_uplan_destroy(hp)
            L.ghx_uplan_destroy(hu)
        _ghx.call("ghx_tune", b"reset", 0)


if __name__ == "__main__":
    main()
