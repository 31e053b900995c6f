#!/usr/bin/env python3
"""Developer probe: the pack of the two x-normal send faces alone (16-B rows at H=2) through the
product kernel, warm, as a function of the field's x extent (row pitch) and of the number of z
planes (footprint). Per launch: graph of 20 launches, device time / 20. One JSON line per case:
us, lines (the 64-B spans' 128-B lines), G lines/s."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    import torch
    from ghex_amd import _ghx
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", default="", help="key=value,... (ghx_tune) before planning")
    ap.add_argument("--pitches", default="516,517,518,520,524,528,532", help="x extents")
    ap.add_argument("--zs", default="512,256,128,32", help="z planes")
    args = ap.parse_args()
    L = _ghx.lib()
    _ghx.call("ghx_tune", b"reset", 0)
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))
    H, NY = 2, 512
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    for ex in (int(x) for x in args.pitches.split(",")):
        for nz in (int(z) for z in args.zs.split(",")):
            ez = nz + 2 * H
            field = torch.zeros((ez, NY + 2 * H, ex), dtype=torch.float64, device=dev)
            d = _ghx.FieldDesc()
            d.dim, d.elem_size = 3, 8
            for k, e in enumerate((ex, NY + 2 * H, ez)):
                d.layout[k] = 2 - k
                d.offsets[k] = H
                d.extents[k] = e
            d.byte_strides[0], d.byte_strides[1] = 8, 8 * ex
            d.byte_strides[2] = 8 * ex * (NY + 2 * H)
            d.num_components, d.has_components = 1, 0
            nx = ex - 2 * H
            boxes = (_ghx.Box * 2)()
            for b, x0 in enumerate((0, nx - H)):
                boxes[b].first[0], boxes[b].last[0] = x0, x0 + H - 1
                boxes[b].first[1], boxes[b].last[1] = 0, NY - 1
                boxes[b].first[2], boxes[b].last[2] = 0, nz - 1
            e = _ghx.PackEntry()
            e.field, e.field_slot, e.buffer_slot, e.buffer_offset = d, 0, 0, 0
            e.boxes, e.n_boxes = ctypes.cast(boxes, ctypes.POINTER(_ghx.Box)), 2
            h = ctypes.c_void_p()
            _ghx.call("ghx_plan_create", ctypes.byref(e), 1, 0, ctypes.byref(h))
            buf = torch.empty(2 * NY * nz * H * 8, dtype=torch.uint8, device=dev)
            fp, bp = _ghx.ptr_array([field.data_ptr()]), _ghx.ptr_array([buf.data_ptr()])
            L.ghx_plan_execute(h, fp, 1, bp, 1, s.cuda_stream)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    L.ghx_plan_execute(h, fp, 1, bp, 1, torch.cuda.current_stream().cuda_stream)
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            us = sorted(ts)[3]
            # distinct 128-B lines holding the packed pieces
            import numpy as np
            pitch = 8 * ex
            z, y = np.meshgrid(np.arange(nz), np.arange(NY), indexing="ij")
            row = (z + H) * pitch * (NY + 2 * H) + (y + H) * pitch
            parts = []
            for x0 in (H, nx):  # first byte of each piece (x index incl. offset)
                a = row + x0 * 8
                parts += [a // 128, (a + 8 * H - 1) // 128]
            lines = np.unique(np.concatenate([p.ravel() for p in parts]))
            print(json.dumps({"tune": args.tune, "x_extent": ex, "pitch": pitch, "z_planes": nz, "us": round(us, 2),
                              "lines": len(lines), "Glines_per_s": round(len(lines) / us / 1e3, 1),
                              "footprint_MB": round(field.numel() * 8 / 1e6, 1)}), flush=True)
            L.ghx_plan_destroy(h)
            del field, buf, g


if __name__ == "__main__":
    main()
