#!/usr/bin/env python3
"""Developer micro-benchmark: time the fused pack/unpack kernels per class of iteration space
(x/y/z faces, edges, corners) and against plain device copies, at 512^3 fp64 (or --N/--halo).

Not part of the product API and not the headline bench (see bench.py)."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--N", type=int, default=512)
    p.add_argument("--halo", type=int, default=2)
    p.add_argument("--iters", type=int, default=50)
    p.add_argument("--tune", default="", help="key=value,... passed to ghx_tune")
    a = p.parse_args()
    import torch
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    L = _ghx.lib()
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))
    N, H = a.N, a.halo
    E = N + 2 * H
    dev = torch.device("cuda", 0)
    base = torch.randn((E, E, E), dtype=torch.float64, device=dev)
    fd = R.make_field_descriptor(R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3),
                                 base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
    hg = R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3)
    recv = hg(R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3))
    # send boxes of the single periodic domain = recv boxes shifted into the interior
    send = []
    for lf, ll, gf, gl in recv:
        send.append((tuple(g for g in gf), tuple(g for g in gl)))
    recv = [(lf, ll) for lf, ll, gf, gl in recv]
    buf = torch.empty(E ** 3 * 8, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def cls(box):
        lf, ll = box
        small = [d for d in range(3) if ll[d] - lf[d] + 1 <= H]
        if len(small) == 1:
            return "face_" + "xyz"[small[0]]
        return {2: "edge", 3: "corner"}[len(small)]

    groups = {}
    for i, b in enumerate(send):
        groups.setdefault(cls(b), []).append(i)
    groups["all"] = list(range(len(send)))
    # short rows (x extent <= H: the request-bound part) vs long rows (streaming)
    groups["short_rows"] = [i for i, b in enumerate(send) if b[1][0] - b[0][0] + 1 <= H]
    groups["long_rows"] = [i for i, b in enumerate(send) if b[1][0] - b[0][0] + 1 > H]

    def plan(boxes, direction):
        arr = (_ghx.Box * len(boxes))()
        for i, (lf, ll) in enumerate(boxes):
            for d in range(3):
                arr[i].first[d], arr[i].last[d] = lf[d], ll[d]
        e = _ghx.PackEntry()
        e.field = fd.desc
        e.field_slot = e.buffer_slot = 0
        e.buffer_offset = 0
        e.boxes = ctypes.cast(arr, ctypes.POINTER(_ghx.Box))
        e.n_boxes = len(boxes)
        h = ctypes.c_void_p()
        _ghx.call("ghx_plan_create", ctypes.byref(e), 1, direction, ctypes.byref(h))
        nb = ctypes.c_uint64()
        nt = ctypes.c_int32()
        _ghx.call("ghx_plan_info", h, ctypes.byref(nb), None, ctypes.byref(nt))
        return h, nb.value, nt.value

    fp = _ghx.ptr_array([fd.data_ptr()])
    bp = _ghx.ptr_array([buf.data_ptr()])

    def time_plan(h):
        for _ in range(5):
            L.ghx_plan_execute(h, fp, 1, bp, 1, s)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.iters)]
        for e0, e1 in ev:
            e0.record()
            L.ghx_plan_execute(h, fp, 1, bp, 1, s)
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        return ts[len(ts) // 2] * 1e3  # median us

    res = {}
    for g, idx in groups.items():
        for direction, boxes in ((0, [send[i] for i in idx]), (1, [recv[i] for i in idx])):
            h, nb, nt = plan(boxes, direction)
            us = time_plan(h)
            res[f"{g}_{'pack' if direction == 0 else 'unpack'}"] = {
                "us": round(us, 2), "bytes": nb, "tiles": nt,
                "GBps_alg": round(2 * nb / us / 1e3, 1)}
            L.ghx_plan_destroy(h)
    # short-row and long-row spaces as two launches on two streams at once (does the hardware
    # overlap them better than one launch that holds both?)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    main = torch.cuda.current_stream()
    for direction, boxes in ((0, send), (1, recv)):
        hs, _, _ = plan([boxes[i] for i in groups["short_rows"]], direction)
        hl, _, _ = plan([boxes[i] for i in groups["long_rows"]], direction)

        def both():
            sa.wait_stream(main)
            sb.wait_stream(main)
            L.ghx_plan_execute(hs, fp, 1, bp, 1, sa.cuda_stream)
            L.ghx_plan_execute(hl, fp, 1, bp, 1, sb.cuda_stream)
            main.wait_stream(sa)
            main.wait_stream(sb)
        for _ in range(5):
            both()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.iters)]
        for e0, e1 in ev:
            e0.record()
            both()
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        res[f"short_long_two_streams_{'pack' if direction == 0 else 'unpack'}"] = {
            "us": round(ts[len(ts) // 2] * 1e3, 2)}
        L.ghx_plan_destroy(hs)
        L.ghx_plan_destroy(hl)
    # plain copies for reference
    for mb in (25, 50, 100, 400):
        nbytes = mb * 1024 * 1024
        x = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)
        for _ in range(5):
            y.copy_(x)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.iters)]
        for e0, e1 in ev:
            e0.record()
            y.copy_(x)
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        us = ts[len(ts) // 2] * 1e3
        res[f"d2d_copy_{mb}MiB"] = {"us": round(us, 2), "GBps_alg": round(2 * nbytes / us / 1e3, 1)}
    print(json.dumps({"N": N, "H": H, "tune": a.tune, "results": res}))


if __name__ == "__main__":
    main()
