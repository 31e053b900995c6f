#!/usr/bin/env python3
"""Developer measurement (not product): the pack / unpack launches of one periodic N^3 fp64
domain (halo H, row pitch (N+2H)*8 B) split by row class — the full 26-neighbour pattern, the
x-normal halos alone (halos (H,H,0,0,0,0): the x faces, short rows only) and the y/z halos alone
((0,0,H,H,H,H): y and z faces and their edges, long rows only) — each kernel by its own events,
back to back with itself and inside the pack+unpack step. Every exchange is checked cell by
cell (halo cells of the halos in use only). One JSON line per (shape, class).
usage: python tools/class_split.py [--shapes N:H,...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLASSES = {"full": lambda H: (H,) * 6, "x_only": lambda H: (H, H, 0, 0, 0, 0),
           "yz_only": lambda H: (0, 0, H, H, H, H)}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="384:1,256:3,512:2")
    ap.add_argument("--tune", default="")
    a = ap.parse_args()
    import torch
    import bench
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    L = _ghx.lib()
    for sh in a.shapes.split(","):
        N, H = (int(x) for x in sh.split(":"))
        E = N + 2 * H
        for cname, halos in CLASSES.items():
            hl = halos(H)
            ctx = ghex_amd.make_context()
            dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
            pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, hl, (True,) * 3),
                                [dd])
            f = torch.full((E, E, E), -1.0, dtype=torch.float64, device=dev)
            ar = torch.arange(N, device=dev, dtype=torch.float64)
            f[H:H + N, H:H + N, H:H + N] = ar.view(1, 1, N) + N * (ar.view(1, N, 1) +
                                                                   N * ar.view(N, 1, 1))
            bis = [pc(R.make_field_descriptor(dd, f.permute(2, 1, 0), (H,) * 3, (E,) * 3))]
            co = R.make_communication_object(ctx)
            plan = co.plan(bis)
            send, _ = co.buffers(plan, dev)
            fp = _ghx.ptr_array([f.data_ptr()])
            sp = _ghx.ptr_array([t.data_ptr() for t in send])
            nbytes = sum(b["size"] for b in plan.send)

            def pack(s):
                _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")

            def unpack(s):
                _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, sp, len(send), s), "unpack")
            kp, ku = bench.launch_durations(torch, dev, stream, _ghx, [pack, unpack])
            pa = bench.launch_durations(torch, dev, stream, _ghx, [pack])[0]
            ua = bench.launch_durations(torch, dev, stream, _ghx, [unpack])[0]
            torch.cuda.synchronize(dev)
            # expected: the wrapped index where the halo is in use, -1 in unused halo cells
            idx = (torch.arange(E, device=dev) - H) % N
            inside = (torch.arange(E, device=dev) >= H) & (torch.arange(E, device=dev) < H + N)
            want = (idx.view(1, 1, E) + N * (idx.view(1, E, 1) + N * idx.view(E, 1, 1))).double()
            use = [inside | (hl[2 * d] > 0) for d in range(3)]  # dims x, y, z
            m = use[0].view(1, 1, E) & use[1].view(1, E, 1) & use[2].view(E, 1, 1)
            # a cell is written when every coordinate outside the interior lies in a used halo
            want = torch.where(m, want, torch.full_like(want, -1.0))
            ok = bool((f == want).all())
            print(json.dumps({"N": N, "H": H, "class": cname, "halos": hl, "verified": ok,
                              "bytes": nbytes,
                              "pack_step_us": round(kp * 1e6, 2),
                              "unpack_step_us": round(ku * 1e6, 2),
                              "pack_alone_us": round(pa * 1e6, 2),
                              "unpack_alone_us": round(ua * 1e6, 2),
                              "pack_alone_GBps": round(2 * nbytes / pa / 1e9, 1)}), flush=True)
            del f, want, send, co, bis, plan
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
