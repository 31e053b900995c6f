#!/usr/bin/env python3
"""Developer measurement (not product): the product's pack and unpack launches (one periodic
N^3 fp64 domain, halo H, layout_map<2,1,0>, row pitch (N+2H)*8 B) by their own events
(ghx_launch_timing, medians of 41) beside the address-set floor probes of bench.pack_read_floor
(tools/pack_floor.hip), over N x H; each shape's exchange is checked cell by cell after the
timing. One JSON line per shape.
usage: python tools/floor_sweep.py [--shapes N:H,...] [--tune k=v,k=v ...]
(each --tune is one setting of ghx_tune keys; the shapes run under each; none = the defaults)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="")
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--no-floor", action="store_true", help="kernels only (no probes)")
    ap.add_argument("--alone", action="store_true",
                    help="also time each kernel back to back with itself (pack, pack, ...), the "
                         "cache state the probes are timed in")
    a = ap.parse_args()
    shapes = [tuple(int(x) for x in sh.split(":")) for sh in a.shapes.split(",") if sh] or \
        [(N, H) for N in (256, 384, 512, 640) for H in (1, 2, 3)]
    settings = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in t.split(",") if kv)
                for t in a.tune] or [{}]
    import torch
    import bench
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    L = _ghx.lib()
    for st in settings:
        _ghx.call("ghx_tune", b"reset", 0)
        for k, v in st.items():
            _ghx.call("ghx_tune", k.encode(), v)
        for N, H in shapes:
            E = N + 2 * H
            ctx = ghex_amd.make_context()
            dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
            pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6,
                                                     (True,) * 3), [dd])
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

            def pack(s):
                _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")

            def unpack(s):
                _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, sp, len(send), s), "unpack")
            kp, ku = bench.launch_durations(torch, dev, stream, _ghx, [pack, unpack])
            alone = {}
            if a.alone:
                alone["pack_alone_us"] = round(
                    bench.launch_durations(torch, dev, stream, _ghx, [pack])[0] * 1e6, 2)
                alone["unpack_alone_us"] = round(
                    bench.launch_durations(torch, dev, stream, _ghx, [unpack])[0] * 1e6, 2)
            torch.cuda.synchronize(dev)
            idx = (torch.arange(E, device=dev) - H) % N
            want = (idx.view(1, 1, E) + N * (idx.view(1, E, 1) + N * idx.view(E, 1, 1))).double()
            ok = bool((f == want).all())
            roof = {"pack_kernel_us": round(kp * 1e6, 2), "unpack_kernel_us": round(ku * 1e6, 2)}
            fl = {} if a.no_floor else bench.pack_read_floor(N, H, roof)
            n = E ** 3 - N ** 3
            print(json.dumps({
                "tune": st, "N": N, "H": H, "row_pitch_bytes": E * 8, "verified": ok,
                "pack_us": roof["pack_kernel_us"], "unpack_us": roof["unpack_kernel_us"],
                "pack_GBps": round(2 * n * 8 / kp / 1e9, 1),
                "pack_floor_us": fl.get("reads_writes_us"),
                "pack_floor_over_kernel": fl.get("floor_over_kernel"),
                "unpack_floor_us": fl.get("write_floor", {}).get("floor_us"),
                "unpack_floor_over_kernel": fl.get("write_floor", {}).get("floor_over_kernel"),
                "pack_floor_dependent_us": fl.get("reads_writes_dependent_us"),
                "pack_dependent_over_kernel": fl.get("dependent_over_kernel"),
                "xface_lines": fl.get("xface_lines"), "xface_only_us": fl.get("xface_only_us"),
                **alone}),
                flush=True)
            del f, want, send, co, bis, plan
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
