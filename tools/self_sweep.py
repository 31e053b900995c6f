#!/usr/bin/env python3
"""Developer sweep of the fused self exchange (ghx_exchange_self -> k_self) under ghx_tune knobs.

For each setting: a fresh plan (tile tables depend on the knobs), one verified exchange (every
cell of the (N+2H)^3 box against the wrapped global index), then the per-launch duration by
differencing hipGraphs of M and M+1 launches (bench.kernel_durations). One JSON line per setting.
Usage: python tools/self_sweep.py --configs '[{}, {"small_tile_rows": 512}]'"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--N", type=int, default=512)
    p.add_argument("--halo", type=int, default=2)
    p.add_argument("--configs", default="[{}]", help="JSON list of dicts of knob overrides")
    a = p.parse_args()
    import torch
    import bench
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    L = _ghx.lib()
    N, H = a.N, a.halo
    E = N + 2 * H
    dev = torch.device("cuda", 0)
    base = torch.full((E, E, E), -1.0, dtype=torch.float64, device=dev)
    ar = torch.arange(N, device=dev, dtype=torch.float64)
    base[H:H + N, H:H + N, H:H + N] = ar.view(1, 1, N) + N * (ar.view(1, N, 1) + N * ar.view(N, 1, 1))
    idx = ((torch.arange(E, device=dev) - H) % N).to(torch.float64)
    expect = idx.view(1, 1, E) + N * (idx.view(1, E, 1) + N * idx.view(E, 1, 1))
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
    stream = torch.cuda.current_stream(dev)
    nbytes = 4 * (E ** 3 - N ** 3) * 8
    for cfg in json.loads(a.configs):
        _ghx.call("ghx_tune", b"reset", 0)
        for k, v in cfg.items():
            _ghx.call("ghx_tune", k.encode(), int(v))
        co = R.make_communication_object(ctx)
        bis = [pc(fd)]
        plan = co.plan(bis)
        send, _ = co.buffers(plan, dev)
        base[:H] = -1.0
        base[:, :H] = -1.0
        base[:, :, :H] = -1.0
        co.exchange(bis).wait()
        ok = bool((base == expect).all())
        fp = _ghx.ptr_array([fd.data_ptr()])
        sp = _ghx.ptr_array([t.data_ptr() for t in send])

        def fused(s):
            rc = L.ghx_exchange_self(plan.h, fp, 1, sp, len(send), s)
            if rc:
                raise RuntimeError(L.ghx_last_error().decode())
        (t,) = bench.kernel_durations(torch, dev, stream, [fused])
        print(json.dumps(dict(cfg=cfg, verified=ok, us=round(t * 1e6, 2),
                              GBps=round(nbytes / t / 1e9, 1))), flush=True)
        del co, plan, send


if __name__ == "__main__":
    main()
