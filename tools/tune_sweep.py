#!/usr/bin/env python3
"""Developer sweep: the bench's pack+unpack step under many ghx_tune settings, in one process.

For each setting a fresh exchange plan is built (tile tables depend on the knobs) and
K steps of (pack, unpack) are timed with HIP events around each kernel (median us)."""
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
    p.add_argument("--iters", type=int, default=40)
    p.add_argument("--configs", default="", help="JSON list of dicts of knob overrides")
    a = p.parse_args()
    import torch
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    L = _ghx.lib()
    N, H = a.N, a.halo
    E = N + 2 * H
    dev = torch.device("cuda", 0)
    base = torch.randn((E, E, E), dtype=torch.float64, device=dev)
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3),
                        [dd])
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
    configs = json.loads(a.configs) if a.configs else [{}]
    s = torch.cuda.current_stream().cuda_stream
    out = []
    for cfg in configs:
        _ghx.call("ghx_tune", b"reset", 0)
        for k, v in cfg.items():
            _ghx.call("ghx_tune", k.encode(), int(v))
        co = R.make_communication_object(ctx)
        bis = [pc(fd)]
        plan = co.plan(bis)
        send, recv = co.buffers(plan, dev)
        fp = _ghx.ptr_array([fd.data_ptr()])
        sp = _ghx.ptr_array([t.data_ptr() for t in send])
        rp = _ghx.ptr_array([t.data_ptr() for t in recv])
        for _ in range(5):
            L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s)
            L.ghx_exchange_unpack(plan.h, fp, 1, rp, len(recv), s)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.iters)]
        for e in ev:
            e[0].record()
            L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s)
            e[1].record()
            L.ghx_exchange_unpack(plan.h, fp, 1, rp, len(recv), s)
            e[2].record()
        torch.cuda.synchronize()
        tp = sorted(e[0].elapsed_time(e[1]) for e in ev)[a.iters // 2] * 1e3
        tu = sorted(e[1].elapsed_time(e[2]) for e in ev)[a.iters // 2] * 1e3
        nbytes = (E ** 3 - N ** 3) * 8
        # the bench's form: hipGraphs of 10 (pack, unpack) steps, 20 replays, device time
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            gs = torch.cuda.current_stream().cuda_stream
            for _ in range(10):
                L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), gs)
                L.ghx_exchange_unpack(plan.h, fp, 1, rp, len(recv), gs)
        g.replay()
        torch.cuda.synchronize()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record()
        for _ in range(20):
            g.replay()
        g1.record()
        torch.cuda.synchronize()
        tg = g0.elapsed_time(g1) * 1e3 / 200
        out.append(dict(cfg=cfg, pack_us=round(tp, 2), unpack_us=round(tu, 2),
                        step_GBps=round(4 * nbytes / (tp + tu) / 1e3, 1),
                        graph_step_us=round(tg, 2), graph_GBps=round(4 * nbytes / tg / 1e3, 1)))
        print(json.dumps(out[-1]), flush=True)
        del co, plan


if __name__ == "__main__":
    main()
