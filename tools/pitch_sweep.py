#!/usr/bin/env python3
"""Developer sweep: the bench's 512^3 H=2 step (same cells, same bytes) on fields whose x rows are
allocated wider than the 516 cells the halo needs (row pitch = 8 * x_alloc bytes): pack / unpack
kernel durations (start/stop events) and the two-launch graph step, per x_alloc. Shows how much
of the step is the x-face lines' address set (the caller's layout) rather than the kernels."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    sys.path.insert(0, ROOT)
    import bench
    L = _ghx.lib()
    N, H = 512, 2
    E = N + 2 * H
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    n = E ** 3 - N ** 3
    fill = sys.argv[2] if len(sys.argv) > 2 else "zeros"
    for xa in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                                "516,518,520,522,524,528,532,536,540,548,560,580").split(",")]:
        base = torch.zeros((E, E, xa), dtype=torch.float64, device=dev)
        if fill == "randn":
            base.normal_()
        elif fill == "index":
            base.copy_(torch.arange(base.numel(), device=dev, dtype=torch.float64).view_as(base))
        logical = base[:, :, :E].permute(2, 1, 0)
        fd = R.make_field_descriptor(dd, logical, (H,) * 3, (E,) * 3)
        co = R.make_communication_object(ctx)
        bis = [pc(fd)]
        plan = co.plan(bis)
        send, recv = co.buffers(plan, dev)
        fp = _ghx.ptr_array([fd.data_ptr()])
        sp = _ghx.ptr_array([t.data_ptr() for t in send])
        rp = _ghx.ptr_array([t.data_ptr() for t in recv])

        def pack(s):
            _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")

        def unpack(s):
            _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, rp, len(recv), s), "unpack")
        kp, ku = bench.launch_durations(torch, dev, stream, _ghx, [pack, unpack])

        def step():
            s = torch.cuda.current_stream(dev).cuda_stream
            pack(s)
            unpack(s)
        r = bench.Runner(torch, dev, stream, step, 100)
        r.prepare(100)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            e0.record(stream)
            r.run(100)
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 100)
        t = sorted(ts)[2]
        print(json.dumps({"fill": fill, "x_alloc": xa, "pitch_bytes": 8 * xa, "pack_kernel_us": round(kp * 1e6, 2),
                          "unpack_kernel_us": round(ku * 1e6, 2), "step_us": round(t, 2),
                          "step_GBps": round(4 * n * 8 / t / 1e3, 1),
                          "pack_frac": round(2 * n * 8 / kp / 1e9 / 8000, 4)}), flush=True)
        del r, co, plan, send, recv, fd, logical, base
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
