#!/usr/bin/env python3
"""Developer measurement (not product): a short program to run under rocprofv3 --pmc
(tools/pmc_ifetch.sh): one periodic N^3 fp64 domain, halo H; `reps` pack + unpack steps, then
`reps` pack launches back to back, then `reps` unpack launches, then the pack's address-set probe
(tools/pack_floor.hip k_lines: per variant j = 0..4 2*5 warm launches and 5 after a cache sweep),
so that the per-kernel counters of the product launches and of the probe come from one process
(tools/parse_pmc_l2.py splits them by position).
usage: python tools/launch_anatomy.py N H [reps] [k=v,k=v (ghx_tune)]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    N, H = int(sys.argv[1]), int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    import ctypes
    import torch
    import bench
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    L = _ghx.lib()
    for kv in filter(None, (sys.argv[4] if len(sys.argv) > 4 else "").split(",")):
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))
    E = N + 2 * H
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    f = torch.zeros((E, E, E), dtype=torch.float64, device=dev)
    bis = [pc(R.make_field_descriptor(dd, f.permute(2, 1, 0), (H,) * 3, (E,) * 3))]
    co = R.make_communication_object(ctx)
    plan = co.plan(bis)
    send, _ = co.buffers(plan, dev)
    fp = _ghx.ptr_array([f.data_ptr()])
    sp = _ghx.ptr_array([t.data_ptr() for t in send])
    for _ in range(reps):  # the step: pack, unpack, pack, ... (launches 0..2*reps-1)
        _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")
        _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, sp, len(send), s), "unpack")
    for _ in range(reps):  # then each alone, back to back
        _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")
    for _ in range(reps):
        _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, sp, len(send), s), "unpack")
    torch.cuda.synchronize(dev)
    lib = bench._floor_lib()
    us = (ctypes.c_double * 10)()
    c = (ctypes.c_int64 * 3)()
    rc = lib.ghx_probe_pack_floor(N, H, 5, us, c)
    print("probe rc", rc, [round(x, 2) for x in us[:8]])


if __name__ == "__main__":
    main()
