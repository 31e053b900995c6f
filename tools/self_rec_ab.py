#!/usr/bin/env python3
"""Developer A/B (not product): the fused self exchange (k_self, the N=1 product exchange) and
the two-launch step with a 0/1 knob off / on (--knob, default tile_records; the plans are
rebuilt per setting), interleaved rounds, kernels' own events (bench.launch_durations, medians), one periodic
512^3 fp64 domain per halo width, every exchange verified. One JSON line per (round, setting, H).
usage: python tools/self_rec_ab.py [--rounds 2] [--halos 1,2,3] [--knob tile_records]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--halos", default="1,2,3")
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--knob", default="tile_records")
    a = ap.parse_args()
    import torch

    import bench
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    L = _ghx.lib()
    N = a.N
    for rnd in range(a.rounds):
        for rec in (0, 1) if rnd % 2 == 0 else (1, 0):
            _ghx.call("ghx_tune", a.knob.encode(), rec)
            for H in (int(h) for h in a.halos.split(",")):
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

                def fused(s):
                    _ghx.check(L.ghx_exchange_self(plan.h, fp, 1, sp, len(send), s), "self")

                def pack(s):
                    _ghx.check(L.ghx_exchange_pack(plan.h, fp, 1, sp, len(send), s), "pack")

                def unpack(s):
                    _ghx.check(L.ghx_exchange_unpack(plan.h, fp, 1, sp, len(send), s), "unpack")
                ks, kp, ku = bench.launch_durations(torch, dev, stream, _ghx, [fused, pack, unpack])
                idx = (torch.arange(E, device=dev) - H) % N
                want = (idx.view(1, 1, E) + N * (idx.view(1, E, 1) + N * idx.view(E, 1, 1))).double()
                f[:H] = -1.0
                fused(stream.cuda_stream)
                torch.cuda.synchronize(dev)
                ok = bool((f == want).all())
                print(json.dumps({"round": rnd, a.knob: rec, "N": N, "H": H,
                                  "self_us": round(ks * 1e6, 2), "pack_us": round(kp * 1e6, 2),
                                  "unpack_us": round(ku * 1e6, 2), "verified": ok}), flush=True)
                del f, want, send, co, bis, plan
                torch.cuda.empty_cache()
    _ghx.call("ghx_tune", b"reset", 0)


if __name__ == "__main__":
    main()
