#!/usr/bin/env python3
"""Developer benchmark: the per-GPU step of bench.py at N = 2, 4, 8 on ONE GPU.

Rank 0 of the (2,1,1) / (2,2,1) / (2,2,2) decomposition is planned through an emulated context
(every rank's domain known, as the setup all-gather would return it); its step — pack launch +
unpack launch, the transport excluded exactly as in bench.py — is then timed from hipGraphs of 10
steps, plain (ghx_exchange_pack/unpack) and mixed (ghx_exchange_pack_self/unpack_peers: the pack
launch completes the self messages, the unpack launch covers the peer messages only). The recv
buffers hold whatever the emulated peers would have sent (their content does not change the
timing). One JSON line per (world, variant)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DECOMP = {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}


class _Ctx:
    def __init__(self, size, table):
        self._n, self._t = size, table

    def rank(self):
        return 0

    def size(self):
        return self._n

    def all_gather_object(self, obj):
        return [self._t[r] for r in range(self._n)]

    distributed = None
    group = None

    def global_rank(self, r):
        return r


def main():
    import torch
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    N, Hw = 512, 2
    E = N + 2 * Hw
    dev = torch.device("cuda", 0)
    base = torch.zeros((E, E, E), dtype=torch.float64, device=dev)
    L = _ghx.lib()
    for kv in filter(None, os.environ.get("GHX_TUNE", "").split(",")):  # e.g. GHX_TUNE=lds=1
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))
    # argv: worlds ("2") or world:decomposition ("2:1,1,2")
    for spec in sys.argv[1:] or ["1", "2", "4", "8"]:
        world = int(spec.split(":")[0])
        parts = (tuple(int(x) for x in spec.split(":")[1].split(",")) if ":" in spec
                 else DECOMP[world])
        G = [parts[d] * N for d in range(3)]
        table = {}
        for r in range(world):
            c = (r % parts[0], (r // parts[0]) % parts[1], r // (parts[0] * parts[1]))
            table[r] = [(r, tuple(c[d] * N for d in range(3)),
                         tuple((c[d] + 1) * N - 1 for d in range(3)))]
        ctx = _Ctx(world, table) if world > 1 else ghex_amd.make_context()
        dd = R.DomainDescriptor(0, table[0][0][1], table[0][0][2])
        pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), tuple(g - 1 for g in G), (Hw,) * 6,
                                                 (True,) * 3), [dd])
        fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (Hw,) * 3, (E,) * 3)
        co = R.make_communication_object(ctx)
        bis = [pc(fd)]
        plan = co.plan(bis)
        send, recv = co.buffers(plan, dev)
        fp = _ghx.ptr_array([fd.data_ptr()])
        sp = _ghx.ptr_array([t.data_ptr() for t in send])
        rp = _ghx.ptr_array([t.data_ptr() for t in recv])
        n_halo = E ** 3 - N ** 3
        variants = [("plain", L.ghx_exchange_pack, L.ghx_exchange_unpack)]
        if co.mixed(plan):
            variants.append(("mixed", L.ghx_exchange_pack_self, L.ghx_exchange_unpack_peers))
        if co.all_self(plan):
            variants.append(("fused", L.ghx_exchange_self, None))
        for name, pf, uf in variants:
            def step(s, pf=pf, uf=uf):
                pf(plan.h, fp, 1, sp, len(send), s)
                if uf is not None:
                    uf(plan.h, fp, 1, rp, len(recv), s)
            side = torch.cuda.Stream(dev)
            with torch.cuda.stream(side):
                step(side.cuda_stream)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    step(torch.cuda.current_stream(dev).cuda_stream)
            g.replay()
            torch.cuda.synchronize(dev)
            reps = 30
            t0 = time.perf_counter()
            for _ in range(reps):
                g.replay()
            torch.cuda.synchronize(dev)
            t = (time.perf_counter() - t0) / (reps * 10)
            print(json.dumps({"world": world, "decomposition": parts, "variant": name,
                              "self_bytes": sum(b["size"] for b in plan.recv if b["rank"] == 0),
                              "us_per_step": round(t * 1e6, 2),
                              "GBps_per_gpu": round(4 * n_halo * 8 / t / 1e9, 1)}), flush=True)
        if world > 1:
            timeline(torch, dev, co, plan, send, recv, fp, sp, rp, L, _ghx, world, parts)
        del co, plan, send, recv


def timeline(torch, dev, co, plan, send, recv, fp, sp, rp, L, _ghx, world, parts):
    """The pipeline's on-device timeline without the transport: every peer's buffers packed on
    its own stream (round order, as ghx_pipeline_run issues them), then every peer's buffers
    unpacked on its stream; per peer, the time from the common start event to its pack (and
    unpack) completing, medians over repetitions. Feeds the overlap model of DESIGN §5.1."""
    from ghex_amd.communication_object import peer_order
    co._split(plan)
    peers = peer_order(0, sorted({x["rank"] for x in plan.send} - {0}), world)
    streams = {p: torch.cuda.Stream(dev, priority=-1) for p in peers}
    main = torch.cuda.current_stream(dev)
    res = {p: {"pack": [], "unpack": []} for p in peers}
    alone = {}
    for p in peers:  # each peer's pack alone (nothing concurrent)
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            for i, x in enumerate(plan.send):
                if x["rank"] == p:
                    L.ghx_exchange_pack_buffer(plan.h, i, fp, 1, sp, len(send), main.cuda_stream)
            e1.record(main)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        alone[p] = sorted(ts)[10]
    for rep in range(25):
        start = torch.cuda.Event(enable_timing=True)
        start.record(main)
        done = {}
        for p in peers:
            s = streams[p]
            s.wait_event(start)
            for i, x in enumerate(plan.send):
                if x["rank"] == p:
                    L.ghx_exchange_pack_buffer(plan.h, i, fp, 1, sp, len(send), s.cuda_stream)
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            done[p] = e
        mid = torch.cuda.Event(enable_timing=True)
        for p in peers:
            main.wait_stream(streams[p])
        mid.record(main)
        udone = {}
        for p in peers:
            s = streams[p]
            s.wait_event(mid)
            for j, x in enumerate(plan.recv):
                if x["rank"] == p:
                    L.ghx_exchange_unpack_buffer(plan.h, j, fp, 1, rp, len(recv), s.cuda_stream)
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            udone[p] = e
        for p in peers:
            main.wait_stream(streams[p])
        torch.cuda.synchronize(dev)
        if rep >= 5:
            for p in peers:
                res[p]["pack"].append(start.elapsed_time(done[p]) * 1e3)
                res[p]["unpack"].append(mid.elapsed_time(udone[p]) * 1e3)
    med = lambda v: round(sorted(v)[len(v) // 2], 2)  # noqa: E731
    print(json.dumps({"world": world, "decomposition": parts, "timeline": [
        {"peer": p, "bytes": sum(x["size"] for x in plan.send if x["rank"] == p),
         "pack_alone_us": round(alone[p], 2), "pack_done_us": med(res[p]["pack"]),
         "unpack_done_us": med(res[p]["unpack"])} for p in peers]}), flush=True)


if __name__ == "__main__":
    main()
