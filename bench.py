#!/usr/bin/env python3
"""bench.py — device-resident halo pack+unpack GB/s (BASELINE.json metric) on MI355X.

Workload (BASELINE configs[1], weak-scaled for N>1 as configs[2]): per GPU one 512^3 fp64 domain
(extent 516^3 with halo 2), 26-neighbour periodic halo. N=1: one periodic domain (all 26
iteration spaces are a self message); N=2/4/8: (2,1,1)/(2,2,1)/(2,2,2) decomposition of the
periodic global grid, one rank per GPU.

A step = the product's exchange step minus transport, fields and buffers resident in HBM: for
N>1 one fused pack launch (every iteration space of every send buffer) + one fused unpack launch
(every recv buffer); at N=1 every message is a self message and the communication object runs
pack+unpack as ONE launch (ghx_exchange_self: each workgroup packs a tile of the buffer, then
unpacks the same bytes; `--unfused` times the two-launch form, also reported as "unfused").
Algorithmic bytes per step per GPU = 4 * n * 8 (pack read + write, unpack read + write),
n = (N+2H)^3 - N^3 halo cells. value = sum over ranks of bytes*K / max over ranks of the K-step
wall time; the K steps replay hipGraphs of --steps-per-graph steps.

Before timing, one full exchange (pack -> RCCL send/recv over xGMI for N>1 -> unpack) is run and
every cell of every rank's (N+2H)^3 box is verified on the GPU against the wrapped global index.
Extra fields: the full exchange time (incl. RCCL), the host-staged rate (pack + D2H + H2D +
unpack through pinned memory), per-kernel HIP-event durations, and on rank 0 at N=1 the oracle's
single-thread CPU pack+unpack on a bounded sample (cpu_baseline).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident halo pack+unpack GB/s, 512^3 fp64 halo=2, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
DECOMP = {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--N", type=int, default=512)
    p.add_argument("--halo", type=int, default=2)
    p.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph")
    p.add_argument("--steps-per-graph", type=int, default=10,
                   help="steps captured per hipGraph (the K timed steps replay K/G graphs)")
    p.add_argument("--unfused", action="store_true",
                   help="N=1: time pack and unpack as two launches instead of the fused self exchange")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true")
    p.add_argument("--tune", default="", help="developer: ghx_tune key=value,... before planning")
    p.add_argument("--cold", action="store_true",
                   help="also time the dominant launch right after a 1 GiB cache-flushing kernel "
                        "(opt-in: its launches would skew a profiler's per-kernel average)")
    p.add_argument("--bulk", action="store_true",
                   help="N>1: also time the zero-copy bulk exchange (IPC puts into peer halos); "
                        "always on at N=1 (self puts)")
    p.add_argument("--force-dist", action="store_true",
                   help="initialise the nccl process group even at world size 1 (path test)")
    p.add_argument("--rehearse", action="store_true",
                   help="developer: N>1 ranks all on cuda:0 (RCCL refuses two ranks per GPU), "
                        "gloo group and the host-staged transport — exercises the N>1 code path "
                        "on a one-GPU box; its numbers are not the metric")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    if args.rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.force_dist
    if distributed:
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if args.rehearse:
            dist.barrier()
        else:
            dist.barrier(device_ids=[local])

    def all_reduce_host(x, op):
        """Reduce one python number over ranks (device tensor on nccl, host tensor on gloo)."""
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if args.rehearse else dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    ghex_amd.native_library()
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        _ghx.call("ghx_tune", k.encode(), int(v))

    N, Hw = args.N, args.halo
    E = N + 2 * Hw
    parts = DECOMP[world]
    G = [parts[d] * N for d in range(3)]
    c = (rank % parts[0], (rank // parts[0]) % parts[1], rank // (parts[0] * parts[1]))
    first = tuple(c[d] * N for d in range(3))
    last = tuple((c[d] + 1) * N - 1 for d in range(3))

    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(rank, first, last)
    hg = R.HaloGenerator((0, 0, 0), tuple(g - 1 for g in G), (Hw,) * 6, (True,) * 3)
    pc = R.make_pattern(ctx, hg, [dd])

    # synthetic field: owned cell = global linear index (exact in fp64), halo = -1
    base = torch.full((E, E, E), -1.0, dtype=torch.float64, device=dev)
    ar = [torch.arange(N, device=dev, dtype=torch.float64) + first[d] for d in range(3)]
    base[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = (
        ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)))
    logical = base.permute(2, 1, 0)  # (x, y, z), x contiguous: layout_map<2,1,0>
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx, staging="host" if args.rehearse else None)
    bis = [pc(fd)]

    # ---- verified full exchange (pack -> RCCL -> unpack) --------------------------------------
    co.exchange(bis).wait()
    idx = [torch.arange(E, device=dev, dtype=torch.int64) - Hw + first[d] for d in range(3)]
    wrap = [(idx[d] % G[d]).to(torch.float64) for d in range(3)]
    expect = wrap[0].view(1, 1, E) + G[0] * (wrap[1].view(1, E, 1) + G[1] * wrap[2].view(E, 1, 1))
    bad = int((base != expect).sum().item())
    del expect
    verified = bad == 0
    if distributed:
        verified = all_reduce_host(bad, dist.ReduceOp.SUM) == 0

    plan = co.plan(bis)
    send, recv = co.buffers(plan, dev)
    n_halo = E ** 3 - N ** 3
    step_bytes = 4 * n_halo * 8
    assert sum(b["size"] for b in plan.send) == n_halo * 8
    stream = torch.cuda.current_stream(dev)
    fptr = _ghx.ptr_array([fd.data_ptr()])
    sptr = _ghx.ptr_array([t.data_ptr() for t in send])
    rptr = _ghx.ptr_array([t.data_ptr() for t in recv])
    L = _ghx.lib()
    ns, nr = len(send), len(recv)

    # N=2/4: a rank has self messages (its periodic wrap in the undecomposed dimensions) AND peer
    # messages; the communication object then completes the self messages inside the pack
    # launch and unpacks the peer messages only (ghx_exchange_pack_self / _unpack_peers)
    mixed = co.fuse_self and co.mixed(plan) and not args.unfused
    pack_fn = L.ghx_exchange_pack_self if mixed else L.ghx_exchange_pack
    unpack_fn = L.ghx_exchange_unpack_peers if mixed else L.ghx_exchange_unpack

    def pack(s):
        rc = pack_fn(plan.h, fptr, 1, sptr, ns, s)
        if rc:
            raise RuntimeError(L.ghx_last_error().decode())

    def unpack(s):
        rc = unpack_fn(plan.h, fptr, 1, rptr, nr, s)
        if rc:
            raise RuntimeError(L.ghx_last_error().decode())

    def fused(s):
        rc = L.ghx_exchange_self(plan.h, fptr, 1, sptr, ns, s)
        if rc:
            raise RuntimeError(L.ghx_last_error().decode())

    # The product's exchange step: at N=1 every message is a self message and the communication
    # object runs pack+unpack as ONE launch (ghx_exchange_self); otherwise pack, transport, unpack.
    use_fused = co.fuse_self and co.all_self(plan) and not args.unfused

    def step_unfused():
        s = torch.cuda.current_stream(dev).cuda_stream
        pack(s)
        unpack(s)

    def step_fused():
        fused(torch.cuda.current_stream(dev).cuda_stream)

    def make_run(step):
        """run(k): exactly k steps, replayed from hipGraphs of G = --steps-per-graph steps
        (+ one graph for the remainder), so the graph-launch cost is paid once per G steps."""
        if args.no_graph:
            def run_eager(k):
                for _ in range(k):
                    step()
            return run_eager
        graphs = {}

        def graph_of(n):
            if n not in graphs:
                side = torch.cuda.Stream(dev)
                side.wait_stream(stream)
                with torch.cuda.stream(side):
                    step()  # warm the capture stream
                stream.wait_stream(side)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(n):
                        step()
                graphs[n] = g
            return graphs[n]

        G = max(1, args.steps_per_graph)

        def run(k):
            for _ in range(k // G):
                graph_of(G).replay()
            if k % G:
                graph_of(k % G).replay()
        return run

    run = make_run(step_fused if use_fused else step_unfused)
    run(args.warmup)
    torch.cuda.synchronize(dev)

    dev_time = {}

    def timed(fn, k, events=False):
        """Host wall time of k calls (barrier + synchronize on both sides, max over ranks); with
        events=True also the device time of the region from HIP events on the launch stream."""
        if distributed:
            barrier()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(k):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        if events:
            dev_time["s"] = e0.elapsed_time(e1) * 1e-3
        if distributed:
            barrier()
        dt = time.perf_counter() - t0
        if distributed:
            dt = all_reduce_host(dt, dist.ReduceOp.MAX)
        return dt

    K = args.steps
    run(K % max(1, args.steps_per_graph) or 1)  # instantiate the remainder graph untimed
    torch.cuda.synchronize(dev)
    T = timed(lambda: run(K), 1, events=True)
    dev_step = dev_time["s"] / K  # device time per step over the timed region (HIP events)
    value = world * step_bytes * K / T / 1e9
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(T / K * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (owned cell = global linear index; verified after a full exchange)",
        "config": {
            "workload": f"{N}^3 fp64 structured 3D halo={Hw}, 26-neighbour periodic, "
                        f"device-resident pack+unpack, decomposition {list(parts)}",
            "N": N, "halo": Hw, "fields": 1, "decomposition": list(parts),
            "launch": ("eager" if args.no_graph else
                       f"hipGraph of {args.steps_per_graph} steps") + ", " +
                      ("fused self-exchange: 1 launch per step (each lane packs its buffer bytes "
                       "and writes the halos from the same registers)" if use_fused else
                       "pack launch completing the self messages + unpack launch of the peer "
                       "messages" if mixed else "pack launch + unpack launch"),
            "bytes_per_step_per_gpu": step_bytes,
            "parallelism": f"{world} rank(s), one domain per GPU",
        },
        "verified": verified,
    }
    if args.rehearse:
        out["rehearsal"] = ("all ranks on cuda:0, gloo + host-staged transport: code-path check, "
                            "not the metric")

    # ---- per-kernel HIP-event durations (dominant kernel roofline) ----------------------------
    # Differential method (removes the fixed cost of the events themselves): hipGraphs of M steps,
    # of M steps + one pack, and of M steps + one pack + one unpack, replayed in interleaved
    # rounds; pack = T1 - T0, unpack = T2 - T1 (each includes its dependent-launch boundary).
    t_pack, t_unpack = kernel_durations(torch, dev, stream, [pack, unpack])
    if use_fused:
        # one launch per step: its average duration over the timed region = device time / K
        (t_fused,) = kernel_durations(torch, dev, stream, [fused])
        launch_bytes, dom_name, dom_t, kname = step_bytes, "self", dev_step, "k_self (pack+unpack)"
    else:
        # two launches per step: the timed region's device time split by their live differential
        # durations (graphs of M and M+1 launches)
        # (mixed: the pack launch also moves the self messages' unpack bytes, the unpack launch
        # only the peer messages')
        self_b = sum(b["size"] for b in plan.recv if b["rank"] == rank) if mixed else 0
        pack_b, unpack_b = 2 * n_halo * 8 + 2 * self_b, 2 * n_halo * 8 - 2 * self_b
        dom_name, dom_d = ("pack", t_pack) if t_pack >= t_unpack else ("unpack", t_unpack)
        launch_bytes = pack_b if dom_name == "pack" else unpack_b
        dom_t = dev_step * dom_d / (t_pack + t_unpack)
        kname = ("k_self<pack + self messages>" if mixed and dom_name == "pack"
                 else f"k_copy<{dom_name}>")
    achieved = launch_bytes / dom_t / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile) and not mixed:  # (profiled: the N=1 launches)
        try:
            tj = json.load(open(tfile))
            ent = tj.get(f"N{N}_H{Hw}", {}).get(dom_name)
            traffic = ent.get("hbm_bytes_per_launch") if ent else None
        except Exception:
            traffic = None
    out["roofline"] = {"bound": "hbm", "kernel": kname,
                       "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                       "traffic_source": (None if traffic is None else
                                          "profiles/pmc_traffic.json: rocprofv3 --pmc of the "
                                          f"N=1 {dom_name} launch of the same bytes" +
                                          ("" if world == 1 else
                                           " (one-domain plan; per-peer buffers at N>1)")),
                       "algorithmic_bytes_per_launch": launch_bytes,
                       "launch_us": round(dom_t * 1e6, 2),
                       "launch_us_source": "HIP events on the launch stream around the timed "
                                           "region, device time per step" +
                                           ("" if use_fused else " x the kernel's share of the "
                                            "step (graph differencing)"),
                       "step_device_us": round(dev_step * 1e6, 2),
                       "pack_us": round(t_pack * 1e6, 2), "unpack_us": round(t_unpack * 1e6, 2)}
    if use_fused:
        out["roofline"]["self_us_differential"] = round(t_fused * 1e6, 2)
    if use_fused:
        # the same step as two launches (what N>1 runs per rank), for comparison
        run_u = make_run(step_unfused)
        run_u(max(5, K % max(1, args.steps_per_graph)))
        Tu = timed(lambda: run_u(K), 1)
        out["unfused"] = {"value": round(world * step_bytes * K / Tu / 1e9, 2),
                          "ms_per_step": round(Tu / K * 1e3, 5)}

    if not args.no_extras:
        # full exchange incl. transport (RCCL for N>1; self-message aliasing for N=1)
        ke = min(K, 50)
        for _ in range(3):
            co.exchange(bis).wait()
        Te = timed(lambda: co.exchange(bis).wait(), ke)
        out["exchange_ms_per_step"] = round(Te / ke * 1e3, 4)
        if world == 1 or args.bulk:
            # zero-copy bulk exchange (BulkCommunicationObject): puts straight into the
            # receivers' halos, no buffers: 2*n*8 bytes moved per step (not the metric's 4*n*8)
            try:
                bco = ghex_amd.make_bulk_communication_object(ctx)
                bco.add_field(bis[0])
                bco.init()
                for _ in range(3):
                    bco.exchange().wait()
                Tb = timed(lambda: bco.exchange().wait(), ke)
                put = bco._puts[0]

                def put_fn(s):
                    rc = L.ghx_put_execute(put[0], put[1], put[2], put[3], put[4], s)
                    if rc:
                        raise RuntimeError(L.ghx_last_error().decode())
                (t_put,) = kernel_durations(torch, dev, stream, [put_fn])
                out["bulk"] = {"exchange_ms_per_step": round(Tb / ke * 1e3, 4),
                               "put_launches": len(bco._puts),
                               "put_us": round(t_put * 1e6, 2) if len(bco._puts) == 1 else None,
                               "bytes_moved_per_step": 2 * n_halo * 8}
                del bco
            except Exception as e:  # reported, never fatal for the headline measurement
                out["bulk"] = {"error": str(e)[:200]}
            co.exchange(bis).wait()
        # host-staged: pack -> D2H (pinned) -> H2D -> unpack (NIC-side buffers, north star)
        hs = [torch.empty(b["size"], dtype=torch.uint8, pin_memory=True) for b in plan.send]

        def staged():
            s = torch.cuda.current_stream(dev).cuda_stream
            pack(s)
            for i, b in enumerate(plan.send):
                hs[i].copy_(send[i][:b["size"]], non_blocking=True)
            for i, b in enumerate(plan.recv):  # N=1: every message is a self message
                j = next(j for j, x in enumerate(plan.send) if x["pair"] == b["pair"])
                recv[i][:b["size"]].copy_(hs[j], non_blocking=True)
            unpack(s)

        if world == 1:
            for _ in range(3):
                staged()
            Ts = timed(staged, min(K, 50))
            pcie = 2 * n_halo * 8
            out["host_staged"] = {
                "GBps_algorithmic": round(step_bytes * min(K, 50) / Ts / 1e9, 2),
                "ms_per_step": round(Ts / min(K, 50) * 1e3, 4),
                "pcie_bytes_per_step": pcie}
            # restore valid halos after the staged copies
            co.exchange(bis).wait()

    if args.cold:
        # the dominant launch with cold caches: an application's stencil sweeps the whole field
        # between exchanges, so its halo rows are not left in the 256 MiB Infinity Cache as
        # they are when the bench replays exchanges back to back. A 1 GiB read-modify-write
        # before every launch evicts them; the flush itself is differenced away.
        fl = torch.zeros(1 << 27, dtype=torch.float64, device=dev)
        dom_fn = fused if use_fused else (pack if dom_name == "pack" else unpack)
        t_cold = cold_duration(torch, dev, stream, dom_fn, lambda s: fl.add_(1.0))
        out["roofline"]["cold_launch_us"] = round(t_cold * 1e6, 2)
        out["roofline"]["cold_achieved"] = round(launch_bytes / t_cold / 1e9, 1)
        # the same with a read-only flush (1 GiB reduction): caches cold but not dirty, so the
        # launch does not also pay for writing back the flush's dirty lines it evicts
        acc = torch.empty((), dtype=torch.float64, device=dev)
        t_clean = cold_duration(torch, dev, stream, dom_fn,
                                lambda s: torch.sum(fl, dim=(0,), out=acc))
        out["roofline"]["cold_clean_launch_us"] = round(t_clean * 1e6, 2)
        out["roofline"]["cold_clean_achieved"] = round(launch_bytes / t_clean / 1e9, 1)
        del fl
        torch.cuda.empty_cache()

    if not args.no_extras:
        # measured device-to-device copy rate: 1 GiB -> 1 GiB, read+write bytes
        a = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            b.copy_(a)
        e1.record()
        e1.synchronize()
        out["roofline"]["measured_d2d_copy_GBps"] = round(2 * a.numel() * 10 /
                                                          (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
        del a, b
        torch.cuda.empty_cache()

    if world == 1 and not args.no_extras:
        # the other BASELINE configs, per GPU (their 8-GPU forms are weak-scaled copies)
        del base, logical, fd, bis, send, recv
        co = None
        torch.cuda.empty_cache()
        out["extra_configs"] = {
            "config4_5fields_256^3_h3_f64f32": bench_config4(torch, dev, ghex_amd, R),
            "config5_unstructured_10M_5pct_levels1": bench_config5(torch, dev, _ghx, 1),
            "config5_unstructured_10M_5pct_levels8": bench_config5(torch, dev, _ghx, 8),
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, Hw, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        barrier()
        dist.destroy_process_group()


def kernel_durations(torch, dev, stream, fns, M=10, rounds=15):
    """Live per-launch durations of the launches `fns` (one step = fns in order) by differencing
    hipGraphs of M steps, M steps + fns[0], M steps + fns[0] + fns[1], ... replayed in interleaved
    rounds (medians). Removes the events' own cost; each includes its dependent-launch boundary."""
    def capture(extra):
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            for f in fns:
                f(side.cuda_stream)
        stream.wait_stream(side)
        with torch.cuda.graph(g):
            s = torch.cuda.current_stream(dev).cuda_stream
            for _ in range(M):
                for f in fns:
                    f(s)
            for f in fns[:extra]:
                f(s)
        return g

    graphs = [capture(e) for e in range(len(fns) + 1)]
    times = [[] for _ in graphs]
    for g in graphs:
        g.replay()
    torch.cuda.synchronize(dev)
    for _ in range(rounds):
        for i, g in enumerate(graphs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.replay()
            e1.record(stream)
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) * 1e-3)
    med = [sorted(t)[len(t) // 2] for t in times]
    return tuple(med[i + 1] - med[i] for i in range(len(fns)))


def cold_duration(torch, dev, stream, fn, flush, M=10, rounds=7):
    """Per-launch duration of fn right after a cache-flushing kernel: median over rounds of
    [graph of M x (flush, fn)] - [graph of M x flush], divided by M."""
    def capture(with_fn):
        side = torch.cuda.Stream(dev)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            flush(side.cuda_stream)
            fn(side.cuda_stream)
        stream.wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            s = torch.cuda.current_stream(dev).cuda_stream
            for _ in range(M):
                flush(s)
                if with_fn:
                    fn(s)
        return g

    g0, g1 = capture(False), capture(True)
    t = [[], []]
    for _ in range(rounds):
        for i, g in enumerate((g0, g1)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.replay()
            e1.record(stream)
            e1.synchronize()
            t[i].append(e0.elapsed_time(e1) * 1e-3)
    med = [sorted(x)[len(x) // 2] for x in t]
    return (med[1] - med[0]) / M


def _time_graph(torch, dev, fn, k=50, per=10):
    stream = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        fn(side.cuda_stream)
    stream.wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per):
            fn(torch.cuda.current_stream(dev).cuda_stream)
    g.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(k // per):
        g.replay()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / (k // per * per)


def bench_config4(torch, dev, ghex_amd, R):
    """BASELINE config 4 on one GPU: 5 fields 256^3 [f64,f32,f64,f32,f64], H=3, one exchange of
    all five (one periodic domain: all self messages -> the fused launch), verified."""
    from ghex_amd import _ghx
    N, H = 256, 3
    E = N + 2 * H
    types = [torch.float64, torch.float32, torch.float64, torch.float32, torch.float64]
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    fields, bis = [], []
    ar = torch.arange(N, device=dev, dtype=torch.float64)
    val = (ar.view(1, 1, N) + N * (ar.view(1, N, 1) + N * ar.view(N, 1, 1)))
    for k, T in enumerate(types):
        f = torch.full((E, E, E), -1, dtype=T, device=dev)
        f[H:H + N, H:H + N, H:H + N] = ((val + k) % (1 << 23)).to(T)
        fields.append(f)
        bis.append(pc(R.make_field_descriptor(dd, f.permute(2, 1, 0), (H,) * 3, (E,) * 3)))
    co = R.make_communication_object(ctx)
    co.exchange(bis).wait()
    idx = (torch.arange(E, device=dev) - H) % N
    wv = (idx.view(1, 1, E) + N * (idx.view(1, E, 1) + N * idx.view(E, 1, 1))).to(torch.float64)
    ok = all(bool((f == ((wv + k) % (1 << 23)).to(f.dtype)).all()) for k, f in enumerate(fields))
    plan = co.plan(bis)
    send, recv = co.buffers(plan, dev)
    fptr = _ghx.ptr_array([f.data_ptr() for f in fields])
    sptr = _ghx.ptr_array([t.data_ptr() for t in send])
    L = _ghx.lib()
    fusedp = co.all_self(plan)

    def step(s):
        if fusedp:
            L.ghx_exchange_self(plan.h, fptr, 5, sptr, len(send), s)
        else:
            L.ghx_exchange_pack(plan.h, fptr, 5, sptr, len(send), s)
            L.ghx_exchange_unpack(plan.h, fptr, 5, sptr, len(send), s)
    t = _time_graph(torch, dev, step)
    n = E ** 3 - N ** 3
    nbytes = 4 * n * (3 * 8 + 2 * 4)
    return {"GBps": round(nbytes / t / 1e9, 1), "us_per_exchange": round(t * 1e6, 2),
            "bytes_per_exchange": nbytes, "verified": ok, "fused_self": fusedp}


def bench_config5(torch, dev, _ghx, levels):
    """BASELINE config 5 shape on one GPU: 10M cells, 5 % halo, 7 peers, random lids (seed
    20260715), levels_first fp64: fused gather of all send lists + fused scatter of all recv
    lists (unstructured plans)."""
    import ctypes
    import numpy as np
    rng = np.random.default_rng(20260715)
    n = 10_000_000
    nh = n // 20
    send = rng.choice(n, size=nh, replace=False)
    recv = rng.permutation(n)[:nh]
    cuts = np.sort(rng.choice(np.arange(1, nh), size=6, replace=False))
    sl, rl = np.split(send, cuts), np.split(recv, cuts)
    vals = torch.randn(n * levels, dtype=torch.float64, device=dev)

    def plan(lists, direction):
        ents, keep = [], []
        for k, l in enumerate(lists):
            e = _ghx.UPackEntry()
            e.data.elem_size, e.data.levels, e.data.levels_first = 8, levels, 1
            e.data.index_stride, e.data.level_stride = levels, 1
            e.field_slot, e.buffer_slot, e.buffer_offset = 0, k, 0
            arr = np.ascontiguousarray(l, dtype=np.int64)
            keep.append(arr)
            e.lids = arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            e.n_lids = len(arr)
            ents.append(e)
        h = ctypes.c_void_p()
        _ghx.call("ghx_uplan_create", (_ghx.UPackEntry * len(ents))(*ents), len(ents), direction,
                  ctypes.byref(h))
        return h

    hp, hu = plan(sl, 0), plan(rl, 1)
    bufs = [torch.empty(len(l) * levels * 8, dtype=torch.uint8, device=dev) for l in sl]
    fp = _ghx.ptr_array([vals.data_ptr()])
    bp = _ghx.ptr_array([b.data_ptr() for b in bufs])
    L = _ghx.lib()

    def step(s):
        L.ghx_uplan_execute(hp, fp, 1, bp, len(bufs), s)
        L.ghx_uplan_execute(hu, fp, 1, bp, len(bufs), s)
    t = _time_graph(torch, dev, step)
    L.ghx_uplan_destroy(hp)
    L.ghx_uplan_destroy(hu)
    nbytes = 4 * nh * levels * 8
    return {"GBps": round(nbytes / t / 1e9, 1), "us_per_exchange": round(t * 1e6, 2),
            "bytes_per_exchange": nbytes, "cells": n, "halo_cells": nh, "peers": 7,
            "index_bytes_per_exchange": 2 * nh * 4}


def cpu_baseline(N, Hw, seconds):
    """The oracle's single-thread C restatement of serialization<cpu>::pack_batch/unpack_batch
    (include/ghex/structured/pack_kernels.hpp:62-158) on the same workload, bounded in time."""
    import numpy as np
    from oracle import oracle as orc
    E = N + 2 * Hw
    a = np.zeros((E, E, E))
    a[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = np.arange(N ** 3, dtype=np.float64).reshape(N, N, N)
    dom = orc.RegularDomain(0, (0, 0, 0), (N - 1,) * 3)
    pat = orc.regular_make_pattern([[dom]], (0, 0, 0), (N - 1,) * 3, (Hw,) * 6, (1, 1, 1))[0][0]
    spec = orc.FieldSpec(a, 8, (2, 1, 0), (Hw,) * 3, (E,) * 3)
    send = list(pat.send.values())[0][1]
    recv = list(pat.recv.values())[0][1]
    nbytes = sum(b.size() for b in send) * 8
    buf = np.zeros(nbytes, np.uint8)
    orc.structured_pack(spec, buf, send)
    orc.structured_unpack(spec, buf, recv)
    t0 = time.perf_counter()
    it = 0
    while True:
        orc.structured_pack(spec, buf, send)
        orc.structured_unpack(spec, buf, recv)
        it += 1
        dt = time.perf_counter() - t0
        if dt >= seconds and it >= 3:
            break
    gbs = 4 * nbytes * it / dt / 1e9
    out = {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"{N}^3 fp64 H={Hw} one periodic domain, pack+unpack x{it} "
                     f"({dt:.1f} s, 1 thread, oracle/ghex_oracle.c row-memcpy restatement)"}
    del a, buf
    out["ranks"] = cpu_baseline_ranks(N, Hw, seconds, orc, nbytes, send, recv)
    return out


def cpu_baseline_ranks(N, Hw, seconds, orc, nbytes, send, recv):
    """the same single-threaded serializer run as independent ranks, one per host
    core of the box's CPU share (each rank its own 512^3 domain and buffer, like the reference's
    one-rank-per-core CPU runs). The C oracle releases the GIL inside its ctypes calls, so the
    ranks are threads of this process; value = bytes summed over ranks / the slowest rank's time."""
    import threading

    import numpy as np
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    ranks = max(1, min(16, share))  # the GPU box grants 16 cores per GPU (its nproc shows more)
    E = N + 2 * Hw
    res = [None] * ranks
    barrier = threading.Barrier(ranks)

    def rank_fn(r):
        a = np.zeros((E, E, E))
        a[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = r
        spec = orc.FieldSpec(a, 8, (2, 1, 0), (Hw,) * 3, (E,) * 3)
        buf = np.zeros(nbytes, np.uint8)
        orc.structured_pack(spec, buf, send)
        orc.structured_unpack(spec, buf, recv)
        barrier.wait()
        t0 = time.perf_counter()
        it = 0
        while True:
            orc.structured_pack(spec, buf, send)
            orc.structured_unpack(spec, buf, recv)
            it += 1
            dt = time.perf_counter() - t0
            if dt >= seconds and it >= 3:
                break
        res[r] = (it, dt)

    th = [threading.Thread(target=rank_fn, args=(r,)) for r in range(ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    total = sum(4 * nbytes * it for it, _ in res)
    slowest = max(dt for _, dt in res)
    its = [it for it, _ in res]
    return {"value": round(total / slowest / 1e9, 3), "unit": "GB/s", "cores": ranks,
            "kind": "port",
            "sample": f"{ranks} independent ranks, each a {N}^3 fp64 H={Hw} periodic domain, "
                      f"pack+unpack x{min(its)}-{max(its)} in {slowest:.1f} s, one thread each "
                      f"(oracle/ghex_oracle.c)"}


if __name__ == "__main__":
    main()
