#!/usr/bin/env python3
"""bench.py — device-resident halo pack+unpack GB/s (BASELINE.json metric) on MI355X.

Workload (BASELINE configs[1], weak-scaled for N>1 as configs[2]): per GPU one 512^3 fp64 domain
(extent 516^3 with halo 2), 26-neighbour periodic halo. N=1: one periodic domain (all 26
iteration spaces are a self message); N=2/4/8: (2,1,1)/(2,2,1)/(2,2,2) decomposition of the
periodic global grid, one rank per GPU.

A step = the per-rank exchange step minus transport, fields and buffers resident in HBM: one
fused pack launch (every iteration space of every send buffer -> the send buffers) + one fused
unpack launch (the recv buffers -> every halo). That is what every rank runs at N>1, and at N=1
the same two launches are timed (the recv buffer of a self message is its send buffer), so the
N=1..8 lines measure the same kernels. Algorithmic bytes per step per GPU = 4 * n * 8 (pack read
+ write, unpack read + write), n = (N+2H)^3 - N^3 halo cells. value = sum over ranks of
bytes*K / max over ranks of the K-step wall time; the K steps replay hipGraphs of
--steps-per-graph steps, every graph instantiated and replayed once BEFORE the timed region.

The product's N=1 exchange runs pack+unpack as ONE launch (k_self: each lane packs its buffer
bytes and writes the halos from the same registers, so the buffer is never read back): it moves
3 * n * 8 bytes and is reported as "fused_self" with exactly those bytes, not as the headline.

Before timing, one full exchange (pack -> RCCL send/recv over xGMI for N>1 -> unpack) is run and
every cell of every rank's (N+2H)^3 box is verified on the GPU against the wrapped global index.
Extra fields: cold-cache launch times (default; --no-cold for profiler runs), the full exchange
time incl. RCCL (one group, and per-peer pipelined), the host-staged rate (pack + D2H + H2D +
unpack through pinned memory), and on rank 0 at N=1 the oracle's single-thread CPU pack+unpack
on a bounded sample (cpu_baseline).

`python bench.py --gpus N` without torchrun spawns the N rank processes itself (before any GPU
call) with MASTER_ADDR=127.0.0.1; under torch.distributed.run it runs as the given rank.
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
    p.add_argument("--steps-per-graph", type=int, default=0,
                   help="steps captured per hipGraph (the K timed steps replay K/G graphs); "
                        "0: all K steps in one graph (at most 1000)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-config-seconds", type=float, default=3.0,
                   help="seconds of CPU work for each extra config's cpu_baseline (configs 4, 5)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true")
    p.add_argument("--tune", default="", help="developer: ghx_tune key=value,... before planning")
    p.add_argument("--no-cold", action="store_true",
                   help="skip the cold-cache launch times (their extra launches of the same "
                        "kernels would skew a profiler's per-kernel averages)")
    p.add_argument("--no-layout", action="store_true",
                   help="skip the padded-layout leg (its launches share the headline kernel's "
                        "grid and would mix into a profiler's per-kernel averages)")
    p.add_argument("--bulk-child", action="store_true",
                   help="internal: the isolated zero-copy leg's rank process (see bulk_isolated)")
    p.add_argument("--bulk-only", type=int, default=0, metavar="N",
                   help="developer: run only the N>1 isolated zero-copy leg — N --bulk-child "
                        "processes (puts + direct, verified), spread over the visible GPUs (all "
                        "on cuda:0 on a one-GPU box), without the headline ranks; rank 0's line")
    p.add_argument("--bulk-timeout", type=float, default=120.0,
                   help="seconds the isolated zero-copy leg (N>1) may take before it is killed")
    p.add_argument("--bulk", action="store_true",
                   help="N>1: also time the zero-copy bulk exchange (IPC puts into peer halos); "
                        "always on at N=1 (self puts)")
    p.add_argument("--force-dist", action="store_true",
                   help="initialise the nccl process group even at world size 1 (path test)")
    p.add_argument("--rehearse", action="store_true",
                   help="developer: N>1 ranks all on cuda:0 (RCCL refuses two ranks per GPU), "
                        "gloo group and the host-staged transport — exercises the N>1 code path "
                        "on a one-GPU box; its numbers are not the metric")
    p.add_argument("--extras-timeout", type=float, default=240.0,
                   help="seconds the extras (after the headline) may take before the line is "
                        "printed without them")
    p.add_argument("--init-timeout", type=float, default=300.0,
                   help="seconds init_process_group + the setup all-gather may take; on expiry "
                        "the line is printed with verified=false and an error, exit 3")
    p.add_argument("--exchange-timeout", type=float, default=300.0,
                   help="seconds the verified full exchange (the first RCCL traffic) may take; "
                        "on expiry as --init-timeout")
    p.add_argument("--headline-timeout", type=float, default=240.0,
                   help="seconds the headline measurement (graphs, warmup, timed region, "
                        "kernel durations) may take; on expiry as --init-timeout (a few seconds "
                        "at the default steps; kept below a 600-s bench limit minus the other "
                        "stages, so a hang there is still reported)")
    return p.parse_args()


# the one JSON line: whether rank 0 printed it, and the guard that can print a null one
_LINE = {"guard": None, "printed": False}


class StageGuard:
    """Bounds the stages before the headline line can be printed (init_process_group, the first
    cross-GPU exchange, the timed region). If a stage does not finish in time — a peer died or
    the transport hangs, which a rank blocked inside RCCL can neither see nor leave — rank 0
    prints the line with value null, verified false and an `error` naming the stage, and every
    rank exits with status 3 (os._exit from the guard thread: the stuck thread cannot be joined,
    and nothing is re-executed or retried). Other ranks report to stderr only."""

    EXIT_CODE = 3

    def __init__(self, line, rank=0):
        self.line = line  # the JSON fields known so far (metric, n_gpus, config ...)
        self.rank = rank

    def expire(self, name, seconds):
        o = dict(self.line)
        o.update(value=None, verified=False, stage=name,
                 error=f"stage '{name}' did not complete within {seconds:.0f} s on rank "
                       f"{self.rank} (a peer or the transport hung); no measurement")
        msg = json.dumps(o)
        if self.rank == 0:
            print(msg, flush=True)
        else:
            print(msg, file=sys.stderr, flush=True)
        sys.stderr.flush()
        os._exit(self.EXIT_CODE)

    def fail(self, name, exc):
        """A stage raised: rank 0 prints the line with value null and the error (the exception
        then propagates, so the process still fails)."""
        o = dict(self.line)
        o.update(value=None, verified=False, stage=name,
                 error=f"stage '{name}' failed on rank {self.rank}: "
                       f"{type(exc).__name__}: {str(exc)[:300]}; no measurement")
        print(json.dumps(o), file=sys.stdout if self.rank == 0 else sys.stderr, flush=True)
        _LINE["printed"] = True

    def stage(self, name, seconds):
        import contextlib
        import threading

        @contextlib.contextmanager
        def guarded():
            done = threading.Event()

            def watch():
                if not done.wait(seconds):
                    self.expire(name, seconds)
            threading.Thread(target=watch, daemon=True, name=f"guard:{name}").start()
            try:
                yield
            except Exception as e:
                done.set()
                self.fail(name, e)
                raise
            finally:
                done.set()
        return guarded()


def spawn_workers(args) -> int:
    """`bench.py --gpus N` outside torchrun: start N fresh rank processes (this process never
    touches the GPU), rank 0's stdout is the JSON line; exit with the worst child status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ)
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(args.gpus),
                   RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(args.gpus),
                   GHX_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                c = p.poll()
                if c is None:
                    continue
                pending.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in pending:  # one rank died: the others would wait for it forever
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


class Runner:
    """run(k): exactly k steps, replayed from hipGraphs of G steps (+ one graph for k % G).
    prepare(k) captures and replays once every graph run(k) will use, so nothing is captured
    or instantiated inside a timed region."""

    def __init__(self, torch, dev, stream, step, G, eager=False):
        self.torch, self.dev, self.stream, self.step = torch, dev, stream, step
        self.G, self.eager, self.graphs = max(1, G), eager, {}

    def _graph(self, n):
        torch = self.torch
        g = self.graphs.get(n)
        if g is None:
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(self.stream)
            with torch.cuda.stream(side):
                self.step()  # warm the capture stream
            self.stream.wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    self.step()
            self.graphs[n] = g
            g.replay()
            torch.cuda.synchronize(self.dev)
        return g

    def prepare(self, k):
        if self.eager:
            return
        if k >= self.G:
            self._graph(self.G)
        if k % self.G:
            self._graph(k % self.G)

    def run(self, k):
        if self.eager:
            for _ in range(k):
                self.step()
            return
        for _ in range(k // self.G):
            self.graphs[self.G].replay()
        if k % self.G:
            self.graphs[k % self.G].replay()


def verify_replay(torch, dev, replay, clear, count_bad, send, recv, deliver=None):
    """Wrong cells after the TIMED kernels alone: halos reset (clear), every send/recv buffer
    byte set to 0xFF (an fp64 NaN, unequal to every expected value), the timed graph replayed
    (replay: the same graph replays the timed region ran). Where peer messages exist, deliver()
    then moves the packed send buffers into the receivers' receive buffers (transport only) and
    the timed graph is replayed once more, so the peer halos too are written by the timed
    graph's own unpack launch. count_bad() checks every cell (summed over ranks)."""
    clear()
    for t in list(send) + list(recv):
        t.fill_(255)
    replay()
    if deliver is not None:
        deliver()
        replay()
    torch.cuda.synchronize(dev)
    return count_bad()


def bulk_child(args):
    """One rank of the isolated zero-copy leg (spawned by bulk_isolated, one process per rank,
    the parent rank's GPU): the same domain and field as the headline, exchanged by
    BulkCommunicationObject — IPC puts straight into the peers' halos over xGMI, ordered by device
    epochs — verified (every cell = its wrapped global index) and timed. A gloo group carries the
    setup; the data moves only through the puts. Rank 0 prints one JSON line."""
    import datetime
    import torch
    import torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=max(60.0, args.bulk_timeout)))
    import ghex_amd
    from ghex_amd.structured import regular as R
    ghex_amd.native_library()
    N, Hw, parts = args.N, args.halo, DECOMP[world]
    E = N + 2 * Hw
    G = [parts[d] * N for d in range(3)]
    c = (rank % parts[0], (rank // parts[0]) % parts[1], rank // (parts[0] * parts[1]))
    first = tuple(c[d] * N for d in range(3))
    last = tuple((c[d] + 1) * N - 1 for d in range(3))
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(rank, first, last)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), tuple(g - 1 for g in G), (Hw,) * 6,
                                             (True,) * 3), [dd])
    base = torch.full((E, E, E), -1.0, dtype=torch.float64, device=dev)
    ar = [torch.arange(N, device=dev, dtype=torch.float64) + first[d] for d in range(3)]
    base[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = (
        ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)))
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (Hw,) * 3, (E,) * 3)
    bco = ghex_amd.make_bulk_communication_object(ctx)
    bco.add_field(pc(fd))
    bco.init()
    bco.exchange().wait()
    idx = [((torch.arange(E, device=dev, dtype=torch.int64) - Hw + first[d]) % G[d]).to(torch.float64)
           for d in range(3)]
    expect = idx[0].view(1, 1, E) + G[0] * (idx[1].view(1, E, 1) + G[1] * idx[2].view(E, 1, 1))
    bad = torch.tensor([float((base != expect).sum().item())])
    del expect
    dist.all_reduce(bad)

    def timed(fn, k):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        t = torch.tensor([time.perf_counter() - t0])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    k = min(args.steps, 50)
    for _ in range(3):
        bco.exchange().wait()
    T = timed(lambda: bco.exchange(), k)
    bco.check_epochs()
    Tw = timed(lambda: bco.exchange().wait(), k)
    n = E ** 3 - N ** 3
    line = {"isolated": True, "verified": bad.item() == 0,
            "exchange_ms_per_step": round(T / k * 1e3, 4),
            "exchange_wait_ms_per_step": round(Tw / k * 1e3, 4),
            "GBps_moved": round(world * 2 * n * 8 * k / T / 1e9, 1),
            "epochs": bco.epochs, "put_launches": len(bco._puts),
            "bytes_moved_per_step_per_gpu": 2 * n * 8,
            "transport": "IPC puts into the peers' fields (over xGMI between GPUs), device epochs; "
                         "gloo for setup only"}
    if rank == 0:  # the puts' result, in case the direct leg below never returns
        print(json.dumps(dict(line, direct={"error": "did not finish"})), flush=True)
    # the direct exchange (CommunicationObject(direct=True)): the pack writes each peer message
    # into the receiver's buffer over xGMI (IPC), device epochs, local unpack; halos reset first
    direct = {}
    try:
        base.fill_(-1.0)
        base[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = (
            ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)))
        co = R.make_communication_object(ctx, direct=True)
        bis = [pc(fd)]
        co.exchange(bis).wait()
        expect = idx[0].view(1, 1, E) + G[0] * (idx[1].view(1, E, 1) + G[1] * idx[2].view(E, 1, 1))
        dbad = torch.tensor([float((base != expect).sum().item())])
        del expect
        dist.all_reduce(dbad)

        def once():
            co.exchange(bis)
            co._valid = False  # stream-ordered back to back: the next one follows on the stream
        for _ in range(3):
            co.exchange(bis).wait()
        Td = timed(once, k)
        co.check_epochs()
        Tdw = timed(lambda: co.exchange(bis).wait(), k)
        direct = {"verified": dbad.item() == 0, "exchange_ms_per_step": round(Td / k * 1e3, 4),
                  "exchange_wait_ms_per_step": round(Tdw / k * 1e3, 4),
                  "GBps_exchange_equivalent": round(world * 4 * n * 8 * k / Td / 1e9, 1),
                  "transport": "pack launch writes each peer message into the receiver's buffer "
                               "(IPC over xGMI), device epochs, local unpack launch"}
        del co
    except Exception as e:  # reported in the line, never fatal for the bulk leg
        direct = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    if rank == 0:
        print(json.dumps(dict(line, direct=direct)), flush=True)
    del bco
    dist.barrier()
    dist.destroy_process_group()


def bulk_only(args) -> int:
    """`bench.py --bulk-only N`: the isolated zero-copy leg of an N-GPU run on its own — N
    --bulk-child processes (each builds its rank's domain, exchanges by IPC puts and then by the
    direct exchange, verifies every cell), spawned by this process, which never touches the GPU.
    Rank r runs on GPU r mod (visible GPUs): on a one-GPU box all N share cuda:0, which keeps an
    N=8 rehearsal at 8 processes on the card (the headline ranks are not started). Prints rank
    0's line (with n_procs and the GPUs used); exits 0 only when every child did and both forms
    verified."""
    import socket
    import torch  # device_count() does not initialise the GPU on this image
    n = args.bulk_only
    if n not in DECOMP or n < 2:
        raise SystemExit("--bulk-only takes 2, 4 or 8")
    ngpu = max(1, torch.cuda.device_count())
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(n) as ex:
        futs = [ex.submit(bulk_isolated, args, r, n, r % ngpu, port, args.bulk_timeout)
                for r in range(n)]
        res = [f.result() for f in futs]
    line = dict(res[0] or {"isolated": True, "error": "rank 0 gave no result"})
    errs = {r: x["error"] for r, x in enumerate(res) if isinstance(x, dict) and "error" in x}
    if errs:
        line["errors"] = errs
    line.update(mode="bulk-only", n_procs=n, gpus_used=min(n, ngpu),
                config={"N": args.N, "halo": args.halo, "decomposition": list(DECOMP[n])})
    print(json.dumps(line), flush=True)
    ok = (not errs and line.get("verified") is True and
          line.get("direct", {}).get("verified") is True)
    return 0 if ok else 1


def bulk_isolated(args, rank, world, local, port_of_rank0, timeout):
    """The zero-copy exchange between GPUs, run in child processes (one per rank, spawned, not
    exec'd) so that whatever happens there — a fault, a hang past --bulk-timeout — cannot take
    the headline line down with it: the parent waits, kills the child's process group on expiry
    and reports an error entry instead."""
    import signal
    import subprocess
    # under torchrun the rank's env says "use the agent's store" (TORCHELASTIC_USE_AGENT_STORE):
    # the children rendezvous on their own port instead, rank 0's child hosting the store
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port_of_rank0), WORLD_SIZE=str(world),
               RANK=str(rank), LOCAL_RANK=str(local))
    cmd = [sys.executable, os.path.abspath(__file__), "--bulk-child", "--gpus", str(world),
           "--steps", str(args.steps), "--N", str(args.N), "--halo", str(args.halo)]
    def die_with_parent():  # the child never outlives this rank (e.g. the extras' watchdog exit)
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    cmd += ["--bulk-timeout", str(timeout)]
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True, preexec_fn=die_with_parent)
    try:
        so, se = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        so, _ = p.communicate()
        lines = [l for l in (so or "").splitlines() if l.startswith("{")]
        if rank == 0 and lines:  # the puts finished, the direct leg did not
            res = json.loads(lines[-1])
            res["error"] = f"timed out after {timeout:.0f} s (after the puts' result)"
            return res
        return {"isolated": True, "error": f"timed out after {timeout:.0f} s"}
    if p.returncode != 0:
        return {"isolated": True, "error": f"exit {p.returncode}: {se.strip()[-300:]}"}
    if rank != 0:
        return None
    lines = [l for l in so.splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else {"isolated": True, "error": "no result line"}


_LINK_TYPES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}


def peer_links(me_dev, peer_devs):
    """Per peer device, what HIP reports about the path from this rank's device to it:
    hipDeviceCanAccessPeer, hipDeviceGetP2PAttribute (performance rank, access, native atomics)
    and hipExtGetLinkTypeAndHopCount (HSA link type: 4 = xGMI). Measurement-side ctypes calls on
    the HIP runtime torch already loaded (no libghx entry point)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = {}
    for pd in sorted(set(peer_devs)):
        r = {"device": pd}
        if pd == me_dev:
            r["same_device"] = True
            out[str(pd)] = r
            continue
        c = ctypes.c_int(0)
        r["can_access_peer"] = (bool(c.value) if hip.hipDeviceCanAccessPeer(
            ctypes.byref(c), me_dev, pd) == 0 else None)
        for name, attr in (("perf_rank", 0), ("access_supported", 1), ("native_atomics", 2)):
            v = ctypes.c_int(0)
            r[name] = (v.value if hip.hipDeviceGetP2PAttribute(ctypes.byref(v), attr, me_dev, pd)
                       == 0 else None)
        lt, hops = ctypes.c_uint32(0), ctypes.c_uint32(0)
        if hip.hipExtGetLinkTypeAndHopCount(me_dev, pd, ctypes.byref(lt), ctypes.byref(hops)) == 0:
            r["link"] = _LINK_TYPES.get(lt.value, str(lt.value))
            r["hops"] = hops.value
        out[str(pd)] = r
    return out


def transport_certificate(torch, dist, dev, plan, me, world, backend):
    """The N>1 line's own evidence of what carried its peer messages: the
    process group's size and backend; on RCCL, the rank count its communicator actually reduces
    over (an all-reduce of ones on the device, so a communicator that spans fewer ranks than the
    job shows here, not in a later number); every rank's device and PCI bus id; and per peer
    rank, the device path (peer_links) and the bytes this rank sends to / receives from it per
    step. `certified` = the backend's ranks equal the world size and every peer is on a distinct
    device."""
    import ctypes
    cert = {"world_size": dist.get_world_size(), "backend": dist.get_backend()}
    if cert["backend"] == "nccl":
        t = torch.ones(1, dtype=torch.float32, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize(dev)
        cert["rccl_ranks"] = int(t.item())
        try:
            v = torch.cuda.nccl.version()
            cert["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception as e:  # reported, not fatal
            cert["rccl_version"] = f"unavailable: {type(e).__name__}"
    else:
        cert["rccl_ranks"] = None
    bus = ctypes.create_string_buffer(64)
    hip = ctypes.CDLL("libamdhip64.so")
    mine = {"device": dev.index, "pci_bus_id": bus.value.decode()
            if hip.hipDeviceGetPCIBusId(bus, 64, dev.index) == 0 else None}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    cert["devices"] = [a["device"] for a in allr]
    cert["pci_bus_ids"] = [a["pci_bus_id"] for a in allr]
    sent, got = {}, {}
    for x in plan.send:
        if x["rank"] != me:
            sent[x["rank"]] = sent.get(x["rank"], 0) + x["size"]
    for x in plan.recv:
        if x["rank"] != me:
            got[x["rank"]] = got.get(x["rank"], 0) + x["size"]
    peers = sorted(set(sent) | set(got))
    try:
        links = peer_links(dev.index, [allr[p]["device"] for p in peers])
    except Exception as e:  # reported; the rank count above is the certificate's core
        links = {str(allr[p]["device"]): {"error": f"{type(e).__name__}: {str(e)[:100]}"}
                 for p in peers}
    cert["peers"] = {str(p): {"bytes_sent_per_step": sent.get(p, 0),
                              "bytes_received_per_step": got.get(p, 0),
                              **links[str(allr[p]["device"])]} for p in peers}
    distinct = len(set(cert["pci_bus_ids"])) == world and None not in cert["pci_bus_ids"]
    cert["certified"] = bool(cert["backend"] == "nccl" and cert["rccl_ranks"] == world and
                             distinct)
    if not cert["certified"]:
        why = []
        if cert["backend"] != "nccl":
            why.append(f"backend {cert['backend']} (not RCCL)")
        elif cert["rccl_ranks"] != world:
            why.append(f"RCCL reduced over {cert['rccl_ranks']} ranks, not {world}")
        if not distinct:
            why.append("ranks share a device")
        cert["why_not"] = "; ".join(why)
    return cert


def main():
    args = parse()
    if args.bulk_child:
        return bulk_child(args)
    if args.bulk_only:
        sys.exit(bulk_only(args))  # before anything touches the GPU
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_workers(args))  # before anything touches the GPU
    import threading

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world not in DECOMP:
        raise SystemExit(f"--gpus must be one of {sorted(DECOMP)}")
    if args.rehearse:
        local = 0
    distributed = world > 1 or args.force_dist
    backend = None
    N, Hw = args.N, args.halo
    parts = DECOMP[world]
    guard = StageGuard({
        "metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "config": {"N": N, "halo": Hw, "decomposition": list(parts)}}, rank)
    _LINE["guard"] = guard
    with guard.stage("init_process_group", args.init_timeout):
        if distributed:
            import datetime
            backend = "gloo" if args.rehearse else "nccl"
            # the process group's own timeout stays above the guard's stages, so a stuck
            # collective is reported by the guard (with a line), not aborted by the watchdog
            pg_timeout = datetime.timedelta(seconds=60 + max(
                args.init_timeout, args.exchange_timeout, args.headline_timeout))
            if args.rehearse:
                dist.init_process_group("gloo", timeout=pg_timeout)
                torch.cuda.set_device(local)
            else:
                torch.cuda.set_device(local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                        timeout=pg_timeout)
        else:
            torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

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

    E = N + 2 * Hw
    G = [parts[d] * N for d in range(3)]
    c = (rank % parts[0], (rank // parts[0]) % parts[1], rank // (parts[0] * parts[1]))
    first = tuple(c[d] * N for d in range(3))
    last = tuple((c[d] + 1) * N - 1 for d in range(3))

    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(rank, first, last)
    hg = R.HaloGenerator((0, 0, 0), tuple(g - 1 for g in G), (Hw,) * 6, (True,) * 3)
    with guard.stage("pattern_setup", args.init_timeout):  # the setup all-gather
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

    idx = [torch.arange(E, device=dev, dtype=torch.int64) - Hw + first[d] for d in range(3)]
    wrap = [(idx[d] % G[d]).to(torch.float64) for d in range(3)]

    def verify():
        """Every cell of this rank's (N+2H)^3 box = its wrapped global index (summed over ranks)."""
        expect = wrap[0].view(1, 1, E) + G[0] * (wrap[1].view(1, E, 1) +
                                                 G[1] * wrap[2].view(E, 1, 1))
        bad = int((base != expect).sum().item())
        del expect
        if distributed:
            bad = int(all_reduce_host(bad, dist.ReduceOp.SUM))
        return bad

    def clear_halos():
        base.fill_(-1.0)
        base[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = (
            ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)))

    # ---- verified full exchange (pack -> RCCL -> unpack) --------------------------------------
    with guard.stage("verified_exchange", args.exchange_timeout):
        co.exchange(bis).wait()
        verified = verify() == 0
    headline = guard.stage("headline", args.headline_timeout)
    headline.__enter__()

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

    def pack(s):
        rc = L.ghx_exchange_pack(plan.h, fptr, 1, sptr, ns, s)
        if rc:
            raise RuntimeError(L.ghx_last_error().decode())

    def unpack(s):
        rc = L.ghx_exchange_unpack(plan.h, fptr, 1, rptr, nr, s)
        if rc:
            raise RuntimeError(L.ghx_last_error().decode())

    def fused(s):
        rc = L.ghx_exchange_self(plan.h, fptr, 1, sptr, ns, s)
        if rc:
            raise RuntimeError(L.ghx_last_error().decode())

    def step():
        s = torch.cuda.current_stream(dev).cuda_stream
        pack(s)
        unpack(s)

    K, W = args.steps, args.warmup
    spg = args.steps_per_graph or min(K, 1000)  # steps per hipGraph
    runner = Runner(torch, dev, stream, step, spg, eager=args.no_graph)
    runner.prepare(W)
    runner.prepare(K)
    runner.run(W)
    torch.cuda.synchronize(dev)

    def timed(fn, k, events=False, box=None):
        """Host wall time of k calls, max over ranks: barrier + synchronize, start the clock,
        the calls, synchronize, stop the clock, barrier (each rank's clock runs from the common
        start to its own completion; the closing barrier's own latency is not charged). With
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
        dt = time.perf_counter() - t0
        if events and box is not None:
            box["s"] = e0.elapsed_time(e1) * 1e-3
        if distributed:
            barrier()
            dt = all_reduce_host(dt, dist.ReduceOp.MAX)
        return dt

    dev_time = {}
    T = timed(lambda: runner.run(K), 1, events=True, box=dev_time)
    dev_step = dev_time["s"] / K  # device time per step over the timed region (HIP events)
    # `verified` refers to the kernels just timed: halos back to -1, every buffer byte to 0xFF,
    # the timed graph replayed once (N>1: then the peer messages' transport and an unpack), every
    # cell checked. The first exchange above (at N=1 the fused k_self) is `verified_fused`.
    verified_fused = verified
    me = rank
    t_sends = [(x["rank"], x["tag"], send[i][:x["size"]]) for i, x in enumerate(plan.send)
               if x["rank"] != me]
    t_recvs = [(x["rank"], x["tag"], recv[i][:x["size"]]) for i, x in enumerate(plan.recv)
               if x["rank"] != me]

    def transport():
        """Deliver the send buffers the replay packed into the receive buffers (N>1)."""
        from ghex_amd.communication_object import route
        if args.rehearse:
            co._exchange_host_staged(plan, t_sends, t_recvs, stream)
        else:
            for w in route(ctx, t_sends, t_recvs):
                w.wait()

    with guard.stage("verify_timed", args.exchange_timeout):
        verified = verify_replay(torch, dev, lambda: runner.run(K), clear_halos, verify,
                                 send, recv, transport if t_recvs else None) == 0
    value = world * step_bytes * K / T / 1e9
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
        "steps": K, "warmup": W, "ms_per_step": round(T / K * 1e3, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (owned cell = global linear index; halos -1 before every verification)",
        "config": {
            "workload": f"{N}^3 fp64 structured 3D halo={Hw}, 26-neighbour periodic, "
                        f"device-resident pack+unpack, decomposition {list(parts)}",
            "N": N, "halo": Hw, "fields": 1, "decomposition": list(parts),
            "launch": ("eager" if args.no_graph else
                       f"hipGraphs of {spg} steps, instantiated before the timed region") +
                      ", pack launch + unpack launch per step",
            "bytes_per_step_per_gpu": step_bytes,
            "parallelism": f"{world} rank(s), one domain per GPU",
            "world_size": world, "backend": backend,
        },
        "verified": verified,
        "verified_what": "after the timed region, on halos reset to -1 and every buffer byte "
                         "set to 0xFF: the timed hipGraphs (k_copy pack + k_copy unpack, K "
                         "steps) replayed" +
                         ("" if world == 1 else ", the peer messages transported into the "
                                                "receive buffers, the timed hipGraphs replayed "
                                                "again (the peer halos written by their unpack)") +
                         "; every cell of every rank checked",
        "verified_fused": verified_fused,
        "verified_fused_what": ("the first exchange: co.exchange() = the fused k_self launch"
                                if world == 1 and co.fuse_self and co.all_self(plan) else
                                "the first exchange: co.exchange() = pack, transport, unpack"),
    }
    if args.rehearse:
        out["rehearsal"] = ("all ranks on cuda:0, gloo + host-staged transport: code-path check, "
                            "not the metric")
    if distributed:
        with guard.stage("transport_certificate", args.exchange_timeout):
            cert = transport_certificate(torch, dist, dev, plan, rank, world, backend)
        out["transport"] = cert
        if cert["backend"] == "nccl" and cert["rccl_ranks"] != world:
            # the peer messages did not cross a communicator of N ranks: not the N-GPU metric
            out["verified"] = False
            out["verified_what"] += f"; NOT certified: {cert.get('why_not')}"

    # ---- per-kernel HIP-event durations (dominant kernel roofline) ----------------------------
    # Differential method (removes the events' own cost): hipGraphs of M steps, of M steps + one
    # pack, and of M steps + one pack + one unpack, replayed in interleaved rounds (medians);
    # pack = T1 - T0, unpack = T2 - T1.
    t_pack, t_unpack = kernel_durations(torch, dev, stream, [pack, unpack])
    if min(t_pack, t_unpack) <= 1e-7:
        # a differential drowned in noise (ranks sharing one GPU in a rehearsal): fall back to
        # chains of one kernel alone (graphs of M packs, of M unpacks)
        t_pack, t_unpack = (chain_duration(torch, dev, stream, pack),
                            chain_duration(torch, dev, stream, unpack))
    # each kernel's own begin-to-end interval (hipExtLaunchKernel start/stop events, the interval
    # a rocprofv3 kernel trace reports), eager steps, medians
    k_pack, k_unpack = launch_durations(torch, dev, stream, _ghx, [pack, unpack])
    if min(k_pack, k_unpack) <= 0:
        k_pack, k_unpack = t_pack, t_unpack
    if distributed:  # the slowest rank's figures (the line is rank 0's)
        dev_step = all_reduce_host(dev_step, dist.ReduceOp.MAX)
        k_pack = all_reduce_host(k_pack, dist.ReduceOp.MAX)
        k_unpack = all_reduce_host(k_unpack, dist.ReduceOp.MAX)
    dom_name, dom_d = ("pack", t_pack) if k_pack >= k_unpack else ("unpack", t_unpack)
    dom_k = max(k_pack, k_unpack)
    # the dominant launch's share of the timed region's device time (HIP events around the K
    # steps on the launch stream), split in the ratio of the kernels' own durations: conservative
    # (the step's inter-launch gaps are charged to the launches), and within a few % of the
    # rocprofv3 kernel-trace mean of the same launches
    dom_t = dev_step * dom_k / (k_pack + k_unpack)
    launch_bytes = 2 * n_halo * 8  # read n*s + write n*s, either kernel
    achieved = launch_bytes / dom_t / 1e9
    traffic, traffic_src, pmc_step_bytes = None, None, None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            # N=1: the one-domain plan; N>1: rank 0's plan of the same decomposition (every rank's
            # plan is a translate of it), profiled on one GPU through tools/emu_rank_bench.py
            cfg = tj.get(f"N{N}_H{Hw}" + ("" if world == 1 else f"_w{world}"), {})
            ent = cfg.get(dom_name)
            if ent:
                traffic = ent.get("hbm_bytes_per_launch")
                traffic_src = ent.get("source", tj.get("source"))
            both = [cfg.get(k, {}).get("hbm_bytes_per_launch") for k in ("pack", "unpack")]
            if all(both):
                pmc_step_bytes = sum(both)
        except Exception:
            traffic = None
    out["roofline"] = {
        "bound": "hbm", "kernel": f"k_copy<{dom_name}>",
        "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
        "traffic_source": traffic_src,
        "algorithmic_bytes_per_launch": launch_bytes,
        "launch_us": round(dom_t * 1e6, 2),
        "launch_us_source": "HIP events on the launch stream around the K timed steps: device "
                            "time per step x the kernel's share of the step, the share from "
                            "the kernels' own start/stop events (pack_kernel_us, "
                            "unpack_kernel_us: hipExtLaunchKernel events, eager steps, medians)",
        "launch_us_kernel_events": round(dom_k * 1e6, 2),
        "pack_kernel_us": round(k_pack * 1e6, 2), "unpack_kernel_us": round(k_unpack * 1e6, 2),
        "launch_us_differential": round(dom_d * 1e6, 2),
        "pack_us": round(t_pack * 1e6, 2), "unpack_us": round(t_unpack * 1e6, 2),
        "step_device_us": round(dev_step * 1e6, 2),
        "step_achieved": round(step_bytes / dev_step / 1e9, 1),
        "step_frac": round(step_bytes / dev_step / 1e9 / HBM_PEAK_GBS, 4),
    }

    headline.__exit__(None, None, None)

    # ---- extras (bounded: the line is printed without them if they overrun) -------------------
    done = threading.Event()
    printed = threading.Lock()

    def emit(o):
        if rank == 0 and printed.acquire(blocking=False):
            print(json.dumps(o), flush=True)
            _LINE["printed"] = True

    extras_done = threading.Event()

    def watchdog():
        # the extras and the teardown after them are bounded: a rank stuck in a collective (a
        # peer failed in the extras) prints the line without them and leaves
        if not extras_done.wait(args.extras_timeout):
            o = dict(out)
            o["extras_error"] = f"extras exceeded {args.extras_timeout:.0f} s; printed without them"
            emit(o)
        if not done.wait(60.0 if extras_done.is_set() else 5.0):
            sys.stdout.flush()
            os._exit(0)

    threading.Thread(target=watchdog, daemon=True).start()
    try:
        extras(args, torch, dist, dev, stream, out, locals())
    except Exception as e:  # reported, never fatal for the headline measurement
        import traceback
        out["extras_error"] = f"{type(e).__name__}: {str(e)[:300]}"
        out["extras_traceback"] = traceback.format_exc()[-1200:]
    extras_done.set()
    emit(out)
    sys.stdout.flush()
    if distributed:
        barrier()
        dist.destroy_process_group()
    done.set()


def extras(args, torch, dist, dev, stream, out, v):
    """Everything after the headline: cold caches, fused self exchange, full exchanges,
    host staging, other configs, CPU baseline."""
    world, rank, K = v["world"], v["rank"], v["K"]
    pack, unpack, fused, timed = v["pack"], v["unpack"], v["fused"], v["timed"]
    co, bis, plan, send, recv = v["co"], v["bis"], v["plan"], v["send"], v["recv"]
    n_halo, step_bytes, launch_bytes = v["n_halo"], v["step_bytes"], v["launch_bytes"]
    ghex_amd, R, L, _ghx, N, Hw = v["ghex_amd"], v["R"], v["L"], v["_ghx"], v["N"], v["Hw"]
    roof = out["roofline"]
    all_reduce_host, local = v["all_reduce_host"], v["local"]
    t_extras = time.perf_counter()

    if not args.no_cold:
        # Cold caches: an application's stencil sweeps the whole field between exchanges, so the
        # halo-adjacent lines are not left in the 256 MiB Infinity Cache as they are when the
        # bench replays steps back to back. A 1 GiB read-only reduction before every launch
        # evicts them without leaving dirty lines (cold, clean); a 1 GiB read-modify-write
        # leaves 1 GiB dirty that the launch then evicts (cold, dirty). Flushes differenced away.
        fl = torch.zeros(1 << 27, dtype=torch.float64, device=dev)
        acc = torch.empty((), dtype=torch.float64, device=dev)
        clean = lambda s: torch.sum(fl, dim=(0,), out=acc)  # noqa: E731
        t_pc = cold_duration(torch, dev, stream, pack, clean)
        t_uc = cold_duration(torch, dev, stream, unpack, clean)
        t_dom = t_pc if roof["kernel"] == "k_copy<pack>" else t_uc
        roof["cold_clean_launch_us"] = round(t_dom * 1e6, 2)
        roof["cold_clean_achieved"] = round(launch_bytes / t_dom / 1e9, 1)
        roof["cold_clean_frac"] = round(launch_bytes / t_dom / 1e9 / HBM_PEAK_GBS, 4)
        roof["cold_clean_pack_us"] = round(t_pc * 1e6, 2)
        roof["cold_clean_unpack_us"] = round(t_uc * 1e6, 2)
        # the step as an application runs it after a stencil sweep: flush, then pack and unpack
        # back to back (the unpack's halo lines are the ones the pack has just fetched; flushed
        # separately, each launch above pays its own misses)
        # the same cold launches by the kernels' own events (like pack_kernel_us): what the
        # launch itself takes after the flush, without the deferred write-back the differenced
        # figures above charge to it
        _ghx_ = v["_ghx"]
        (kpc,) = cold_launch_durations(torch, dev, stream, _ghx_, [pack], clean)
        (kuc,) = cold_launch_durations(torch, dev, stream, _ghx_, [unpack], clean)
        kspc, ksuc = cold_launch_durations(torch, dev, stream, _ghx_, [pack, unpack], clean)
        roof["cold_clean_kernel_events_us"] = {
            "pack": round(kpc * 1e6, 2), "unpack": round(kuc * 1e6, 2),
            "step_pack": round(kspc * 1e6, 2), "step_unpack": round(ksuc * 1e6, 2),
            "method": "flush, then the launch(es) with hipExtLaunchKernel start/stop events, "
                      "medians of 15; step_*: flush, pack, unpack"}
        # which memory served the bytes: the timed steps replay back to back, so
        # the step's whole footprint (pack line reads + buffer writes + buffer reads + halo lines,
        # the two launches' PMC bytes, ~145 MB at 512^3 H=2) stays in the 256 MB Infinity Cache
        # and the headline `frac` is a warm figure; after the 1 GiB read-only sweep the same
        # launch is served from HBM. Both, by the kernel's own events.
        k_cold = kpc if roof["kernel"] == "k_copy<pack>" else kuc
        k_warm = roof["launch_us_kernel_events"] * 1e-6
        pf = v.get("pmc_step_bytes")
        roof["cold"] = {
            "launch_us": round(k_cold * 1e6, 2),
            "achieved": round(launch_bytes / k_cold / 1e9, 1),
            "frac": round(launch_bytes / k_cold / 1e9 / HBM_PEAK_GBS, 4),
            "step_us": round((kspc + ksuc) * 1e6, 2),
            "step_frac": round(step_bytes / (kspc + ksuc) / 1e9 / HBM_PEAK_GBS, 4),
            "served_by": "HBM: every launch follows a 1 GiB read-only sweep that evicts the "
                         "halo-adjacent lines from the Infinity Cache (as an application's stencil "
                         "sweep does)"}
        roof["warm"] = {
            "launch_us": round(k_warm * 1e6, 2),
            "frac": round(launch_bytes / k_warm / 1e9 / HBM_PEAK_GBS, 4),
            "served_by": "Infinity Cache (256 MB MALL): steps replayed back to back"
                         + (f"; the step's PMC footprint {pf / 1e6:.1f} MB fits in it" if pf
                            else ""),
            "note": "the headline roofline.frac is this regime (the step share of the timed "
                    "region); frac against the HBM peak is a conservative yardstick here"}
        t_sc = cold_duration(torch, dev, stream, lambda s: (pack(s), unpack(s)), clean)
        roof["cold_clean_step_us"] = round(t_sc * 1e6, 2)
        roof["cold_clean_step_GBps"] = round(step_bytes / t_sc / 1e9, 1)
        dirty = lambda s: fl.add_(1.0)  # noqa: E731
        t_dirty = cold_duration(torch, dev, stream, pack if t_dom == t_pc else unpack, dirty)
        roof["cold_dirty_launch_us"] = round(t_dirty * 1e6, 2)
        t_sd = cold_duration(torch, dev, stream, lambda s: (pack(s), unpack(s)), dirty)
        roof["cold_dirty_step_us"] = round(t_sd * 1e6, 2)
        if world == 1 and co.fuse_self and co.all_self(plan):
            v["cold_fused"] = (cold_duration(torch, dev, stream, fused, clean),
                               cold_duration(torch, dev, stream, fused, dirty))
        del fl
        torch.cuda.empty_cache()

    if world == 1 and co.fuse_self and co.all_self(plan):
        # The product's N=1 exchange: ONE launch (k_self). Each lane packs its buffer bytes and
        # writes the halos from the same registers: read n*s + buffer write n*s + halo write n*s.
        (t_f,) = kernel_durations(torch, dev, stream, [fused])
        moved = 3 * n_halo * 8
        out["fused_self"] = {
            "kernel": "k_self", "launch_us": round(t_f * 1e6, 2), "bytes_moved": moved,
            "GBps_moved": round(moved / t_f / 1e9, 1),
            "frac_moved": round(moved / t_f / 1e9 / HBM_PEAK_GBS, 4),
            "exchange_equivalent_GBps": round(step_bytes / t_f / 1e9, 1),
            **({"cold_clean_launch_us": round(v["cold_fused"][0] * 1e6, 2),
                "cold_dirty_launch_us": round(v["cold_fused"][1] * 1e6, 2)}
               if "cold_fused" in v else {}),
            "note": "pack+unpack of the same cells in one launch; the buffer is written but "
                    "never read back, so bytes_moved = 3*n*8 (the metric's 4*n*8 is the "
                    "two-launch step)"}

    if args.no_extras:
        return
    # full exchange incl. transport (RCCL for N>1; self-message aliasing for N=1)
    ke = min(K, 50)
    for _ in range(3):
        co.exchange(bis).wait()
    Te = timed(lambda: co.exchange(bis).wait(), ke)
    out["exchange_ms_per_step"] = round(Te / ke * 1e3, 4)
    if world > 1 and not args.rehearse:
        # the transport alone: the same peer messages as one RCCL group per step, no pack or
        # unpack (what exchange_ms_per_step adds to the two kernels)
        from ghex_amd.communication_object import route
        me = rank
        tsends = [(x["rank"], x["tag"], send[i][:x["size"]]) for i, x in enumerate(plan.send)
                  if x["rank"] != me]
        trecvs = [(x["rank"], x["tag"], recv[i][:x["size"]]) for i, x in enumerate(plan.recv)
                  if x["rank"] != me]

        def transport_only():
            for w in route(v["ctx"], tsends, trecvs):
                w.wait()
            torch.cuda.current_stream(dev).synchronize()
        try:
            for _ in range(3):
                transport_only()
            Tt = timed(transport_only, ke)
            out["transport_ms_per_step"] = round(Tt / ke * 1e3, 4)
            out["transport_bytes_per_step_per_gpu"] = sum(t.numel() for _, _, t in tsends)
        except Exception as e:  # reported; the legs after it still run
            out["transport_error"] = f"{type(e).__name__}: {str(e)[:200]}"
        co.exchange(bis).wait()  # halos valid again (the recv buffers were overwritten)
    if world > 1:
        # per-peer streams (rehearsal: the host-staged form of the same pipeline over gloo); the
        # pair communicators are created here, at the first pipelined exchange: their failure is
        # reported in this leg and never reaches the headline
        try:
            cop = R.make_communication_object(v["ctx"], pipelined=True,
                                              staging="host" if args.rehearse else None)
            v["clear_halos"]()
            cop.exchange(bis).wait()
            okp = v["verify"]() == 0
            for _ in range(3):
                cop.exchange(bis).wait()
            Tp = timed(lambda: cop.exchange(bis).wait(), ke)
            out["exchange_pipelined"] = {"ms_per_step": round(Tp / ke * 1e3, 4), "verified": okp,
                                         "mode": "per-peer streams: pack, " +
                                                 ("D2H, gloo send/recv, H2D" if args.rehearse else
                                                  "one RCCL group on the pair's own communicator") +
                                                 " and unpack of each peer's buffers on its stream"}
            del cop
        except Exception as e:  # reported; the legs after it still run
            out["exchange_pipelined"] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
        co.exchange(bis).wait()  # halos valid again
    if world > 1:
        # the unstructured path between real ranks at BASELINE config 5's size (10M cells per
        # rank; the pattern built from reduced halos): setup time, verified, timed
        try:
            out["unstructured_exchange"] = bench_unstructured(v, torch, dist, dev, args)
        except Exception as e:  # reported; the legs after it still run
            out["unstructured_exchange"] = {"error": f"{type(e).__name__}: {str(e)[:200]}"}
    # the north star's other halo widths, same decomposition, same two-launch step, verified
    out["halo_widths"] = {str(h): bench_halo(h, v, torch, dist, dev, stream, args)
                          for h in (1, 3) if h != Hw}
    if world == 1 and N == 512 and Hw == 2 and not args.no_layout:
        # the same cells and bytes in a field whose x rows are allocated 2 cells wider (row pitch
        # 4,144 B instead of 4,128 B): what the x-face lines' address set costs
        out["layout_x_alloc_518"] = bench_halo(Hw, v, torch, dist, dev, stream, args, x_alloc=518)
    if world > 1 and not args.bulk:
        # the zero-copy exchange between GPUs, isolated in child processes (bulk_isolated); every
        # rank takes part (the children rendezvous among themselves on a fresh port)
        try:
            import socket
            port = 0
            if rank == 0:
                sk = socket.socket()
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
                sk.close()
            port = int(all_reduce_host(float(port), dist.ReduceOp.MAX))
            # inside the extras' own budget (the watchdog prints without them at
            # --extras-timeout): every rank agrees on the time the children get
            left = args.extras_timeout - (time.perf_counter() - t_extras) - 30.0
            left = all_reduce_host(left, dist.ReduceOp.MIN)
            if args.rehearse and world > 4:
                # every rank and its child on the ONE GPU of a rehearsal: 2N processes would pass
                # the test box's limit of 16 per GPU (at N=8 on 8 GPUs each GPU holds two)
                res = {"isolated": True, "skipped": "rehearsal with all ranks on one GPU (2N "
                                                    "processes on it); runs at N=2/4 and as "
                                                    "--bulk-only 8"}
            elif left < 30.0:
                res = {"isolated": True, "skipped": "the extras' time budget is spent"}
            else:
                res = bulk_isolated(args, rank, world, local, port, min(args.bulk_timeout, left))
            if rank == 0:
                out["bulk"] = res
        except Exception as e:  # reported, never fatal for the headline measurement
            out["bulk"] = {"isolated": True, "error": f"{type(e).__name__}: {str(e)[:200]}"}
    if world == 1 or args.bulk:
        # zero-copy bulk exchange (BulkCommunicationObject): puts straight into the
        # receivers' halos, no buffers: 2*n*8 bytes moved per step (not the metric's 4*n*8)
        try:
            bco = ghex_amd.make_bulk_communication_object(v["ctx"])
            bco.add_field(bis[0])
            bco.init()
            for _ in range(3):
                bco.exchange().wait()
            # stream-ordered (device epochs): K exchanges back to back, one host sync at the end;
            # and with a host wait after every exchange (what a caller that blocks pays)
            Tb = timed(lambda: bco.exchange(), ke)
            bco.check_epochs()
            Tbw = timed(lambda: bco.exchange().wait(), ke)
            # the whole exchange (epochs + puts) captured into a graph of 10 and replayed
            Tbg = _time_graph(torch, dev, lambda s: bco.exchange(), k=min(K, 50))
            bco.check_epochs()
            put = bco._puts[0]

            def put_fn(s):
                rc = L.ghx_put_execute(put[0], put[1], put[2], put[3], put[4], s)
                if rc:
                    raise RuntimeError(L.ghx_last_error().decode())
            (t_put,) = kernel_durations(torch, dev, stream, [put_fn])
            out["bulk"] = {"exchange_ms_per_step": round(Tb / ke * 1e3, 4),
                           "exchange_wait_ms_per_step": round(Tbw / ke * 1e3, 4),
                           "exchange_graph_ms_per_step": round(Tbg * 1e3, 4),
                           "epochs": bco.epochs,
                           "put_launches": len(bco._puts),
                           "put_us": round(t_put * 1e6, 2) if len(bco._puts) == 1 else None,
                           "bytes_moved_per_step": 2 * n_halo * 8}
            del bco
        except Exception as e:  # reported, never fatal for the headline measurement
            out["bulk"] = {"error": str(e)[:200]}
        co.exchange(bis).wait()
    if world == 1:
        out["host_staged"] = host_staged(torch, dev, co, plan, send, recv, pack, unpack, timed,
                                         step_bytes, n_halo, min(K, 50))
        co.exchange(bis).wait()  # restore valid halos after the staged copies

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
        roof["measured_d2d_copy_GBps"] = round(2 * a.numel() * 10 /
                                               (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
        del a, b
        torch.cuda.empty_cache()
        if world == 1:
            roof["read_floor"] = pack_read_floor(N, Hw, roof)
            if "fused_self" in out:
                out["fused_self"]["floor"] = fused_floor(N, Hw, out["fused_self"]["launch_us"])

    if world == 1:
        # the other BASELINE configs, per GPU (their 8-GPU forms are weak-scaled copies)
        for k in ("base", "logical", "fd", "bis", "send", "recv"):
            v.pop(k, None)
        del bis, send, recv
        co = None
        torch.cuda.empty_cache()
        cs = None if (rank != 0 or args.no_cpu_baseline) else args.cpu_config_seconds
        ex = out["extra_configs"] = {}
        # each config reported on its own: a failure is recorded in its entry and the ones after
        # it (and the headline's cpu_baseline) still run
        try:
            ex["config4_5fields_256^3_h3_f64f32"] = bench_config4(torch, dev, ghex_amd, R, cs)
        except Exception as e:
            ex["config4_5fields_256^3_h3_f64f32"] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
        torch.cuda.empty_cache()
        try:
            pats, t_all, t_rank = config5_patterns()
            for lv in (1, 8):
                name = f"config5_unstructured_10M_5pct_levels{lv}"
                try:
                    ex[name] = bench_config5(torch, dev, _ghx, lv, pats, cs)
                except Exception as e:
                    ex[name] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
                torch.cuda.empty_cache()
            ex["config5_pattern_setup"] = {
                "ranks": 8, "cells_per_rank": int(pats[0][0].size - pats[0][1].size),
                "seconds_all_ranks": round(t_all, 2), "seconds_max_rank": round(t_rank, 2),
                "what": "8 ranks as threads of this process (LoopbackWorld), each generating its "
                        "domain and running the product make_pattern<unstructured> (reduced halos)"}
            del pats
        except Exception as e:
            ex["config5_pattern_setup"] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, Hw, args.cpu_seconds)


def _floor_lib():
    import ctypes
    path = os.path.join(ROOT, "tools", "lib", "libpackfloor.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    for name in ("ghx_probe_pack_floor", "ghx_probe_unpack_floor"):
        f = getattr(L, name)
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                      ctypes.POINTER(ctypes.c_int64)]
    L.ghx_probe_fused_floor.restype = ctypes.c_int
    L.ghx_probe_fused_floor.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double)]
    L.ghx_probe_multi_floor.restype = ctypes.c_int
    L.ghx_probe_multi_floor.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int64)]
    P32 = ctypes.POINTER(ctypes.c_int32)
    L.ghx_probe_index_floor.restype = ctypes.c_int
    L.ghx_probe_index_floor.argtypes = [ctypes.c_int64, ctypes.c_int, P32, ctypes.c_int64, P32,
                                        ctypes.c_int64, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double)]
    return L


def index_floor(cells, levels, sends, recvs, k_gather, k_scatter):
    """Config 5's index-list floor (tools/pack_floor.hip ghx_probe_index_floor): the simplest
    gather / scatter kernels over the same lid lists (one value per lane, no plan), timed by their
    own begin/end events like the product's launches (k_gather / k_scatter, seconds).
    floor_over_kernel = probe time / product time (above 1: the product is faster)."""
    import ctypes

    import numpy as np
    try:
        L = _floor_lib()
        if L is None:
            return {"error": "tools/lib/libpackfloor.so not built (make -C tools)"}
        sl = np.ascontiguousarray(np.concatenate([l for *_, l in sends]), dtype=np.int32)
        rl = np.ascontiguousarray(np.concatenate([l for *_, l in recvs]), dtype=np.int32)
        us = (ctypes.c_double * 4)()
        P32 = ctypes.POINTER(ctypes.c_int32)
        rc = L.ghx_probe_index_floor(cells, levels, sl.ctypes.data_as(P32), sl.size,
                                     rl.ctypes.data_as(P32), rl.size, 21, us)
        if rc:
            return {"error": f"HIP call failed at tools/pack_floor.hip:{rc}"}
        return {"gather_us": round(us[0], 2), "scatter_us": round(us[2], 2),
                "gather_cold_us": round(us[1], 2), "scatter_cold_us": round(us[3], 2),
                "pack_kernel_us": round(k_gather * 1e6, 2),
                "unpack_kernel_us": round(k_scatter * 1e6, 2),
                "gather_floor_over_kernel": round(us[0] / (k_gather * 1e6), 3) if k_gather else None,
                "scatter_floor_over_kernel": round(us[2] / (k_scatter * 1e6), 3)
                if k_scatter else None,
                "what": "the simplest gather / scatter kernels over the same lid lists (one fp64 "
                        "value per lane, no plan), kernel-own events, medians of 21"}
    except Exception as e:  # reported, never fatal
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}


def multi_floor(N, H, elem_sizes, k_pack, k_unpack):
    """Config 4's address-set floors (tools/pack_floor.hip ghx_probe_multi_floor): the fields
    (element sizes `elem_sizes`) in one allocation at 2 MiB-aligned offsets. Pack: one 16-B load
    per 128-B field line the pack reads (x-face lines first) + the buffer writes. Unpack: every
    halo row's bytes written once (16/8/4-B pieces from an address-ordered list), the write set
    the unpack must issue (unpack_floor_us, as write_floor of pack_read_floor); with the buffer
    read streamed first beside it (unpack_reads_writes_us). Kernel-own events, medians of 21,
    beside the product's pack / unpack launches (k_pack / k_unpack, seconds).
    floor_over_kernel = probe time / product time (above 1: the product is faster)."""
    import ctypes
    try:
        L = _floor_lib()
        if L is None:
            return {"error": "tools/lib/libpackfloor.so not built (make -C tools)"}
        us = (ctypes.c_double * 6)()
        c = (ctypes.c_int64 * 3)()
        es = (ctypes.c_int * len(elem_sizes))(*elem_sizes)
        rc = L.ghx_probe_multi_floor(N, H, len(elem_sizes), es, 21, us, c)
        if rc:
            return {"error": f"HIP call failed at tools/pack_floor.hip:{rc}"}
        return {"lines": c[0], "pieces": c[1], "halo_bytes": c[2],
                "pack_floor_us": round(us[0], 2), "pack_floor_cold_us": round(us[1], 2),
                "unpack_floor_us": round(us[4], 2), "unpack_floor_cold_us": round(us[5], 2),
                "unpack_reads_writes_us": round(us[2], 2),
                "unpack_reads_writes_cold_us": round(us[3], 2),
                "pack_kernel_us": round(k_pack * 1e6, 2),
                "unpack_kernel_us": round(k_unpack * 1e6, 2),
                "pack_floor_over_kernel": round(us[0] / (k_pack * 1e6), 3) if k_pack else None,
                "unpack_floor_over_kernel": round(us[4] / (k_unpack * 1e6), 3)
                if k_unpack else None}
    except Exception as e:  # reported, never fatal
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}


def fused_floor(N, Hw, launch_us):
    """The fused self exchange's mirror (tools/pack_floor.hip ghx_probe_fused_floor): one launch
    that loads one vector per field line the pack reads, streams the buffer writes and writes
    every halo piece once — k_self's memory work without its index arithmetic."""
    import ctypes
    try:
        L = _floor_lib()
        if L is None:
            return {"error": "tools/lib/libpackfloor.so not built (make -C tools)"}
        us = (ctypes.c_double * 2)()
        rc = L.ghx_probe_fused_floor(N, Hw, 21, us)
        if rc:
            return {"error": f"HIP call failed at tools/pack_floor.hip:{rc}"}
        return {"floor_us": round(us[0], 2), "floor_cold_us": round(us[1], 2),
                "floor_over_kernel": round(us[0] / launch_us, 3) if launch_us else None}
    except Exception as e:  # reported, never fatal
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}


def pack_read_floor(N, Hw, roof):
    """The launches' address-set floors on this box (developer measurement, tools/pack_floor.hip
    via tools/lib/libpackfloor.so). Pack: a kernel that does nothing but load one
    16-B vector from each 128-B field line the pack must read (x-face lines first, as the pack
    dispatches them) and stream the buffer writes. Unpack ("write_floor"): a kernel that writes
    each halo row's bytes once (16-B pieces where aligned; floor_us), and the same with the
    buffer read (streamed first / interleaved with the writes). Timed like
    pack_kernel_us (the kernel's own begin/end events, medians). floor_over_kernel = floor time /
    kernel time: above 1 the kernel is FASTER than its probe, below 1 slower."""
    import ctypes
    try:
        L = _floor_lib()
        if L is None:
            return {"error": "tools/lib/libpackfloor.so not built (make -C tools)"}
        us = (ctypes.c_double * 10)()
        c = (ctypes.c_int64 * 3)()
        rc = L.ghx_probe_pack_floor(N, Hw, 21, us, c)
        if rc:
            return {"error": f"HIP call failed at tools/pack_floor.hip:{rc}"}
        out = {"xface_lines": c[0], "long_lines": c[1],
               "xface_only_us": round(us[0], 2), "long_only_us": round(us[2], 2),
               "reads_us": round(us[4], 2), "reads_writes_us": round(us[6], 2),
               "reads_writes_cold_us": round(us[7], 2),
               "reads_writes_dependent_us": round(us[8], 2),
               "reads_writes_dependent_cold_us": round(us[9], 2),
               "pack_kernel_us": roof.get("pack_kernel_us"),
               "floor_over_kernel": round(us[6] / roof["pack_kernel_us"], 3)
               if roof.get("pack_kernel_us") else None,
               "dependent_over_kernel": round(us[8] / roof["pack_kernel_us"], 3)
               if roof.get("pack_kernel_us") else None}
        rc = L.ghx_probe_unpack_floor(N, Hw, 21, us, c)
        if rc:
            out["write_floor"] = {"error": f"HIP call failed at tools/pack_floor.hip:{rc}"}
        else:
            # the floor: the halo pieces' writes alone (the unpack must issue them whatever it
            # does with its buffer reads). The two probes that add the buffer reads (streamed
            # first; interleaved with the writes, as the kernel issues them) are reported beside
            # it: both are slower than the kernel, which overlaps its reads better
            fl = us[4]
            out["write_floor"] = {
                "xface_pieces": c[0], "long_pieces": c[1],
                "xface_writes_us": round(us[0], 2), "long_writes_us": round(us[2], 2),
                "writes_us": round(us[4], 2), "writes_reads_us": round(us[6], 2),
                "writes_reads_cold_us": round(us[7], 2),
                "writes_reads_interleaved_us": round(us[8], 2),
                "writes_reads_interleaved_cold_us": round(us[9], 2),
                "floor_us": round(fl, 2),
                "unpack_kernel_us": roof.get("unpack_kernel_us"),
                "floor_over_kernel": round(fl / roof["unpack_kernel_us"], 3)
                if roof.get("unpack_kernel_us") else None}
        return out
    except Exception as e:  # reported, never fatal
        return {"error": f"{type(e).__name__}: {str(e)[:200]}"}


def host_staged(torch, dev, co, plan, send, recv, pack, unpack, timed, step_bytes, n_halo, k):
    """N=1 host-staged step: pack -> D2H into pinned memory -> H2D -> unpack (the NIC-side path
    of the north star; every message of the N=1 plan is a self message). Forms:
      runtime        hipMemcpyAsync D2H then H2D on the exchange stream (the runtime picks the
                     copy engines)
      probe          the same copies on the SDMA engines ghex_amd.staging measured (H2D starts
                     on its engine once the D2H has completed; L2 acquire before the unpack)
      probe_chunks_C the message in C chunks: H2D of chunk i behind the D2H of chunk i only, so
                     the two engines run both directions at once
    The line's value is the fastest form; every form's ms per step is listed."""
    from ghex_amd.staging import Copier
    hs = [torch.empty(b["size"], dtype=torch.uint8, pin_memory=True) for b in plan.send]
    pairs = []
    for i, b in enumerate(plan.recv):
        j = next(j for j, x in enumerate(plan.send) if x["pair"] == b["pair"])
        pairs.append((i, j, b["size"]))
    stream = torch.cuda.current_stream(dev)

    def runtime():
        s = stream.cuda_stream
        pack(s)
        for i, b in enumerate(plan.send):
            hs[i].copy_(send[i][:b["size"]], non_blocking=True)
        for i, j, n in pairs:
            recv[i][:n].copy_(hs[j], non_blocking=True)
        unpack(s)

    cp = Copier.for_device(dev)
    ev = torch.cuda.Event()

    def probe(chunks=1):
        s = stream.cuda_stream
        pack(s)
        ev.record(stream)
        ev.synchronize()
        last = []
        for i, j, n in pairs:
            c = (n + chunks - 1) // chunks
            for o in range(0, n, c):
                m = min(c, n - o)
                t = cp.d2h(hs[j].data_ptr() + o, send[j].data_ptr() + o, m)
                last.append(cp.h2d(recv[i].data_ptr() + o, hs[j].data_ptr() + o, m, after=t))
        for t in last:
            cp.wait(t)
        cp.acquire(stream)
        unpack(s)

    forms = {"runtime": runtime, "probe": probe}
    for c in (2, 4, 8):
        forms[f"probe_chunks_{c}"] = (lambda c=c: probe(c))
    res = {}
    for name, fn in forms.items():
        for _ in range(3):
            fn()
        res[name] = timed(fn, k) / k
    best = min(res, key=res.get)
    return {"GBps_algorithmic": round(step_bytes / res[best] / 1e9, 2),
            "ms_per_step": round(res[best] * 1e3, 4), "form": best,
            "forms_ms": {n: round(t * 1e3, 4) for n, t in res.items()},
            "pcie_bytes_per_step": 2 * n_halo * 8, "copy_engines": cp.info(),
            "note": "pack, D2H of the whole message into pinned memory, H2D back, unpack; "
                    "algorithmic bytes 4*n*8 per step"}


def launch_durations(torch, dev, stream, _ghx, fns, reps=41):
    """Median begin-to-end duration of each kernel launched by `fns` (one step = fns in order,
    each ONE kernel launch) over `reps` eager steps on `stream`, from the start/stop events
    libghx records around each kernel (ghx_launch_timing). (0, ...) if a step launched a
    different number of kernels."""
    import ctypes
    s = stream.cuda_stream
    for _ in range(3):
        for f in fns:
            f(s)
    torch.cuda.synchronize(dev)
    n = reps * len(fns)
    ms = (ctypes.c_float * n)()
    got = ctypes.c_int32()
    _ghx.call("ghx_launch_timing", 1)
    try:
        for _ in range(reps):
            for f in fns:
                f(s)
        _ghx.call("ghx_launch_timing_read", ms, n, ctypes.byref(got))
    finally:
        _ghx.call("ghx_launch_timing", 0)
    if got.value != n:
        return (0.0,) * len(fns)
    per = [sorted(ms[i::len(fns)]) for i in range(len(fns))]
    return tuple(p[len(p) // 2] * 1e-3 for p in per)


def cold_launch_durations(torch, dev, stream, _ghx, fns, flush, reps=15):
    """Like launch_durations, each step preceded by flush(s) (a torch kernel, not timed): the
    kernels' own start/stop events right after a cache flush, medians. Unlike cold_duration (a
    graph difference), this excludes the write-back of the lines a launch leaves dirty, which
    the NEXT flush pays."""
    import ctypes
    s = stream.cuda_stream
    flush(s)
    for f in fns:
        f(s)
    torch.cuda.synchronize(dev)
    n = reps * len(fns)
    ms = (ctypes.c_float * n)()
    got = ctypes.c_int32()
    _ghx.call("ghx_launch_timing", 1)
    try:
        for _ in range(reps):
            flush(s)
            for f in fns:
                f(s)
        _ghx.call("ghx_launch_timing_read", ms, n, ctypes.byref(got))
    finally:
        _ghx.call("ghx_launch_timing", 0)
    if got.value != n:
        return (0.0,) * len(fns)
    per = [sorted(ms[i::len(fns)]) for i in range(len(fns))]
    return tuple(p[len(p) // 2] * 1e-3 for p in per)


def kernel_durations(torch, dev, stream, fns, M=10, rounds=31):
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
    # per-round differences (the graphs of one round run back to back: slow drifts cancel),
    # then the median over rounds
    out = []
    for i in range(len(fns)):
        d = sorted(times[i + 1][r] - times[i][r] for r in range(rounds))
        out.append(d[len(d) // 2])
    return tuple(out)


def bench_unstructured(v, torch, dist, dev, args, cells=None):
    """BASELINE config 5 between the real ranks at its size: every rank's domain from
    tools/config5_gen.cpp (10M cells, gids rank*10^7 + i, 5 % halo from the other ranks,
    mt19937_64 seed 20260715, permuted storage), the product make_pattern<unstructured> over the
    context (reduced halos, timed as setup_s, max over ranks), levels 1, fp64, value gid*100.
    One CommunicationObject.exchange per step over the context's transport (RCCL; gloo + host
    staging in a rehearsal); `verified`: after the timed region, outer cells reset to -1, one
    more exchange, every cell of every rank checked. Bytes per rank and step: 2 * (sent +
    received values) * 8."""
    import numpy as np
    from ghex_amd import unstructured as U
    from tools import config5 as C5
    rank, world, ctx, K = v["rank"], v["world"], v["ctx"], v["K"]
    cells = C5.CELLS if cells is None else cells
    gids, outer = C5.generate(rank, world, cells)
    red = v["all_reduce_host"]
    red(0.0, dist.ReduceOp.SUM)  # start the setup clock together
    t0 = time.perf_counter()
    dd = U.DomainDescriptor(rank, gids, outer)
    pc = U.make_pattern(ctx, U.HaloGenerator(), [dd])
    t_setup = red(time.perf_counter() - t0, dist.ReduceOp.MAX)
    n_send = sum(len(l) for *_, l in pc.lid_arrays(0, 0))
    want = torch.from_numpy(gids.astype(np.float64) * 100.0).to(dev)
    field = want.clone()
    out_t = torch.from_numpy(outer).to(dev)
    field[out_t] = -1.0
    fd = U.make_field_descriptor(dd, field)
    co = U.make_communication_object(ctx, staging="host" if args.rehearse else None)
    bis = [pc(fd)]

    def count_bad():
        torch.cuda.synchronize(dev)
        return int(red(float((field != want).sum().item()), dist.ReduceOp.SUM))
    co.exchange(bis).wait()
    bad_first = count_bad()
    ke = min(K, 50)
    for _ in range(3):
        co.exchange(bis).wait()
    T = v["timed"](lambda: co.exchange(bis).wait(), ke)
    field[out_t] = -1.0
    co.exchange(bis).wait()
    bad = count_bad()
    nbytes = 2 * (n_send + outer.size) * 8
    out = {"cells_per_rank": cells, "halo_cells_per_rank": int(outer.size),
           "send_cells_rank0": n_send, "peers": len(pc.lid_arrays(0, 0)),
           "setup_s": round(t_setup, 3),
           "setup_what": "DomainDescriptor + make_pattern<unstructured> (reduced halos), max "
                         "over ranks",
           "ms_per_exchange": round(T / ke * 1e3, 4),
           "GBps_per_rank_algorithmic": round(nbytes * ke / T / 1e9, 2),
           "transport": "gloo + host staging (rehearsal)" if args.rehearse else "RCCL",
           "verified": bad == 0 and bad_first == 0,
           "verified_what": "first exchange, and one exchange after the timed region on outer "
                            "cells reset to -1: every cell of every rank"}
    del co, bis, fd, field, want
    torch.cuda.empty_cache()
    return out


def bench_halo(h, v, torch, dist, dev, stream, args, x_alloc=None):
    """The headline's step (pack launch + unpack launch, hipGraphs instantiated beforehand) for
    halo width h on the same decomposition, after a verified full exchange; one dict. x_alloc:
    allocate the field's x rows this many cells wide (the logical field is its first N+2h)."""
    N, world, rank, R, _ghx, L = v["N"], v["world"], v["rank"], v["R"], v["_ghx"], v["L"]
    parts = DECOMP[world]
    G = [parts[d] * N for d in range(3)]
    c = (rank % parts[0], (rank // parts[0]) % parts[1], rank // (parts[0] * parts[1]))
    first = tuple(c[d] * N for d in range(3))
    last = tuple((c[d] + 1) * N - 1 for d in range(3))
    E = N + 2 * h
    dd = R.DomainDescriptor(rank, first, last)
    pc = R.make_pattern(v["ctx"], R.HaloGenerator((0, 0, 0), tuple(g - 1 for g in G), (h,) * 6,
                                                  (True,) * 3), [dd])
    alloc = torch.full((E, E, x_alloc or E), -1.0, dtype=torch.float64, device=dev)
    base = alloc[:, :, :E]
    ar = [torch.arange(N, device=dev, dtype=torch.float64) + first[d] for d in range(3)]
    base[h:h + N, h:h + N, h:h + N] = (
        ar[0].view(1, 1, N) + G[0] * (ar[1].view(1, N, 1) + G[1] * ar[2].view(N, 1, 1)))
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (h,) * 3, (E,) * 3)
    co = R.make_communication_object(v["ctx"], staging="host" if args.rehearse else None)
    bis = [pc(fd)]
    interior = base[h:h + N, h:h + N, h:h + N].clone()
    w = [((torch.arange(E, device=dev) - h + first[d]) % G[d]).to(torch.float64) for d in range(3)]

    def count_bad():
        bad = int((base != w[0].view(1, 1, E) + G[0] * (w[1].view(1, E, 1) + G[1] *
                                                         w[2].view(E, 1, 1))).sum().item())
        if world > 1:
            t = torch.tensor([float(bad)], dtype=torch.float64,
                             device="cpu" if args.rehearse else dev)
            dist.all_reduce(t)
            bad = int(t.item())
        return bad

    def clear():
        base.fill_(-1.0)
        base[h:h + N, h:h + N, h:h + N] = interior

    co.exchange(bis).wait()
    bad_fused = count_bad()  # the first exchange (N=1: the fused k_self launch)
    plan = co.plan(bis)
    send, recv = co.buffers(plan, dev)
    fptr = _ghx.ptr_array([fd.data_ptr()])
    sptr = _ghx.ptr_array([x.data_ptr() for x in send])
    rptr = _ghx.ptr_array([x.data_ptr() for x in recv])

    def pack(s):
        _ghx.check(L.ghx_exchange_pack(plan.h, fptr, 1, sptr, len(send), s), "pack")

    def unpack(s):
        _ghx.check(L.ghx_exchange_unpack(plan.h, fptr, 1, rptr, len(recv), s), "unpack")

    def step():
        s = torch.cuda.current_stream(dev).cuda_stream
        pack(s)
        unpack(s)
    K = min(v["K"], 100)
    runner = Runner(torch, dev, stream, step, args.steps_per_graph or K, eager=args.no_graph)
    runner.prepare(K)
    runner.run(K)
    # the median of 5 timed regions of K steps each (one region of 20 steps is ~0.5 ms of host
    # wall time, where one scheduling hiccup of the host moved the figure by 25 % between boxes)
    Ts = sorted(v["timed"](lambda: runner.run(K), 1) for _ in range(5))
    T = Ts[len(Ts) // 2]
    me = rank
    t_sends = [(x["rank"], x["tag"], send[i][:x["size"]]) for i, x in enumerate(plan.send)
               if x["rank"] != me]
    t_recvs = [(x["rank"], x["tag"], recv[i][:x["size"]]) for i, x in enumerate(plan.recv)
               if x["rank"] != me]

    def deliver():
        from ghex_amd.communication_object import route
        if args.rehearse:
            co._exchange_host_staged(plan, t_sends, t_recvs, stream)
        else:
            for wk in route(v["ctx"], t_sends, t_recvs):
                wk.wait()
    # `verified`: the timed graph itself (k_copy pack + unpack), replayed on reset halos/buffers
    bad = verify_replay(torch, dev, lambda: runner.run(K), clear, count_bad, send, recv,
                        deliver if t_recvs else None)
    t_p, t_u = kernel_durations(torch, dev, stream, [pack, unpack])
    k_p, k_u = launch_durations(torch, dev, stream, _ghx, [pack, unpack])
    n = E ** 3 - N ** 3
    out = {"value": round(world * 4 * n * 8 * K / T / 1e9, 2), "unit": "GB/s",
           "ms_per_step": round(T / K * 1e3, 5), "steps": K, "timed_regions": len(Ts),
           "ms_per_step_range": [round(Ts[0] / K * 1e3, 5), round(Ts[-1] / K * 1e3, 5)],
           "pack_us": round(t_p * 1e6, 2),
           "unpack_us": round(t_u * 1e6, 2), "pack_kernel_us": round(k_p * 1e6, 2),
           "unpack_kernel_us": round(k_u * 1e6, 2), "bytes_per_step_per_gpu": 4 * n * 8,
           "verified": bad == 0, "verified_fused": bad_fused == 0}
    if x_alloc:
        out["row_pitch_bytes"] = 8 * x_alloc
    del runner, co, base, alloc, fd, bis, send, recv, interior, t_sends, t_recvs
    torch.cuda.empty_cache()
    if world == 1 and not x_alloc:
        out["read_floor"] = pack_read_floor(N, h, out)
    return out


def chain_duration(torch, dev, stream, fn, M=20, rounds=7):
    """Per-launch duration of fn from a graph of M back-to-back launches (median of rounds)."""
    side = torch.cuda.Stream(dev)
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        fn(side.cuda_stream)
    stream.wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(M):
            fn(s)
    g.replay()
    torch.cuda.synchronize(dev)
    t = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        g.replay()
        e1.record(stream)
        e1.synchronize()
        t.append(e0.elapsed_time(e1) * 1e-3 / M)
    return sorted(t)[len(t) // 2]


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


def _graph_of(torch, dev, fn, per=10):
    """A hipGraph of `per` back-to-back calls of fn (one eager call first, on a side stream)."""
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
    return g


def _time_graph(torch, dev, fn, k=50, per=10, keep=None):
    """Seconds per call of fn, from replays of a graph of `per` calls (k calls in all); with
    keep = a dict, the graph is returned in keep["graph"] (to replay the timed launches again
    for verification)."""
    g = _graph_of(torch, dev, fn, per)
    g.replay()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(k // per):
        g.replay()
    torch.cuda.synchronize(dev)
    if keep is not None:
        keep["graph"] = g
    return (time.perf_counter() - t0) / (k // per * per)


CONFIG4_TYPES = ("f64", "f32", "f64", "f32", "f64")


def bench_config4(torch, dev, ghex_amd, R, cpu_seconds=None):
    """BASELINE config 4 on one GPU: 5 fields 256^3 [f64,f32,f64,f32,f64], H=3, one exchange of
    all five (one periodic domain: all self messages). Timed: the per-rank form every rank runs
    at N>1, one fused pack launch + one fused unpack launch over all five fields (hipGraph of
    10); `verified`: that timed graph replayed once on halos reset to -1 and buffers set to 0xFF,
    every cell of every field checked. `verified_fused`: the first co.exchange() (the fused
    k_self launch). cpu_baseline: the oracle's single-thread serializer on the same five fields
    (cpu_seconds None: skipped)."""
    from ghex_amd import _ghx
    N, H = 256, 3
    E = N + 2 * H
    types = [torch.float64 if t == "f64" else torch.float32 for t in CONFIG4_TYPES]
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    fields, bis, interiors = [], [], []
    ar = torch.arange(N, device=dev, dtype=torch.float64)
    val = (ar.view(1, 1, N) + N * (ar.view(1, N, 1) + N * ar.view(N, 1, 1)))
    for k, T in enumerate(types):
        f = torch.full((E, E, E), -1, dtype=T, device=dev)
        f[H:H + N, H:H + N, H:H + N] = ((val + k) % (1 << 23)).to(T)
        fields.append(f)
        interiors.append(f[H:H + N, H:H + N, H:H + N].clone())
        bis.append(pc(R.make_field_descriptor(dd, f.permute(2, 1, 0), (H,) * 3, (E,) * 3)))
    del val
    idx = (torch.arange(E, device=dev) - H) % N
    wv = (idx.view(1, 1, E) + N * (idx.view(1, E, 1) + N * idx.view(E, 1, 1))).to(torch.float64)

    def all_ok():
        return all(bool((f == ((wv + k) % (1 << 23)).to(f.dtype)).all())
                   for k, f in enumerate(fields))

    co = R.make_communication_object(ctx)
    co.exchange(bis).wait()
    ok_fused = all_ok()
    plan = co.plan(bis)
    send, recv = co.buffers(plan, dev)
    fptr = _ghx.ptr_array([f.data_ptr() for f in fields])
    sptr = _ghx.ptr_array([t.data_ptr() for t in send])
    L = _ghx.lib()
    fusedp = co.all_self(plan)

    def fused(s):
        _ghx.check(L.ghx_exchange_self(plan.h, fptr, 5, sptr, len(send), s), "exchange_self")

    def two(s):  # the per-rank form at N>1: pack launch + unpack launch (self: recv IS send)
        _ghx.check(L.ghx_exchange_pack(plan.h, fptr, 5, sptr, len(send), s), "pack")
        _ghx.check(L.ghx_exchange_unpack(plan.h, fptr, 5, sptr, len(send), s), "unpack")
    t = _time_graph(torch, dev, fused) if fusedp else None
    keep = {}
    t2 = _time_graph(torch, dev, two, keep=keep)
    # verify the timed two-launch graph itself
    for f, inner in zip(fields, interiors):
        f.fill_(-1)
        f[H:H + N, H:H + N, H:H + N] = inner
    for b in send:
        b.fill_(0xFF)
    torch.cuda.synchronize(dev)
    keep["graph"].replay()
    torch.cuda.synchronize(dev)
    ok = all_ok()
    del keep

    def pk(s):
        _ghx.check(L.ghx_exchange_pack(plan.h, fptr, 5, sptr, len(send), s), "pack")

    def up(s):
        _ghx.check(L.ghx_exchange_unpack(plan.h, fptr, 5, sptr, len(send), s), "unpack")
    kp, ku = launch_durations(torch, dev, torch.cuda.current_stream(dev), _ghx, [pk, up])
    n = E ** 3 - N ** 3
    nbytes = 4 * n * (3 * 8 + 2 * 4)
    out = {"GBps": round(nbytes / t2 / 1e9, 1), "frac": round(nbytes / t2 / 1e9 / HBM_PEAK_GBS, 4),
           "us_per_exchange": round(t2 * 1e6, 2),
           "bytes_per_exchange": nbytes, "form": "pack launch + unpack launch",
           "verified": ok,
           "verified_what": "the timed hipGraph (10 x (pack + unpack) of all 5 fields) replayed "
                            "once on halos reset to -1 and buffers set to 0xFF; every cell of "
                            "every field checked",
           "verified_fused": ok_fused,
           "verified_fused_what": "the first co.exchange() (the fused k_self launch)",
           "fused_self": {"us_per_exchange": round(t * 1e6, 2),
                          "bytes_moved": 3 * n * (3 * 8 + 2 * 4)} if fusedp else None,
           "floor": multi_floor(N, H, [8 if t == "f64" else 4 for t in CONFIG4_TYPES], kp, ku)}
    if cpu_seconds:
        gpu_buf = send[0][:plan.send[0]["size"]].cpu().numpy()
        out["cpu_baseline"] = cpu_baseline_config4(cpu_seconds, gpu_buf)
    del co, bis, fields, interiors, send, recv, wv
    torch.cuda.empty_cache()
    return out


def config5_patterns(world=8, cells=None):
    """BASELINE config 5's domains for `world` ranks (tools/config5_gen.cpp: gids rank*10^7 + i,
    5 % halo from the other ranks, mt19937_64 seed 20260715, permuted storage) and every rank's
    product make_pattern<unstructured>, the ranks emulated as threads of this process
    (ghex_amd.context.LoopbackWorld: each passes only its own domain; reduced halos travel).
    Returns ([(gids, outer, send lid arrays, recv lid arrays)] per rank, setup seconds)."""
    from ghex_amd import unstructured as U
    from ghex_amd.context import LoopbackWorld
    from tools import config5 as C5
    cells = C5.CELLS if cells is None else cells

    def rank_fn(ctx):
        r = ctx.rank()
        gids, outer = C5.generate(r, world, cells)
        t0 = time.perf_counter()
        dd = U.DomainDescriptor(r, gids, outer)
        pc = U.make_pattern(ctx, U.HaloGenerator(), [dd])
        t = time.perf_counter() - t0
        return gids, outer, pc.lid_arrays(0, 0), pc.lid_arrays(0, 1), t

    t0 = time.perf_counter()
    res = LoopbackWorld(world).run(rank_fn)
    return [r[:4] for r in res], time.perf_counter() - t0, max(r[4] for r in res)


def bench_config5(torch, dev, _ghx, levels, pats, cpu_seconds=None):
    """BASELINE config 5 on one GPU as rank 0 of 8: rank 0's send and receive lid lists from
    the product pattern (config5_patterns), levels_first fp64, value(gid, level) = gid*100 +
    level. Timed: one fused gather launch over the 7 send lists + one fused scatter launch over
    the 7 receive lists (hipGraph of 10). `verified`: that timed graph replayed once on send
    buffers set to 0xFF, outer cells reset to -1 and receive buffers holding what each peer's
    own send list packs (its gids' values): every send-buffer value and every cell checked.
    cpu_baseline: the oracle's data_descriptor<cpu> get/set (cpu_seconds None: skipped)."""
    import ctypes
    import numpy as np
    gids, outer, sends, recvs = pats[0]
    n = gids.size
    host = (gids.astype(np.float64)[:, None] * 100.0 +
            np.arange(levels, dtype=np.float64)[None, :])
    want = torch.from_numpy(host).to(dev)  # (n, levels): levels fastest
    vals = want.clone()
    out_t = torch.from_numpy(outer).to(dev)
    # what each peer packs for rank 0 (its send list with the same tag), checked to be the gids
    # of rank 0's receive list: the two ends of every message agree
    peer_bytes = []
    for rid, rr, tag, lids in recvs:
        pg, _, psend, _ = pats[rr]
        plids = next(l for (i, q, tg, l) in psend if q == 0 and tg == tag)
        if not np.array_equal(pg[plids], gids[lids]):
            raise RuntimeError(f"config5 pattern: rank {rr}'s send list to 0 (tag {tag}) does "
                               "not carry rank 0's receive gids")
        peer_bytes.append(np.ascontiguousarray(host[lids]).view(np.uint8).reshape(-1))

    def plan(lists, direction):
        ents, keep = [], []
        for k, (_, _, _, l) in enumerate(lists):
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

    hp, hu = plan(sends, 0), plan(recvs, 1)
    sbufs = [torch.empty(len(l) * levels * 8, dtype=torch.uint8, device=dev) for *_, l in sends]
    rbufs = [torch.from_numpy(b).to(dev) for b in peer_bytes]
    fp = _ghx.ptr_array([vals.data_ptr()])
    sp = _ghx.ptr_array([b.data_ptr() for b in sbufs])
    rp = _ghx.ptr_array([b.data_ptr() for b in rbufs])
    L = _ghx.lib()

    def step(s):
        _ghx.check(L.ghx_uplan_execute(hp, fp, 1, sp, len(sbufs), s), "uplan pack")
        _ghx.check(L.ghx_uplan_execute(hu, fp, 1, rp, len(rbufs), s), "uplan unpack")
    keep = {}
    t = _time_graph(torch, dev, step, keep=keep)
    # verify the timed graph
    vals[out_t] = -1.0
    for b in sbufs:
        b.fill_(0xFF)
    torch.cuda.synchronize(dev)
    keep["graph"].replay()
    torch.cuda.synchronize(dev)
    bad = int((vals != want).sum().item())
    for (_, _, _, l), b in zip(sends, sbufs):
        exp = torch.from_numpy(np.ascontiguousarray(host[l])).to(dev).view(-1)
        bad += int((b.view(torch.float64) != exp).sum().item())
    del keep
    # the two launches by their own events, beside the index-list floor probe
    def gather(st):
        _ghx.check(L.ghx_uplan_execute(hp, fp, 1, sp, len(sbufs), st), "uplan pack")

    def scatter(st):
        _ghx.check(L.ghx_uplan_execute(hu, fp, 1, rp, len(rbufs), st), "uplan unpack")
    k_g, k_s = launch_durations(torch, dev, torch.cuda.current_stream(dev), _ghx,
                                [gather, scatter])
    n_send = sum(len(l) for *_, l in sends)
    n_recv = sum(len(l) for *_, l in recvs)
    nbytes = 2 * (n_send + n_recv) * levels * 8
    res = {"GBps": round(nbytes / t / 1e9, 1), "frac": round(nbytes / t / 1e9 / HBM_PEAK_GBS, 4),
           "us_per_exchange": round(t * 1e6, 2),
           "bytes_per_exchange": nbytes, "cells": int(n - outer.size), "halo_cells": n_recv,
           "send_cells": n_send, "peers": len(sends), "levels": levels,
           "index_bytes_per_exchange": (n_send + n_recv) * 4,
           "verified": bad == 0,
           "verified_what": "the timed hipGraph (10 x (gather + scatter)) replayed once: send "
                            "buffers set to 0xFF, outer cells to -1, receive buffers holding each "
                            "peer's packed send list; every send value and every cell checked",
           "inputs": "rank 0 of 8 (tools/config5_gen.cpp), lists from the product's "
                     "make_pattern<unstructured> with the 8 ranks as threads",
           "index_floor": index_floor(int(n), levels, sends, recvs, k_g, k_s)}
    if cpu_seconds:
        res["cpu_baseline"] = cpu_baseline_config5(cpu_seconds, host, sends, recvs, peer_bytes,
                                                   [b.cpu().numpy() for b in sbufs], levels)
    L.ghx_uplan_destroy(hp)
    L.ghx_uplan_destroy(hu)
    del vals, want, sbufs, rbufs
    torch.cuda.empty_cache()
    return res


def _cpu_info():
    """CPU model (/proc/cpuinfo), nproc, and the cores this process may run on."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        share = sorted(os.sched_getaffinity(0))
    except AttributeError:
        share = list(range(os.cpu_count() or 1))
    return model, os.cpu_count(), share


def _pin(core):
    """Pin the CALLING thread to one core (Linux: sched_setaffinity with pid 0 applies to the
    calling thread), the in-process form of BASELINE.md's `taskset -c <core>`."""
    try:
        os.sched_setaffinity(0, {core})
        return True
    except (AttributeError, OSError):
        return False


def _median_of_25(times):
    """25 iterations, the first 5 dropped, the median of the other 20."""
    t = sorted(times[5:25])
    return t[len(t) // 2] if t else None


def _cpu_quota():
    """Cores granted by the cgroup's CPU quota (cgroup v2 cpu.max, or v1 cfs quota); None when
    unlimited or unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // per)
    except (OSError, ValueError):
        return None


def _mem_available():
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    return None


# host memory the CPU-baseline ranks may hold together: the GPU box caps one command at about
# 270 GiB of host RAM (the bench process and torch hold the rest)
CPU_RANKS_MEM_BUDGET = 128 << 30


def cpu_rank_count(share, per_rank_bytes, env=None, quota=None, avail=None):
    """How many independent single-thread ranks the CPU baseline runs, and why: one per core of
    this process's affinity set (`nproc` ranks), capped by the cgroup CPU quota,
    by the box's declared per-GPU CPU share (OMP_NUM_THREADS: the GPU box sets it to the cores a
    one-GPU job owns and asks that worker pools stay within it) and by host memory (each rank
    holds its own field). Returns (ranks, [reasons for every cap that bound])."""
    env = os.environ if env is None else env
    n = max(1, len(share))
    caps = [(n, f"affinity set {n} cores")]
    if quota:
        caps.append((quota, f"cgroup CPU quota {quota} cores"))
    try:
        omp = int(env.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    if omp > 0:
        caps.append((omp, f"OMP_NUM_THREADS={omp}: the box's CPU share for this job"))
    budget = CPU_RANKS_MEM_BUDGET
    if avail:
        budget = min(budget, avail // 2)
    mem_cap = max(1, int(budget // max(1, per_rank_bytes)))
    caps.append((mem_cap, f"host memory: {budget / 2**30:.0f} GiB budget / "
                          f"{per_rank_bytes / 2**30:.2f} GiB per rank"))
    ranks = min(c for c, _ in caps)
    return ranks, [why for c, why in caps if c == ranks]


def _serializer_loop(orc, spec, buf, send, recv, seconds):
    """pack+unpack iterations, each timed, until >= 25 iterations AND >= `seconds`."""
    times = []
    t0 = time.perf_counter()
    while True:
        a = time.perf_counter()
        orc.structured_pack(spec, buf, send)
        orc.structured_unpack(spec, buf, recv)
        b = time.perf_counter()
        times.append(b - a)
        if b - t0 >= seconds and len(times) >= 25:
            return times, b - t0


def cpu_baseline(N, Hw, seconds):
    """The oracle's single-thread C restatement of serialization<cpu>::pack_batch/unpack_batch
    (include/ghex/structured/pack_kernels.hpp:62-158) on the same workload, bounded in time,
    run in a thread pinned to one core (the first core of this process's affinity set).
    value = throughput over the whole sample; median_of_25 = BASELINE.md §4's figure."""
    import threading

    import numpy as np
    from oracle import oracle as orc
    model, nproc, share = _cpu_info()
    E = N + 2 * Hw
    dom = orc.RegularDomain(0, (0, 0, 0), (N - 1,) * 3)
    pat = orc.regular_make_pattern([[dom]], (0, 0, 0), (N - 1,) * 3, (Hw,) * 6, (1, 1, 1))[0][0]
    send = list(pat.send.values())[0][1]
    recv = list(pat.recv.values())[0][1]
    nbytes = sum(b.size() for b in send) * 8
    res = {}

    def one():
        res["pinned"] = _pin(share[0])
        a = np.zeros((E, E, E))
        a[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = np.arange(N ** 3, dtype=np.float64).reshape(N, N, N)
        spec = orc.FieldSpec(a, 8, (2, 1, 0), (Hw,) * 3, (E,) * 3)
        buf = np.zeros(nbytes, np.uint8)
        orc.structured_pack(spec, buf, send)
        orc.structured_unpack(spec, buf, recv)
        res["times"], res["dt"] = _serializer_loop(orc, spec, buf, send, recv, seconds)
    th = threading.Thread(target=one)
    th.start()
    th.join()
    times, dt = res["times"], res["dt"]
    it = len(times)
    med = _median_of_25(times)
    out = {"value": round(4 * nbytes * it / dt / 1e9, 3), "unit": "GB/s", "cores": 1,
           "kind": "port", "cpu_model": model, "nproc": nproc, "affinity_cores": len(share),
           "pinned_core": share[0] if res["pinned"] else None,
           "median_of_25_ms": round(med * 1e3, 3),
           "median_of_25_GBps": round(4 * nbytes / med / 1e9, 3),
           "sample": f"{N}^3 fp64 H={Hw} one periodic domain, pack+unpack x{it} "
                     f"({dt:.1f} s, 1 thread pinned to core {share[0]}, "
                     f"oracle/ghex_oracle.c row-memcpy restatement); value = throughput over "
                     f"the sample, median_of_25 = BASELINE.md §4 (25 iterations, first 5 "
                     f"dropped, median)"}
    out["ranks"] = cpu_baseline_ranks(N, Hw, seconds, orc, nbytes, send, recv)
    return out


def cpu_baseline_ranks(N, Hw, seconds, orc, nbytes, send, recv):
    """SURVEY §8(d) / BASELINE.md §4: the same single-threaded serializer run as independent
    ranks, one per core (cpu_rank_count: the affinity set, capped by the CPU quota, the box's
    CPU share and host memory, the binding caps named in the line), each rank its own 512^3
    domain and buffer, pinned to its own core. The C oracle releases the GIL inside its ctypes
    calls, so the ranks are threads of this process (no re-exec from a process that has touched
    the GPU). value = bytes summed over ranks / the slowest rank's time; median_of_25 = ranks x
    bytes / the slowest rank's median iteration."""
    import threading

    import numpy as np
    model, nproc, share = _cpu_info()
    E = N + 2 * Hw
    ranks, why = cpu_rank_count(share, E ** 3 * 8 + nbytes, quota=_cpu_quota(),
                                avail=_mem_available())
    res = [None] * ranks
    pinned = [False] * ranks
    barrier = threading.Barrier(ranks)

    def rank_fn(r):
        pinned[r] = _pin(share[r])
        a = np.zeros((E, E, E))
        a[Hw:Hw + N, Hw:Hw + N, Hw:Hw + N] = r
        spec = orc.FieldSpec(a, 8, (2, 1, 0), (Hw,) * 3, (E,) * 3)
        buf = np.zeros(nbytes, np.uint8)
        orc.structured_pack(spec, buf, send)
        orc.structured_unpack(spec, buf, recv)
        barrier.wait()
        res[r] = _serializer_loop(orc, spec, buf, send, recv, seconds)
        del a, buf

    th = [threading.Thread(target=rank_fn, args=(r,)) for r in range(ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    total = sum(4 * nbytes * len(tm) for tm, _ in res)
    slowest = max(dt for _, dt in res)
    its = [len(tm) for tm, _ in res]
    med = max(_median_of_25(tm) for tm, _ in res)
    return {"value": round(total / slowest / 1e9, 3), "unit": "GB/s", "cores": ranks,
            "kind": "port", "cpu_model": model, "nproc": nproc, "affinity_cores": len(share),
            "cpu_quota_cores": _cpu_quota(), "rank_cap": why,
            "pinned": all(pinned),
            "median_of_25_GBps": round(ranks * 4 * nbytes / med / 1e9, 3),
            "sample": f"{ranks} independent ranks, each a {N}^3 fp64 H={Hw} periodic domain "
                      f"pinned to its own core ({share[0]}..{share[ranks - 1]}), pack+unpack "
                      f"x{min(its)}-{max(its)} in {slowest:.1f} s, one thread each "
                      f"(oracle/ghex_oracle.c); median_of_25 = BASELINE.md §4 per rank, the "
                      f"slowest rank's median"}


def _pinned_loop(one_pass, seconds):
    """Run one_pass in a thread pinned to the first core of the affinity set until >= 25 passes
    AND >= `seconds`; returns (per-pass times, total seconds, pinned core or None)."""
    import threading
    _, _, share = _cpu_info()
    res = {}

    def body():
        res["pinned"] = _pin(share[0])
        one_pass()  # warm (page-faults the buffers)
        times = []
        t0 = time.perf_counter()
        while True:
            a = time.perf_counter()
            one_pass()
            b = time.perf_counter()
            times.append(b - a)
            if b - t0 >= seconds and len(times) >= 25:
                res["times"], res["dt"] = times, b - t0
                return
    th = threading.Thread(target=body)
    th.start()
    th.join()
    return res["times"], res["dt"], (share[0] if res["pinned"] else None)


def cpu_baseline_config4(seconds, gpu_buf):
    """Config 4's CPU path: the oracle's single-thread restatement of the reference serializer
    (serialization<cpu>::pack_batch/unpack_batch, include/ghex/structured/pack_kernels.hpp:62-158)
    packing and unpacking all five fields of the one message (communication_object::allocate's
    layout, oracle.plan_buffers), pinned to one core. `matches_gpu`: its packed message equals
    the GPU's (the timed graph's) on every field byte."""
    import numpy as np
    from oracle import oracle as orc
    model, nproc, share = _cpu_info()
    N, H = 256, 3
    E = N + 2 * H
    dom = orc.RegularDomain(0, (0, 0, 0), (N - 1,) * 3)
    pat = orc.regular_make_pattern([[dom]], (0, 0, 0), (N - 1,) * 3, (H,) * 6, (1, 1, 1))[0][0]
    val = np.arange(N ** 3, dtype=np.float64).reshape(N, N, N)
    specs = []
    for k, t in enumerate(CONFIG4_TYPES):
        dt = np.float64 if t == "f64" else np.float32
        a = np.full((E, E, E), -1, dtype=dt)
        a[H:H + N, H:H + N, H:H + N] = ((val + k) % (1 << 23)).astype(dt)
        specs.append(orc.FieldSpec(a, a.itemsize, (2, 1, 0), (H,) * 3, (E,) * 3))
    del val
    items = [(k, 0, pat, sp.elem, sp.elem, 1, 0) for k, sp in enumerate(specs)]
    (sb,) = orc.plan_buffers(items, receive=False).values()
    (rb,) = orc.plan_buffers(items, receive=True).values()
    buf = np.zeros(sb.size, np.uint8)

    def one_pass():
        for pf in sb.fields:
            orc.structured_pack(specs[pf.field_index], buf, pf.boxes, pf.offset)
        for pf in rb.fields:
            orc.structured_unpack(specs[pf.field_index], buf, pf.boxes, pf.offset)
    one_pass()
    n = E ** 3 - N ** 3
    same = buf.size == gpu_buf.size and all(
        np.array_equal(buf[pf.offset:pf.offset + n * specs[pf.field_index].elem],
                       gpu_buf[pf.offset:pf.offset + n * specs[pf.field_index].elem])
        for pf in sb.fields)
    times, dt, core = _pinned_loop(one_pass, seconds)
    nbytes = 4 * n * (3 * 8 + 2 * 4)
    med = _median_of_25(times)
    return {"value": round(nbytes * len(times) / dt / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "port", "cpu_model": model, "nproc": nproc, "pinned_core": core,
            "median_of_25_GBps": round(nbytes / med / 1e9, 3), "matches_gpu": bool(same),
            "sample": f"the whole config-4 exchange (5 fields 256^3, H=3, one message) pack+"
                      f"unpack x{len(times)} in {dt:.1f} s, 1 thread (oracle/ghex_oracle.c "
                      f"row-memcpy restatement)"}


def cpu_baseline_config5(seconds, host, sends, recvs, peer_bytes, gpu_sbufs, levels):
    """Config 5's CPU path: the oracle's restatement of data_descriptor<cpu>::get/set
    (include/ghex/unstructured/user_concepts.hpp:385-440: one memcpy per value) over rank 0's
    7 send and 7 receive lists, pinned to one core. `matches_gpu`: every packed send buffer
    equals the GPU's (the timed graph's), bit for bit."""
    import numpy as np
    from oracle import oracle as orc
    model, nproc, share = _cpu_info()
    vals = np.ascontiguousarray(host).reshape(-1).copy()
    sb = [np.zeros(len(l) * levels * 8, np.uint8) for *_, l in sends]
    sl = [np.ascontiguousarray(l, dtype=np.int64) for *_, l in sends]
    rl = [np.ascontiguousarray(l, dtype=np.int64) for *_, l in recvs]

    def one_pass():
        for l, b in zip(sl, sb):
            orc.unstructured_get(vals, b, 8, l, levels, True, levels, 1)
        for l, b in zip(rl, peer_bytes):
            orc.unstructured_set(vals, b, 8, l, levels, True, levels, 1)
    one_pass()
    same = all(np.array_equal(a, b) for a, b in zip(sb, gpu_sbufs)) and \
        np.array_equal(vals, np.ascontiguousarray(host).reshape(-1))
    times, dt, core = _pinned_loop(one_pass, seconds)
    n_send, n_recv = sum(map(len, sl)), sum(map(len, rl))
    nbytes = 2 * (n_send + n_recv) * levels * 8
    med = _median_of_25(times)
    return {"value": round(nbytes * len(times) / dt / 1e9, 3), "unit": "GB/s", "cores": 1,
            "kind": "port", "cpu_model": model, "nproc": nproc, "pinned_core": core,
            "median_of_25_GBps": round(nbytes / med / 1e9, 3), "matches_gpu": bool(same),
            "sample": f"rank 0's 7 gathers + 7 scatters (levels={levels}) x{len(times)} in "
                      f"{dt:.1f} s, 1 thread (oracle/ghex_oracle.c get/set restatement)"}


if __name__ == "__main__":
    try:
        main()
    except Exception as e:  # a line with value null and the error, then the failure itself
        if _LINE["guard"] is not None and not _LINE["printed"]:
            _LINE["guard"].fail("main", e)
        raise
