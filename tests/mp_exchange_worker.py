"""Worker for tests/test_gpu_multiproc.py: one rank of a real multi-process exchange, every rank
on cuda:0 of the test box (RCCL needs one GPU per rank, so the transport here is gloo with
host-staged buffers — the product's staging="host" mode). Launched with RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in the environment; exits 0 when every cell of the rank's field
(owned + halo) holds the wrapped global linear index after the exchange.

With mode "bulk" the exchange is the zero-copy BulkCommunicationObject instead: every rank puts
its send regions straight into the peers' fields through IPC mappings (same GPU here, peer
GPUs over xGMI on a multi-GPU node). Modes "direct*": the CommunicationObject's direct form
(the pack writes into the receivers' buffers through IPC mappings; device epochs). Mode "pipe" is the pipelined host-staged exchange (one
stream per peer: pack, D2H, send as soon as that copy landed, H2D + unpack per arrived message).

usage: python tests/mp_exchange_worker.py <px> <py> <pz> <N> <H> [n_exchanges] [staged|stagedrt|bulk|bulkhost|bulkmixed|bulkrace|bulkgraph|sched|pipe|pipert|direct|directloop|directrace|directgraph|directnoepoch|directmany|udirect|slowdirect|slowbulk]
(udirect: <px> <py> <pz> = world split, <N> = cells per rank, <H> = levels)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_jitter(rank):
    """GHX_SOAK_JITTER=1 (tools/epoch_soak.py): before each exchange of the race / graph loops a
    rank queues 0-3 busy kernels (seeded per rank), so the ranks' streams drift apart and the
    epochs alone keep them in step. Otherwise a no-op."""
    if os.environ.get("GHX_SOAK_JITTER") != "1":
        return lambda: None
    import random
    import torch
    rng = random.Random(1000 + rank)
    scratch = torch.ones(1 << 25, device="cuda")  # 128 MiB: tens of microseconds per kernel

    def jitter():
        for _ in range(rng.randrange(4)):
            scratch.mul_(1.0)
    return jitter


def _export_probe(tag, t):
    """GHX_WORKER_EXPORT_PROBE=1: try ghx_ipc_export on `t` and print the outcome."""
    import ctypes
    import time

    from ghex_amd import _ghx
    L = _ghx.lib()
    h = (ctypes.c_ubyte * 64)()
    off = ctypes.c_uint64()
    rc = L.ghx_ipc_export(ctypes.c_void_p(t.data_ptr()), h, ctypes.byref(off))
    print(f"export_probe {tag} rc={rc} t={time.time():.3f} "
          f"{L.ghx_last_error().decode()[:100] if rc else ''}", flush=True)


_kept = []


def main():
    px, py, pz, N, Hw = (int(v) for v in sys.argv[1:6])
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    mode = sys.argv[7] if len(sys.argv) > 7 else "staged"
    import numpy as np
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == px * py * pz
    torch.cuda.set_device(0)
    import ghex_amd
    from ghex_amd.structured import regular as R
    from tests import helpers as H
    from tests.gpu_util import device_field
    ghex_amd.native_library()
    jitter = make_jitter(rank)
    if mode == "udirect":
        sys.exit(unstructured_direct(rank, world, N, Hw, reps))
    if mode in ("slowdirect", "slowbulk"):
        sys.exit(slow_peer(mode, rank, world, N, Hw, (px, py, pz)))
    ranks, gf, gl = H.cube_domains(N, (px, py, pz))
    dom = ranks[rank][0]
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(dom.id, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    bad = 0
    probe = os.environ.get("GHX_WORKER_EXPORT_PROBE") == "1"  # developer diagnosis
    if probe:
        _export_probe("start", torch.empty((N + 2 * Hw,) * 3, dtype=torch.float64, device="cuda"))
    co = None
    for layout in [(2, 1, 0), (0, 2, 1)]:
        a, _ = H.linear_index_field(dom, N, Hw, gl, layout=layout)
        if probe:
            _export_probe("after_field_numpy", torch.empty(a.shape, dtype=torch.float64,
                                                           device="cuda"))
        expect = H.expected_linear_halo(a, dom, N, Hw, gl, layout=layout)
        if probe:
            _export_probe("after_expect_numpy", torch.empty(a.shape, dtype=torch.float64,
                                                            device="cuda"))
        base, logical = device_field(a, layout)
        if os.environ.get("GHX_DIAG_SYNC") == "1":  # developer diagnosis: export after a sync
            torch.cuda.synchronize()
        part = os.environ.get("GHX_DIAG_TEARDOWN", "")  # developer diagnosis: one teardown part
        if part and layout != (2, 1, 0) and co is not None:
            from ghex_amd import _ghx as G
            import ctypes as C
            if part == "imports":
                for b in co._imports:
                    G.lib().ghx_ipc_close(C.c_void_p(b))
                co._imports = []
            elif part == "puts":
                for h, *_ in co._puts:
                    G.lib().ghx_put_destroy(h)
                co._puts = []
            elif part == "epochs" and co._ep is not None:
                G.lib().ghx_epochs_destroy(co._ep)
                co._ep = None
            elif part == "free":
                junk = torch.empty(1 << 22, dtype=torch.float64, device="cuda")
                del junk
                torch.cuda.empty_cache()
            _export_probe(f"after_{part}", base)
        prime = os.environ.get("GHX_DIAG_PRIME", "0")  # developer diagnosis: exports first
        if prime in ("1", "small"):
            _export_probe("prime_small", torch.empty(1 << 18, dtype=torch.float64, device="cuda"))
        if prime in ("1", "big"):
            _export_probe("prime_field_size", torch.empty(a.shape, dtype=torch.float64,
                                                          device="cuda"))
        if prime == "self":
            _export_probe("prime_self", base)
        if probe:
            _export_probe("field", base)
        fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
        if mode in ("bulk", "bulkhost"):
            co = ghex_amd.make_bulk_communication_object(
                ctx, epochs="host" if mode == "bulkhost" else "device", timeout=60)
            co.add_field(pc(fd))
            for _ in range(reps):
                co.exchange().wait()
        elif mode == "bulkmixed":
            # two emulated hosts (even / odd ranks): puts between ranks of one host, a host-staged
            # buffered exchange of the pattern's remote part for the others, one exchange()
            os.environ["GHX_HOSTNAME"] = f"emulated-host-{rank % 2}"
            co = ghex_amd.make_bulk_communication_object(ctx, timeout=60,
                                                         remote_options={"staging": "host"})
            co.add_field(pc(fd))
            for _ in range(reps):
                co.exchange().wait()
            assert (co._co is not None) == (world > 1)
        elif mode == "bulkrace":
            # device epochs only order the exchanges: per exchange k, on the stream and with no
            # host synchronisation, the field is rewritten (owned cells x f_k, halos -f_k), the
            # exchange runs, and the halos are compared with the expected values x f_k into a
            # device counter. A put that landed before its target opened, or a halo read before
            # every source finished, would leave cells of another epoch behind.
            co = ghex_amd.make_bulk_communication_object(ctx, timeout=60)
            co.add_field(pc(fd))
            src = torch.from_numpy(a).cuda()
            exp_d = torch.from_numpy(expect).cuda()
            nbad = torch.zeros((), dtype=torch.int64, device="cuda")
            h = None
            for k in range(4 * reps):
                f = float(k % 5 + 1)
                base.copy_(src * f)
                jitter()
                h = co.exchange()
                nbad += (base != exp_d * f).sum()
            h.wait()
            bad += int(nbad.item())
            continue
        elif mode == "bulkgraph":
            # the whole bulk exchange (epoch open, puts, epoch close) captured once into a graph
            # and replayed: the epoch counters live in memory, so every replay is a new epoch
            co = ghex_amd.make_bulk_communication_object(ctx, timeout=60)
            co.add_field(pc(fd))
            co.exchange().wait()
            src = torch.from_numpy(a).cuda()
            exp_d = torch.from_numpy(expect).cuda()
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                co.exchange()
            torch.cuda.current_stream().wait_stream(side)
            with torch.cuda.graph(g):
                co.exchange()
            nbad = torch.zeros((), dtype=torch.int64, device="cuda")
            for k in range(3 * reps):
                f = float(k % 5 + 1)
                base.copy_(src * f)
                jitter()
                g.replay()
                nbad += (base != exp_d * f).sum()
            torch.cuda.synchronize()
            co.check_epochs()
            bad += int(nbad.item())
            continue
        elif mode == "directmany":
            # 70 fields in one direct exchange: the plans split into launch groups, each with
            # its own slot map of the receive buffers' second copies; rewritten, exchanged and
            # checked on the stream with no host synchronisation
            co = R.make_communication_object(ctx, direct=True, epoch_timeout=60)
            srcs = [torch.from_numpy(a).cuda() + k for k in range(70)]
            views = [device_field(a + k, layout) for k in range(70)]
            bases = [b for b, _ in views]
            bis = [pc(R.make_field_descriptor(dd, v, (Hw,) * 3, (N + 2 * Hw,) * 3))
                   for _, v in views]
            exp_d = torch.from_numpy(expect).cuda()
            nbad = torch.zeros((), dtype=torch.int64, device="cuda")
            for k in range(2 * reps):
                f = float(k % 5 + 1)
                for b, s in zip(bases, srcs):
                    b.copy_(s * f)
                jitter()
                co.exchange(bis)
                co._valid = False
                for j, b in enumerate(bases):
                    nbad += (b != (exp_d + j) * f).sum()
            torch.cuda.synchronize()
            co.check_epochs()
            bad += int(nbad.item())
            continue
        elif mode in ("direct", "directloop", "directrace", "directgraph", "directnoepoch"):
            # the pack writes every peer message straight into the receiver's buffer (IPC),
            # device epochs order it; the receiver unpacks locally (no transport step)
            co = R.make_communication_object(ctx, direct=True, epoch_timeout=60)
            if mode == "direct":
                for _ in range(reps):
                    co.exchange([pc(fd)]).wait()
                if world > 1:
                    # the single-buffered helpers refuse a plan with epoch parity set (they would
                    # pack past the end of the local send buffers)
                    for helper in (co.pack_only, co.unpack_only, co.pack_self_only,
                                   co.unpack_peers_only):
                        try:
                            helper([pc(fd)])
                        except RuntimeError as e:
                            assert "direct exchange" in str(e), e
                        else:
                            raise AssertionError(f"{helper.__name__} ran on a direct plan")
            elif mode == "directloop":
                # back to back on the stream, one host wait at the end: the ranks' devices stay
                # in step through the epochs alone (tools/prof_direct.sh traces this)
                co.exchange([pc(fd)]).wait()
                for _ in range(reps):
                    co.exchange([pc(fd)])
                    co._valid = False
                co.exchange([pc(fd)]).wait()
            else:
                # rewrite / exchange / check on the stream with no host synchronisation (race),
                # or the exchange captured once into a graph and replayed (graph): a pack that
                # wrote into a buffer its receiver still unpacked from, or an unpack before every
                # source's writes landed, would leave values of another exchange behind
                src = torch.from_numpy(a).cuda()
                exp_d = torch.from_numpy(expect).cuda()
                co.exchange([pc(fd)]).wait()
                run = lambda: co.exchange([pc(fd)])
                if mode == "directnoepoch":
                    # negative control of the soak (tools/epoch_soak.py): the same loop with the
                    # epoch launch left out, so nothing orders the ranks' packs and unpacks; the
                    # check must see values of other exchanges
                    for d in co._direct.values():
                        d["ep_saved"], d["ep"] = d["ep"], None
                if mode == "directgraph":
                    g = torch.cuda.CUDAGraph()
                    side = torch.cuda.Stream()
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        co.exchange([pc(fd)])
                        co._valid = False
                    torch.cuda.current_stream().wait_stream(side)
                    with torch.cuda.graph(g):
                        co.exchange([pc(fd)])
                        co._valid = False
                    run = g.replay
                nbad = torch.zeros((), dtype=torch.int64, device="cuda")
                for k in range(4 * reps):
                    f = float(k % 5 + 1)
                    base.copy_(src * f)
                    jitter()
                    run()
                    co._valid = False  # the next exchange is ordered on the stream, not awaited
                    nbad += (base != exp_d * f).sum()
                torch.cuda.synchronize()
                for d in co._direct.values():
                    if "ep_saved" in d:
                        d["ep"] = d.pop("ep_saved")
                dist.barrier()
                co.check_epochs()
                bad += int(nbad.item())
                continue
        elif mode == "sched":  # schedule_exchange on a side stream, host-staged transport
            co = R.make_communication_object(ctx, staging="host")
            s = torch.cuda.Stream()
            for _ in range(reps):
                h = co.schedule_exchange(s, [pc(fd)])
                h.schedule_wait(s)
                assert co.has_scheduled_exchange()
                h.wait()
        elif mode == "pipe":  # per-peer streams: pack -> D2H -> send as landed -> H2D -> unpack
            co = R.make_communication_object(ctx, staging="host", pipelined=True)
            for _ in range(reps):
                co.exchange([pc(fd)]).wait()
        elif mode == "stagedrt":  # host staging with hipMemcpyAsync (runtime-chosen engines)
            co = R.make_communication_object(ctx, staging="host", copy_engine="runtime")
            for _ in range(reps):
                co.exchange([pc(fd)]).wait()
        elif mode == "pipert":
            co = R.make_communication_object(ctx, staging="host", pipelined=True,
                                             copy_engine="runtime")
            for _ in range(reps):
                co.exchange([pc(fd)]).wait()
        else:
            co = R.make_communication_object(ctx, staging="host")
            for _ in range(reps):
                co.exchange([pc(fd)]).wait()
        got = base.cpu().numpy()
        if os.environ.get("GHX_DIAG_KEEPCO") == "1":  # developer diagnosis: no teardown
            _kept.append((co, base))
        if os.environ.get("GHX_DIAG_BARRIER") == "1":  # developer diagnosis: ordered teardown
            torch.cuda.synchronize()
            dist.barrier()
            del co
            import gc
            gc.collect()
            dist.barrier()
            co = None
        nb = int(np.count_nonzero(got != expect))
        bad += nb
    t = torch.tensor([bad])
    dist.all_reduce(t)
    if rank == 0:
        print(f"{mode} world {world} parts {(px, py, pz)} N {N} H {Hw}: bad cells {int(t.item())}")
    dist.barrier()
    del co
    dist.destroy_process_group()
    sys.exit(0 if int(t.item()) == 0 else 1)


def slow_peer(mode, rank, world, N, Hw, parts):
    """Modes slowdirect / slowbulk (an epoch failure must reach both sides): after
    one good exchange, rank 1 arrives 5 s late at the second one while the epoch timeout is
    1.5 s.
    slowbulk (open + close): rank 0's open wait times out — its puts still write into rank 1's
      halos — so rank 0 raises the open-phase timeout and rank 1, whose own waits pass, raises
      that rank 0 failed (the FAIL mark on rank 0's done flag).
    slowdirect (one-launch close, double-buffered receive buffers): rank 0's close times out;
      its pack wrote the copy rank 1 was not reading, so rank 1's second exchange is valid and
      raises nothing; at the third exchange rank 0's done flag carries FAIL and rank 1 raises.
    Exit 0 when every rank raised (or not) as expected."""
    import time

    import torch
    import torch.distributed as dist
    import ghex_amd
    from ghex_amd.structured import regular as R
    from tests import helpers as H
    from tests.gpu_util import device_field
    ranks, gf, gl = H.cube_domains(N, parts)
    dom = ranks[rank][0]
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(dom.id, dom.first, dom.last)
    pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    base, logical = device_field(a, (2, 1, 0))
    fd = R.make_field_descriptor(dd, logical, (Hw,) * 3, (N + 2 * Hw,) * 3)
    if mode == "slowdirect":
        co = R.make_communication_object(ctx, direct=True, epoch_timeout=1.5)
        ex = lambda: co.exchange([pc(fd)])  # noqa: E731
    else:
        co = ghex_amd.make_bulk_communication_object(ctx, timeout=1.5)
        co.add_field(pc(fd))
        ex = co.exchange
    ex().wait()  # both on time
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 1:
        time.sleep(5.0)
    def attempt():
        try:
            ex().wait()
            return ""
        except RuntimeError as e:
            return str(e)
    err = attempt()
    if mode == "slowbulk":
        want = "open phase timed out" if rank == 0 else "failed an epoch wait"
        ok = want in err
    else:
        ok = ("close phase timed out" in err) if rank == 0 else err == ""
        if rank == 1 and ok:  # the late rank's halos are all valid
            exp = H.expected_linear_halo(a, dom, N, Hw, gl)
            ok = bool((base.cpu().numpy() == exp).all())
        torch.cuda.synchronize()
        dist.barrier()
        err3 = attempt()
        ok = ok and ("failed an epoch wait" in err3 if rank == 1 else err3 != "")
        err = err + " | third: " + err3
    print(f"{mode} rank {rank}: {'ok' if ok else 'WRONG'}: {err or 'no error raised'}", flush=True)
    t = torch.tensor([0 if ok else 1])
    dist.all_reduce(t)
    if rank == 0 and int(t.item()) == 0:
        print(f"{mode} world {world}: bad cells 0 (both sides raised)")
    dist.barrier()
    del co
    dist.destroy_process_group()
    return 0 if int(t.item()) == 0 else 1


def unstructured_direct(rank, world, cells, levels, reps):
    """Mode udirect: an unstructured exchange through CommunicationObject(direct=True) between
    the processes — every rank owns `cells` cells (gids rank*10^6 + i) and holds cells/4 halo
    cells drawn from the other ranks, in a random storage order, `levels` levels (levels first);
    value(gid, level) = gid*100 + level; every halo value checked after each exchange."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import ghex_amd
    from ghex_amd import unstructured as U
    rng = np.random.default_rng(4242 + rank)
    nh = cells // 4
    others = np.array([r for r in range(world) if r != rank])
    owner = others[rng.integers(0, len(others), size=4 * nh)]
    halo = np.unique(owner.astype(np.int64) * 1_000_000 + rng.integers(0, cells, size=4 * nh))
    halo = rng.permutation(halo)[:nh]
    gids = np.concatenate([rank * 1_000_000 + np.arange(cells, dtype=np.int64), halo])
    perm = rng.permutation(len(gids))
    gids = gids[perm]
    outer = np.nonzero(perm >= cells)[0]
    ctx = ghex_amd.make_context()
    dd = U.DomainDescriptor(rank, gids, outer)
    pc = U.make_pattern(ctx, U.HaloGenerator(), [dd])
    want = gids.astype(np.float64)[:, None] * 100.0 + np.arange(levels)[None, :]
    init = want.copy()
    init[outer] = -1.0
    field = torch.from_numpy(init).cuda()  # (cells, levels): levels fastest
    fd = U.make_field_descriptor(dd, field)
    co = U.make_communication_object(ctx, direct=True, epoch_timeout=60)
    bad = 0
    for _ in range(reps):
        field[torch.from_numpy(outer).cuda()] = -1.0
        co.exchange([pc(fd)]).wait()
        bad += int(np.count_nonzero(field.cpu().numpy() != want))
    t = torch.tensor([bad])
    dist.all_reduce(t)
    if rank == 0:
        print(f"udirect world {world} cells {cells} levels {levels}: bad cells {int(t.item())}")
    dist.barrier()
    del co
    dist.destroy_process_group()
    return 0 if int(t.item()) == 0 else 1


if __name__ == "__main__":
    main()
