"""Fixed cost of the zero-copy exchanges' device epochs, isolated (developer measurement).

Two "ranks" in one process share one flag block (two attachments of the same shm segment) and
run on two streams of the one GPU, each exchange being ONLY the epoch launches — open, close —
with no data launch in between, so the time per exchange is the protocol's own: the launches,
the handshake through the host-memory flags, the per-XCD release / acquire fences.

    python tools/epoch_bench.py [K] [one]   -> one JSON line ("one": the one-launch close)

Reported: us_per_exchange (K back-to-back exchanges per stream, host wall time / K, both streams
running concurrently), us_per_exchange_graph (the same K exchanges captured into one hipGraph per
stream and replayed), the XCD count and fence grid, and the epoch counters after the run (both
must equal the number of exchanges). DESIGN.md §5 quotes it."""
import ctypes
import json
import os
import secrets
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    one = len(sys.argv) > 2 and sys.argv[2] == "one"  # the one-launch close (phase 2)
    phases = (2,) if one else (0, 1)
    import torch
    from ghex_amd import _ghx
    _ghx.lib()
    name = f"/ghx_epb_{os.getpid()}_{secrets.token_hex(4)}".encode()
    eps = []
    for r in range(2):
        h = ctypes.c_void_p()
        _ghx.call("ghx_epochs_create", name, 1 if r == 0 else 0, 2, r, 10.0, ctypes.byref(h))
        eps.append(h)
    _ghx.call("ghx_epochs_unlink", name)
    for r in range(2):
        peer = _ghx.i32_array([1 - r])
        _ghx.call("ghx_epochs_peers", eps[r], peer, 1, peer, 1)
    nx, fg = ctypes.c_int32(), ctypes.c_int32()
    _ghx.call("ghx_epochs_info", eps[0], ctypes.byref(nx), ctypes.byref(fg))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def exchanges(k):
        for _ in range(k):
            for r in range(2):
                s = streams[r].cuda_stream
                for ph in phases:
                    _ghx.call("ghx_epochs_enqueue", eps[r], ph, s)

    exchanges(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    exchanges(K)
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / K
    # the same sequence captured: one graph of G exchanges per stream, replayed concurrently
    G = 100
    graphs = []
    for r in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(streams[r]):
            with torch.cuda.graph(g, stream=streams[r]):
                s = torch.cuda.current_stream().cuda_stream
                for _ in range(G):
                    for ph in phases:
                        _ghx.call("ghx_epochs_enqueue", eps[r], ph, s)
        graphs.append(g)
    reps = max(1, K // G)
    for r in range(2):  # the first replay of each (both needed: each waits for the other)
        with torch.cuda.stream(streams[r]):
            graphs[r].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for r in range(2):
            with torch.cuda.stream(streams[r]):
                graphs[r].replay()
    torch.cuda.synchronize()
    t_graph = (time.perf_counter() - t0) / (reps * G)
    st = []
    for r in range(2):
        err, ep = ctypes.c_int32(), ctypes.c_uint64()
        _ghx.call("ghx_epochs_status", eps[r], ctypes.byref(err), ctypes.byref(ep))
        st.append({"error": err.value, "epoch": ep.value})
    n_ex = 20 + K + G * (reps + 1)
    out = {"tool": "tools/epoch_bench.py", "mode": "one-launch close (phase 2)" if one else
           "open + close (phases 0, 1)", "exchanges": K, "launches_per_exchange": len(phases),
           "us_per_exchange": round(t_eager * 1e6, 2),
           "us_per_exchange_graph": round(t_graph * 1e6, 2),
           "n_xcc": nx.value, "close_grid": fg.value, "status": st,
           "epochs_ok": all(x["error"] == 0 and x["epoch"] == n_ex for x in st),
           "note": "two ranks (one flag block, two streams, one GPU), each exchange = the epoch "
                   "launches with no data launch: the protocol's fixed cost incl. the cross-rank "
                   "handshake"}
    for h in eps:
        _ghx.call("ghx_epochs_destroy", h)
    print(json.dumps(out), flush=True)
    return 0 if out["epochs_ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
