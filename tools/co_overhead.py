"""Developer measurement (not product): where the time of one drop-in exchange goes at N=1
(512^3 fp64 H=2, CommunicationObject.exchange = the fused k_self launch).

  wait_us        co.exchange(bis).wait() back to back (what a caller's loop pays)
  queued_us      co.exchange(bis) back to back without waiting (the host keeps the queue fed:
                 device-bound if the host is faster than the kernel)
  host_call_us   host time inside one exchange() call while the device is busy
  roundtrip_us   an empty kernel launch + event synchronize (the HIP round trip floor)
  kernel_us      the k_self launch by its own events (ghx_launch_timing)
One JSON line. Run: python tools/co_overhead.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import ghex_amd  # noqa: E402
from ghex_amd import _ghx  # noqa: E402
from ghex_amd.structured import regular as R  # noqa: E402


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    N, H = 512, 2
    E = N + 2 * H
    dev = torch.device("cuda", 0)
    base = torch.zeros((E, E, E), dtype=torch.float64, device=dev)
    ctx = ghex_amd.make_context()
    dd = R.DomainDescriptor(0, (0, 0, 0), (N - 1,) * 3)
    pc = R.make_pattern(ctx, R.HaloGenerator((0, 0, 0), (N - 1,) * 3, (H,) * 6, (True,) * 3), [dd])
    fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (H,) * 3, (E,) * 3)
    co = R.make_communication_object(ctx)
    bis = [pc(fd)]
    for _ in range(50):
        co.exchange(bis).wait()
    torch.cuda.synchronize()
    K = 2000
    out = {"what": "512^3 fp64 H=2, one rank, CommunicationObject.exchange (fused k_self)"}

    reps = []
    for _ in range(5):
        t = time.perf_counter()
        for _ in range(K):
            co.exchange(bis).wait()
        reps.append((time.perf_counter() - t) / K * 1e6)
    out["wait_us"] = round(med(reps), 2)

    reps = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(K):
            co.exchange(bis)
            co._valid = False  # the next exchange without waiting (stream order keeps it correct)
        torch.cuda.synchronize()
        reps.append((time.perf_counter() - t) / K * 1e6)
    out["queued_us"] = round(med(reps), 2)

    # host time of the call itself: a long kernel keeps the device busy meanwhile
    big = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    reps = []
    for _ in range(5):
        torch.cuda.synchronize()
        for _ in range(20):
            big.mul_(1.0)  # ~ms of queued device work
        t = time.perf_counter()
        for _ in range(200):
            co.exchange(bis)
            co._valid = False
        reps.append((time.perf_counter() - t) / 200 * 1e6)
        torch.cuda.synchronize()
    out["host_call_us"] = round(med(reps), 2)
    del big

    x = torch.empty(1, device=dev)
    ev = torch.cuda.Event()
    reps = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(K):
            x.add_(1.0)
            ev.record()
            ev.synchronize()
        reps.append((time.perf_counter() - t) / K * 1e6)
    out["roundtrip_us"] = round(med(reps), 2)

    L = _ghx.lib()
    L.ghx_launch_timing(1)
    for _ in range(25):
        co.exchange(bis).wait()
    import ctypes
    buf = (ctypes.c_float * 64)()
    n = ctypes.c_int32()
    _ghx.call("ghx_launch_timing_read", buf, 64, ctypes.byref(n))  # before disabling (drops)
    L.ghx_launch_timing(0)
    ks = [buf[i] * 1e3 for i in range(n.value)][5:]
    out["kernel_us"] = round(med(ks), 2) if ks else None
    out["note"] = ("wait_us - kernel_us is what a synchronous caller pays beyond the kernel: the "
                   "launch and completion round trip (roundtrip_us for an empty kernel) plus the "
                   "host call (host_call_us), which the queued loop hides")
    print(json.dumps(out), flush=True)
    if "--profile" in sys.argv:
        # where the host call's time goes (the device kept busy, as for host_call_us)
        import cProfile
        import pstats
        big = torch.empty(1 << 28, dtype=torch.float32, device=dev)
        for _ in range(40):
            big.mul_(1.0)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(500):
            co.exchange(bis)
            co._valid = False
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
        # single primitives, timed alone
        s = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        prims = {
            "current_stream": lambda: torch.cuda.current_stream(0),
            "event_record": lambda: ev.record(s),
            "cuda_stream_attr": lambda: s.cuda_stream,
            "data_ptr": lambda: base.data_ptr(),
            "str_device": lambda: str(dev),
        }
        res = {}
        for k, f in prims.items():
            t = time.perf_counter()
            for _ in range(20000):
                f()
            res[k] = round((time.perf_counter() - t) / 20000 * 1e6, 3)
        torch.cuda.synchronize()
        print(json.dumps({"primitives_us": res}), flush=True)


if __name__ == "__main__":
    main()
