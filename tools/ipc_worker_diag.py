"""Developer diagnosis (not product): why ghx_ipc_export (hipIpcGetMemHandle, dmabuf IPC) fails
for 2-3 of 4 worker processes at 256^3 in tests/test_gpu_multiproc.py while bench.py's bulk
children at the same size export fine. One rank of a gloo group: the worker's field set-up, then
export attempts of the field's allocation, each logged with its time; MODE selects what happens
before the first attempt:
  plain    as the worker (numpy field, H2D copy, export)
  barrier  a gloo barrier first (every rank has finished its H2D copy)
  sync     torch.cuda.synchronize() first
  early    the device allocation exported BEFORE the numpy work and the copy
  pattern  as plain, with the worker's make_pattern (libghx) before the field
  bulk     as the worker: make_pattern, then BulkCommunicationObject.init() exports the field
Then up to 20 more attempts 50 ms apart. Usage: RANK=.. WORLD_SIZE=.. MASTER_*=..
python tools/ipc_worker_diag.py N MODE"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    N, mode = int(sys.argv[1]), sys.argv[2]
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    import ghex_amd
    from ghex_amd import _ghx
    from tests import helpers as H
    ghex_amd.native_library()
    L = _ghx.lib()
    Hw = 2
    ranks, gf, gl = H.cube_domains(N, (2, 2, 1) if world == 4 else (world, 1, 1))
    dom = ranks[rank][0]
    E = N + 2 * Hw
    log = []

    def attempt(t, tag):
        h = (ctypes.c_ubyte * 64)()
        off = ctypes.c_uint64()
        rc = L.ghx_ipc_export(ctypes.c_void_p(t.data_ptr()), h, ctypes.byref(off))
        log.append({"tag": tag, "t": round(time.perf_counter() - t0, 3), "rc": rc,
                    "err": L.ghx_last_error().decode()[:120] if rc else ""})
        return rc == 0

    t0 = time.perf_counter()
    pc = None
    if mode in ("pattern", "bulk"):
        from ghex_amd.structured import regular as R
        ctx = ghex_amd.make_context()
        dd = R.DomainDescriptor(dom.id, dom.first, dom.last)
        pc = R.make_pattern(ctx, R.HaloGenerator(gf, gl, (Hw,) * 6, (True,) * 3), [dd])
    early = None
    if mode == "early":
        early = torch.empty((E, E, E), dtype=torch.float64, device="cuda")
        attempt(early, "early_alloc")
    a, _ = H.linear_index_field(dom, N, Hw, gl)
    expect = H.expected_linear_halo(a, dom, N, Hw, gl)
    if early is not None:
        early.copy_(torch.from_numpy(a))
        base = early
    else:
        base = torch.from_numpy(a).cuda()
    if mode == "barrier":
        dist.barrier()
    if mode == "sync":
        torch.cuda.synchronize()
    if mode == "bulk":
        fd = R.make_field_descriptor(dd, base.permute(2, 1, 0), (Hw,) * 3, (E,) * 3)
        co = ghex_amd.make_bulk_communication_object(ctx, timeout=60)
        co.add_field(pc(fd))
        try:
            co.init()
            log.append({"tag": "bulk_init", "t": round(time.perf_counter() - t0, 3), "rc": 0})
        except Exception as e:
            log.append({"tag": "bulk_init", "t": round(time.perf_counter() - t0, 3), "rc": -1,
                        "err": str(e)[:160]})
    ok = attempt(base, "first")
    k = 0
    while not ok and k < 20:
        time.sleep(0.05)
        k += 1
        ok = attempt(base, f"retry{k}")
    dist.barrier()
    print(json.dumps({"rank": rank, "world": world, "N": N, "mode": mode, "ok": ok,
                      "attempts": log, "expect_cells": int(expect.size)}), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
