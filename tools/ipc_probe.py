"""Which device allocations ghx_ipc_export accepts (hipIpcGetMemHandle under dmabuf IPC):
tensors of several sizes, made on the device (torch.full) or copied from host memory
(torch.from_numpy(...).cuda(), as tests/gpu_util.device_field does), in one process. Prints one
JSON line per case. Usage: python tools/ipc_probe.py [E,E,... [how,how,...]] (defaults: all)"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import ghex_amd
    from ghex_amd import _ghx
    ghex_amd.native_library()
    L = _ghx.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    keep = []
    sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
        [20, 64, 100, 132, 200, 260, 300, 516]
    hows = sys.argv[2].split(",") if len(sys.argv) > 2 else ["full", "from_numpy", "empty"]
    for E in sizes:
        for how in hows:
            if how == "full":
                t = torch.full((E, E, E), -1.0, dtype=torch.float64, device="cuda")
            elif how == "empty":
                t = torch.empty((E, E, E), dtype=torch.float64, device="cuda")
            else:
                t = torch.from_numpy(np.full((E, E, E), -1.0)).cuda()
            torch.cuda.synchronize()
            keep.append(t)
            h = (ctypes.c_ubyte * 64)()
            off = ctypes.c_uint64()
            rc = L.ghx_ipc_export(ctypes.c_void_p(t.data_ptr()), h, ctypes.byref(off))
            base, size = ctypes.c_void_p(), ctypes.c_size_t()
            hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size),
                                      ctypes.c_void_p(t.data_ptr()))
            print(json.dumps({"E": E, "how": how, "bytes": t.numel() * 8, "rc": rc,
                              "err": L.ghx_last_error().decode() if rc else "",
                              "offset": off.value, "range": size.value, "ptr": hex(t.data_ptr()),
                              "ptr_mod_2MiB": t.data_ptr() % (2 << 20)}), flush=True)


if __name__ == "__main__":
    main()
