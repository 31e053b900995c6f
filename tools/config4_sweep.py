#!/usr/bin/env python3
"""Developer measurement (not product): BASELINE config 4 (5 fields 256^3 [f64,f32,f64,f32,f64],
H=3) through bench.bench_config4 under plan-shaping ghx_tune settings: the verified two-launch
step, the pack / unpack launches by their own events and the five-field floor probe
(tools/pack_floor.hip ghx_probe_multi_floor). One JSON line per setting.
usage: python tools/config4_sweep.py [--settings JSON list of ghx_tune dicts]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (round 5's first pass, before short-row tiles were sized per field: 512-row tiles and
# xcd_pair 0 were both faster than the plan-wide rule's 2048, profiles/r05_config4_sweep.jsonl)
SETTINGS = [{}] + [{"small_tile_rows": r} for r in (256, 512, 1024)] + \
    [{"xcd_pair": 0}, {"xcd_pair": 0, "small_tile_rows": 512}, {"short_pol": 1}]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", default="")
    a = ap.parse_args()
    settings = json.loads(a.settings) if a.settings else SETTINGS
    import torch
    import bench
    import ghex_amd
    from ghex_amd import _ghx
    from ghex_amd.structured import regular as R
    dev = torch.device("cuda", 0)
    for st in settings:
        _ghx.call("ghx_tune", b"reset", 0)
        for k, v in st.items():
            _ghx.call("ghx_tune", k.encode(), v)
        r = bench.bench_config4(torch, dev, ghex_amd, R)
        fl = r.get("floor", {})
        print(json.dumps({"tune": st, "GBps": r["GBps"], "us_per_exchange": r["us_per_exchange"],
                          "verified": r["verified"], "pack_kernel_us": fl.get("pack_kernel_us"),
                          "unpack_kernel_us": fl.get("unpack_kernel_us"),
                          "pack_floor_us": fl.get("pack_floor_us"),
                          "unpack_floor_us": fl.get("unpack_floor_us"),
                          "unpack_reads_writes_us": fl.get("unpack_reads_writes_us")}),
              flush=True)
    _ghx.call("ghx_tune", b"reset", 0)


if __name__ == "__main__":
    main()
