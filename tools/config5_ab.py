#!/usr/bin/env python3
"""Developer A/B (not product): BASELINE config 5 (rank 0 of 8, 10M cells, lists from the
product's make_pattern<unstructured>) through bench.bench_config5 under ghx_tune settings, in the
given order (plans rebuilt per setting): the verified gather + scatter step and each launch by
its own events beside the index-list floor probe. One JSON line per (setting, levels).
usage: python tools/config5_ab.py [--settings JSON list of dicts] [--levels 1,8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settings", default='[{"fast_addr": 0}, {}, {"fast_addr": 0}, {}]')
    ap.add_argument("--levels", default="1,8")
    a = ap.parse_args()
    import torch
    import bench
    from ghex_amd import _ghx
    dev = torch.device("cuda", 0)
    pats = bench.config5_patterns()[0]
    for st in json.loads(a.settings):
        for lv in (int(x) for x in a.levels.split(",")):
            _ghx.call("ghx_tune", b"reset", 0)
            for k, v in st.items():
                _ghx.call("ghx_tune", k.encode(), int(v))
            r = bench.bench_config5(torch, dev, _ghx, lv, pats)
            fl = r.get("index_floor", {})
            print(json.dumps({"tune": st, "levels": lv, "GBps": r.get("GBps"),
                              "us_per_exchange": r.get("us_per_exchange"),
                              "verified": r.get("verified"),
                              "gather_us": fl.get("pack_kernel_us"),
                              "scatter_us": fl.get("unpack_kernel_us"),
                              "gather_floor_us": fl.get("gather_us"),
                              "scatter_floor_us": fl.get("scatter_us")}), flush=True)
    _ghx.call("ghx_tune", b"reset", 0)


if __name__ == "__main__":
    main()
