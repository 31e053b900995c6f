#!/usr/bin/env python3
"""Developer sweep: bench.py's config-5 (unstructured, 10M cells, 5 % halo, 7 peers) timing under
ghx_tune settings given as arguments ("key=v,key=v" each). One JSON line per setting."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ghex_amd import _ghx
    dev = torch.device("cuda", 0)
    for t in sys.argv[1:] or [""]:
        _ghx.call("ghx_tune", b"reset", 0)
        for kv in filter(None, t.split(",")):
            k, v = kv.split("=")
            _ghx.call("ghx_tune", k.encode(), int(v))
        r = {lv: bench.bench_config5(torch, dev, _ghx, lv) for lv in (1, 8)}
        print(json.dumps({"tune": t, "levels1": r[1]["GBps"], "levels8": r[8]["GBps"],
                          "us1": r[1]["us_per_exchange"], "us8": r[8]["us_per_exchange"]}),
              flush=True)


if __name__ == "__main__":
    main()
