#!/usr/bin/env python3
"""Developer soak (GPU box): the seeded random exchanges of tests/test_gpu_fuzz.py over seed
ranges far beyond the suite's 60 structured / 40 unstructured seeds, within a time budget. Each
seed is the suite's own case (draw_case / draw_unstructured) checked the suite's own way (every
cell against the oracle's exchange, every packed byte against the oracle's buffer). One progress
line per 25 seeds on stderr; one JSON summary line on stdout with every failing seed and its
error. --direct runs the same structured cases through the direct exchange's double-buffered
launches (run_case_direct). usage: python tools/fuzz_soak.py --structured 60:2000
--unstructured 40:2000 --direct 230:2000 --seconds 400"""
import argparse
import json
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--structured", default="60:1000")
    p.add_argument("--unstructured", default="40:1000")
    p.add_argument("--direct", default="0:0",
                   help="seed range of the double-buffered direct form (run_case_direct)")
    p.add_argument("--udirect", default="0:0",
                   help="seed range of the unstructured direct form (run_unstructured_direct)")
    p.add_argument("--seconds", type=float, default=300)
    a = p.parse_args()
    import torch
    if not torch.cuda.is_available():
        raise SystemExit("fuzz_soak needs a GPU")
    import ghex_amd
    ghex_amd.native_library()
    from tests import test_gpu_fuzz as F
    t0 = time.time()
    out = {"structured": {"ran": 0, "failed": []}, "unstructured": {"ran": 0, "failed": []},
           "direct": {"ran": 0, "failed": []}, "udirect": {"ran": 0, "failed": []}}
    kinds = [("structured", a.structured, lambda s: F.run_case(F.draw_case(s))),
             ("unstructured", a.unstructured, lambda s: F.run_unstructured(F.draw_unstructured(s))),
             ("direct", a.direct, lambda s: F.run_case_direct(F.draw_case(s))),
             ("udirect", a.udirect, lambda s: F.run_unstructured_direct(F.draw_unstructured(s)))]
    kinds = [k for k in kinds if k[1].split(":")[0] != k[1].split(":")[1]]
    share = a.seconds / len(kinds)
    for i, (name, rng, fn) in enumerate(kinds):
        lo, hi = (int(x) for x in rng.split(":"))
        stop = t0 + share * (i + 1)
        rec = out[name]
        rec["first_seed"] = lo
        for seed in range(lo, hi):
            if time.time() > stop:
                break
            try:
                got = fn(seed)
                if isinstance(got, int):  # the direct forms: peer messages checked
                    rec["peer_messages"] = rec.get("peer_messages", 0) + got
            except Exception as e:
                rec["failed"].append({"seed": seed, "error": f"{type(e).__name__}: {str(e)[:300]}",
                                      "where": traceback.format_exc()[-600:]})
            rec["ran"] += 1
            rec["last_seed"] = seed
            if rec["ran"] % 25 == 0:
                print(f"{name}: {rec['ran']} seeds, {len(rec['failed'])} failed, "
                      f"{time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    out["seconds"] = round(time.time() - t0, 1)
    print(json.dumps(out), flush=True)
    return 1 if any(v["failed"] for v in out.values() if isinstance(v, dict)) else 0


if __name__ == "__main__":
    sys.exit(main())
