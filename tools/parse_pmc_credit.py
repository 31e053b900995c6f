#!/usr/bin/env python3
"""Summarise tools/pmc_credit.sh: per row class (matched by workgroup count to the classes of
tools/microbench.py) and direction, the fabric requests, their mean latency (LEVEL / REQ, L2
cycles) and the mean number in flight (LEVEL / active cycles).

GRBM_GUI_ACTIVE counts the profiled dispatch window, which carries a fixed overhead; the
8-workgroup corner launch of the same halo width (a few hundred requests) measures it, and it is
subtracted before the per-cycle figures (`cycles_eff`)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_pmc_split import main as split  # noqa: E402


def summarise(d):
    out = {"source": "tools/pmc_credit.sh + tools/parse_pmc_credit.py (rocprofv3 --pmc, "
                     "per-dispatch medians; microbench.py classes, eager launches)"}
    for h in sorted(x for x in os.listdir(d) if x.startswith("h")):
        lines = [l for l in open(os.path.join(d, h, "time.json")) if l.startswith("{")]
        res = json.loads(lines[-1])["results"]
        s = split(os.path.join(d, h))
        raw = {}
        for cls, r in res.items():
            if "tiles" not in r:
                continue
            pack = cls.endswith("_pack")
            # k_copy<PACK, seg_s, RUNS=false, ...> (round 6 added DBL / UU / REC parameters)
            pre = f"k_copy<{'true' if pack else 'false'}, ghx::seg_s, false"
            c = next((v for k, v in s.items()
                      if k.startswith(pre) and k.endswith(f" wg={r['tiles']}")), None)
            if c:
                raw[cls] = (r, c)
        base = raw["corner_pack"][1]["GRBM_GUI_ACTIVE"]
        rows = {"overhead_cycles": base}
        for cls, (r, c) in raw.items():
            if cls.startswith(("corner", "edge", "face_y", "face_z")):
                continue  # tiny, or face_y/face_z: same workgroup count, not told apart
            eff = c["GRBM_GUI_ACTIVE"] - base
            rd, rl = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_RDREQ_LEVEL_sum"]
            wr, wl = c["TCC_EA0_WRREQ_sum"], c["TCC_EA0_WRREQ_LEVEL_sum"]
            rows[cls] = {"tiles": r["tiles"], "bytes": r["bytes"], "rd_req": rd, "wr_req": wr,
                         "wr_64B": c["TCC_EA0_WRREQ_64B_sum"],
                         "rd_latency": round(rl / rd, 1), "wr_latency": round(wl / wr, 1),
                         "cycles_eff": eff, "rd_per_cycle": round(rd / eff, 3),
                         "wr_per_cycle": round(wr / eff, 3), "rd_in_flight": round(rl / eff),
                         "wr_in_flight": round(wl / eff),
                         "rd_credit_stall": c["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"]}
        out[h] = rows
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1]), indent=1))
