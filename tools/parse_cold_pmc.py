#!/usr/bin/env python3
"""Summarise tools/cold_pmc.sh output: per cache state (mode) and kernel (pack / unpack), the
median of each counter over the dispatches, plus derived figures: bytes (128-B reads, 64-B and
32-B writes), mean in-flight latency in L2 cycles (LEVEL / requests: Little's law over the
request queue), and stall cycles per request. Usage: parse_cold_pmc.py <out dir> [label]"""
import collections
import csv
import glob
import json
import os
import sys


def summarise(d):
    res = {}
    for mdir in sorted(glob.glob(os.path.join(d, "*/"))):
        mode = os.path.basename(mdir.rstrip("/"))
        acc = collections.defaultdict(list)
        for p in sorted(glob.glob(f"{mdir}/p*/pmc_counter_collection.csv")):
            for row in csv.DictReader(open(p)):
                k = row["Kernel_Name"]
                if "k_copy" not in k and "k_self" not in k:
                    continue
                kind = "self" if "k_self" in k else ("pack" if "k_copy<true" in k else "unpack")
                acc[(kind, row["Counter_Name"])].append(float(row["Counter_Value"]))
        med = {k: sorted(v)[len(v) // 2] for k, v in acc.items()}
        for kind in sorted({k for k, _ in med}):
            g = {c: v for (kk, c), v in med.items() if kk == kind}
            r = dict(g)
            rd, wr = g.get("TCC_EA0_RDREQ_sum"), g.get("TCC_EA0_WRREQ_sum")
            if rd:
                r["read_lat_cycles"] = round(g.get("TCC_EA0_RDREQ_LEVEL_sum", 0) / rd, 1)
                r["read_bytes"] = rd * 128
            if wr:
                r["write_lat_cycles"] = round(g.get("TCC_EA0_WRREQ_LEVEL_sum", 0) / wr, 1)
                w64 = g.get("TCC_EA0_WRREQ_64B_sum", 0)
                r["write_bytes"] = w64 * 64 + (wr - w64) * 32
                r["write_partial_32B_reqs"] = wr - w64
            res.setdefault(mode, {})[kind] = r
    return res


if __name__ == "__main__":
    out = {"source": sys.argv[1], "label": sys.argv[2] if len(sys.argv) > 2 else "",
           "pmc": summarise(sys.argv[1])}
    t = os.path.join(sys.argv[1], "time.json")
    if os.path.exists(t):
        lines = [l for l in open(t) if l.startswith("{")]
        if lines:
            out["time"] = json.loads(lines[-1])
    print(json.dumps(out, indent=1))
