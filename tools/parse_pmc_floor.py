#!/usr/bin/env python3
"""Summarise tools/pmc_floor.sh: per unpack-floor probe variant, the median per-dispatch
counters of its k_pieces / k_pieces_il launches (fabric write and read requests, 64-B writes,
LEVEL / REQ latency, in flight). Compare with the unpack kernel's rows of
tools/parse_pmc_credit.py (all_unpack)."""
import collections
import csv
import glob
import json
import os
import sys

NAMES = {"2": "writes_only", "3": "writes_plus_buffer_streamed_first",
         "4": "writes_buffer_interleaved"}


def main(d):
    out = {"source": "tools/pmc_floor.sh + tools/parse_pmc_floor.py (rocprofv3 --pmc, "
                     "per-dispatch medians of the probe launches)"}
    for vdir in sorted(glob.glob(os.path.join(d, "v*"))):
        v = os.path.basename(vdir)[1:]
        acc = collections.defaultdict(list)
        for p in glob.glob(f"{vdir}/p*/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(p)):
                if "k_pieces" not in row["Kernel_Name"]:
                    continue
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
        med = {k: sorted(x)[len(x) // 2] for k, x in acc.items()}
        r = {"counters": med}
        wr, rd = med.get("TCC_EA0_WRREQ_sum"), med.get("TCC_EA0_RDREQ_sum")
        if wr and med.get("TCC_EA0_WRREQ_LEVEL_sum"):
            r["wr_latency"] = round(med["TCC_EA0_WRREQ_LEVEL_sum"] / wr, 1)
        if rd and med.get("TCC_EA0_RDREQ_LEVEL_sum"):
            r["rd_latency"] = round(med["TCC_EA0_RDREQ_LEVEL_sum"] / rd, 1)
        out[NAMES.get(v, v)] = r
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
