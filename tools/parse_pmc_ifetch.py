#!/usr/bin/env python3
"""Summarise tools/pmc_ifetch.sh output: per kernel (pack, unpack, probe k_lines by grid) the
median of each counter over its launches."""
import collections
import csv
import glob
import json
import sys


def main(d):
    acc = collections.defaultdict(list)
    for p in sorted(glob.glob(f"{d}/p*/**/pmc_counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(p)):
            k = row["Kernel_Name"]
            if "k_copy" in k:
                kind = "pack" if "k_copy<true" in k else "unpack"
            elif "k_lines" in k:
                kind = "probe_k_lines"
            else:
                continue
            acc[(kind, row["Counter_Name"])].append(float(row["Counter_Value"]))
    out = collections.defaultdict(dict)
    for (kind, c), v in sorted(acc.items()):
        out[kind][c] = sorted(v)[len(v) // 2]
    for kind, r in out.items():
        if r.get("SQ_IFETCH"):
            r["ifetch_latency"] = round(r.get("SQ_IFETCH_LEVEL", 0) / r["SQ_IFETCH"], 1)
        if r.get("SQ_WAVES"):
            r["wave_cycles_per_wave"] = round(r.get("SQ_WAVE_CYCLES", 0) / r["SQ_WAVES"], 1)
            r["wait_inst_per_wave"] = round(r.get("SQ_WAIT_INST_ANY", 0) / r["SQ_WAVES"], 1)
            if "SQ_ACTIVE_INST_VALU" in r:
                r["valu_active_per_wave"] = round(r["SQ_ACTIVE_INST_VALU"] / r["SQ_WAVES"], 1)
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
