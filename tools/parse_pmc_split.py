#!/usr/bin/env python3
"""Summarise tools/pmc_split.sh: median counter value per (kernel, workgroups, counter)."""
import collections
import csv
import glob
import json
import re
import sys


def main(d):
    acc = collections.defaultdict(list)
    for p in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(p)):
            m = re.search(r"(k_\w+<[^>]*>)", row["Kernel_Name"])
            if not m:
                continue
            wg = int(row.get("Grid_Size", row.get("Grid_Size_X", 0))) // 256
            acc[(m.group(1), wg, row["Counter_Name"])].append(float(row["Counter_Value"]))
    out = collections.defaultdict(dict)
    for (k, wg, c), v in sorted(acc.items()):
        out[f"{k} wg={wg}"][c] = sorted(v)[len(v) // 2]
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
