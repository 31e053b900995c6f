#!/usr/bin/env python3
"""Summarise tools/pmc_ifetch.sh output by launch position (tools/launch_anatomy.py's order):
pack / unpack inside the step, pack / unpack back to back, and the probe's variants (k_lines
j = 0 x-face lines, 1 long-row lines, 2 all lines, 3 all lines + buffer writes, 4 the same with
dependent writes; warm = the launches not preceded by a cache sweep). Medians per group."""
import collections
import csv
import glob
import json
import sys

REPS = 20
PROBE_REPS = 5


def main(d):
    out = collections.defaultdict(dict)
    for p in sorted(glob.glob(f"{d}/p*/**/pmc_counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(p)))
        disp = sorted({int(r["Dispatch_Id"]) for r in rows})
        by = collections.defaultdict(dict)
        names = {}
        for r in rows:
            by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        copies = [i for i in disp if "k_copy" in names[i] and "seg_s" in names[i]]
        lines = [i for i in disp if "k_lines" in names[i]]
        groups = {"pack_step": copies[0:2 * REPS:2], "unpack_step": copies[1:2 * REPS:2],
                  "pack_alone": copies[2 * REPS:3 * REPS], "unpack_alone": copies[3 * REPS:4 * REPS]}
        per = 3 * PROBE_REPS  # per variant: 2*reps warm + reps after a sweep
        for j in range(5):
            groups[f"probe_j{j}_warm"] = lines[j * per:j * per + 2 * PROBE_REPS]
            groups[f"probe_j{j}_cold"] = lines[j * per + 2 * PROBE_REPS:(j + 1) * per]
        for g, ids in groups.items():
            for c in {k for i in ids for k in by[i]}:
                v = sorted(by[i][c] for i in ids if c in by[i])
                if v:
                    out[g][c] = v[len(v) // 2]
    for g, r in out.items():
        if r.get("TCC_HIT_sum") is not None and r.get("TCC_MISS_sum") is not None:
            t = r["TCC_HIT_sum"] + r["TCC_MISS_sum"]
            r["l2_hit_rate"] = round(r["TCC_HIT_sum"] / t, 3) if t else None
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
