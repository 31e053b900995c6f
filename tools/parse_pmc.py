#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per kernel (pack/unpack) median counter values and the HBM
bytes per launch with the gfx950 corrections of MI355X_MICROARCH.md §HBM (FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE reports half of a wide streaming read: RDREQ are 128-B
requests tallied at 64 B, so read bytes are taken from the request counters instead)."""
import collections
import csv
import glob
import json
import sys


def main(d):
    acc = collections.defaultdict(list)
    for p in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
        for row in csv.DictReader(open(p)):
            k = row["Kernel_Name"]
            if "k_self" in k:
                kind = "self"
            elif "k_copy" in k:
                kind = "pack" if "k_copy<true" in k else "unpack"
            else:
                continue
            acc[(kind, row["Counter_Name"])].append(float(row["Counter_Value"]))
    med = {k: sorted(v)[len(v) // 2] for k, v in acc.items()}
    out = {}
    for kind in sorted({k for k, _ in med}):
        g = lambda c: med.get((kind, c))
        r = {c: g(c) for c in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum",
                               "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum",
                               "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")}
        fetch_kib = r["FETCH_SIZE"] or 0
        write_kib = r["WRITE_SIZE"] or 0
        r["read_bytes_FETCH_SIZE_x2"] = fetch_kib * 1024 * 2  # guide: FETCH_SIZE reads 1/2
        r["write_bytes_WRITE_SIZE"] = write_kib * 1024
        r["hbm_bytes_per_launch"] = r["read_bytes_FETCH_SIZE_x2"] + r["write_bytes_WRITE_SIZE"]
        out[kind] = r
    return out


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1]), indent=1))
