#!/usr/bin/env python3
"""profiles/pmc_traffic.json's per-rank-plan entries (N512_H2_w2/w4/w8, what bench.py quotes as
roofline.traffic at N>1) from tools/pmc_emu.sh passes: the fused pack / unpack launch of rank 0's
plan (the k_copy row with the largest grid), HBM bytes per launch = TCC_EA0_RDREQ x 128 B (the
gfx950 read correction of MI355X_MICROARCH.md: FETCH_SIZE counts a 128-B request as 64 B) +
WRITE_SIZE x 1 KiB. Usage: tools/pmc_emu_traffic.py <tag> <pmc_emu dir> <world> [...]
(pairs of dir and world); writes profiles/<tag>_pmc_emu_w<W>.json and updates pmc_traffic.json."""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import parse_pmc_split  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def entry(rows):
    best = {}
    for k, v in rows.items():
        m = re.match(r"k_copy<(true|false),.*wg=(\d+)$", k)
        if not m:
            continue
        kind = "pack" if m.group(1) == "true" else "unpack"
        wg = int(m.group(2))
        if kind not in best or wg > best[kind][0]:
            best[kind] = (wg, v)
    return {kind: {"hbm_bytes_per_launch": v["TCC_EA0_RDREQ_sum"] * 128 + v["WRITE_SIZE"] * 1024,
                   "read_bytes": v["TCC_EA0_RDREQ_sum"] * 128,
                   "write_bytes": v["WRITE_SIZE"] * 1024, "workgroups": wg}
            for kind, (wg, v) in best.items()}


def main(tag, pairs):
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    traffic = json.load(open(tp))
    for d, w in pairs:
        rows = parse_pmc_split.main(d)
        out = os.path.join(ROOT, "profiles", f"{tag}_pmc_emu_w{w}.json")
        json.dump(rows, open(out, "w"), indent=1)
        e = entry(rows)
        src = (f"profiles/{tag}_pmc_emu_w{w}.json (rocprofv3 --pmc over tools/emu_rank_bench.py "
               f"{w}: rank 0's plan of the {w}-rank decomposition on one GPU, tools/pmc_emu.sh; "
               f"tools/pmc_emu_traffic.py)")
        for v in e.values():
            v["source"] = src
        traffic[f"N512_H2_w{w}"] = e
    json.dump(traffic, open(tp, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[2:]
    main(sys.argv[1], [(a[i], int(a[i + 1])) for i in range(0, len(a), 2)])
