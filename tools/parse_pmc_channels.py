#!/usr/bin/env python3
"""Summarise tools/pmc_channels.sh: per run (tune) and per pitch (the probe's plans run in pitch
order, equal dispatch counts), the x-face launch's read requests per (XCD, L2 channel), their
max/mean skew, and the launch time. Usage: parse_pmc_channels.py <out-dir> [n_pitches]"""
import glob
import json
import os
import sys

import numpy as np


def load(path):
    d = json.load(open(path))["rocprofiler-sdk-tool"][0]
    inst = d["counters"][0]["instances"]
    idx = [(i["dimensions"][0]["index"], i["dimensions"][1]["index"]) for i in inst]
    recs = []
    for r in d["callback_records"]["counter_collection"]:
        v = [x["value"] for x in r["records"]]
        dd = r["dispatch_data"]
        recs.append((dd["dispatch_info"]["dispatch_id"], np.array(v),
                     dd["end_timestamp"] - dd["start_timestamp"]))
    return idx, sorted(recs, key=lambda x: x[0])


def main(out, npitch=2):
    res = []
    for j in sorted(glob.glob(os.path.join(out, "j*")), key=lambda p: int(p.rsplit("j", 1)[1] or 0)):
        k = j.rsplit("j", 1)[1]
        tf = os.path.join(out, f"tune{k}.txt")
        tune = open(tf).read().strip() if os.path.exists(tf) else ""
        f = glob.glob(os.path.join(j, "*results.json"))
        if not f:
            continue
        idx, recs = load(f[0])
        per = len(recs) // npitch
        for p in range(npitch):
            part = recs[p * per:(p + 1) * per][2:]
            M = np.zeros((8, 16))
            for _, v, _ in part:
                for (ch, x), val in zip(idx, v):
                    M[x, ch] += val
            M /= max(1, len(part))
            t = sorted(x[2] for x in part)[len(part) // 2] / 1e3
            res.append({"tune": tune, "pitch_index": p, "rdreq": round(M.sum()),
                        "skew_xcd_channel_max_over_mean": round(M.max() / M.mean(), 3),
                        "skew_channel_max_over_mean": round(M.sum(0).max() / M.sum(0).mean(), 3),
                        "launch_us": round(t, 2),
                        "Glines_per_s": round(M.sum() / t / 1e3, 1)})
            print(json.dumps(res[-1]))
    return res


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
