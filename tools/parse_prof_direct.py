"""Summarise tools/prof_direct.sh (rocprofv3 kernel traces of the 2-process direct exchange) into
one JSON: per rank and kernel, count / mean / min / max duration; the epoch launches per
exchange; and per exchange (open start -> unpack end on the rank's stream) the span and the span
minus the pack and unpack kernels (what the epochs add: their launches, fences and the wait for
the peer, which shares the GPU here).

usage: python tools/parse_prof_direct.py gpurun_out/prof_direct [worker mode, default directloop]"""
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    for k in ("k_epoch_open", "k_epoch_close1", "k_epoch_close", "k_epoch", "k_sys_release",
              "k_sys_acquire"):
        if k + "(" in name:
            return k
    if "k_copy<true" in name:
        return "k_copy<pack>"
    if "k_copy<false" in name:
        return "k_copy<unpack>"
    if "k_self" in name:
        return "k_self"
    return name[:60]


def main(d, mode="directloop"):
    how = ("back to back on the stream" if mode == "directloop" else
           "each awaited on the host")
    out = {"source": "tools/prof_direct.sh: rocprofv3 --kernel-trace of tests/mp_exchange_worker.py "
                     f"2 1 1 128 2 40 {mode} (two field layouts, 40 exchanges each, {how}), "
                     "2 processes sharing one MI355X: a close kernel's duration includes its wait "
                     "for the peer's pack", "ranks": {}}
    for r in (0, 1):
        files = glob.glob(os.path.join(d, f"r{r}", "**", "*kernel_trace.csv"), recursive=True)
        if not files:
            continue
        rows = []
        with open(files[0]) as fh:
            for row in csv.DictReader(fh):
                rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]),
                             short(row["Kernel_Name"])))
        rows.sort()
        per = {}
        for s, e, k in rows:
            per.setdefault(k, []).append((e - s) / 1e3)
        kern = {k: {"count": len(v), "avg_us": round(statistics.mean(v), 2),
                    "median_us": round(statistics.median(v), 2),
                    "min_us": round(min(v), 2), "max_us": round(max(v), 2)} for k, v in per.items()}
        # exchanges: each data pack (k_copy<pack> or the mixed k_self) starts one, preceded by
        # a k_epoch_open in the two-launch form; it ends with the next unpack
        spans, extra, launches = [], [], []
        i = 0
        while i < len(rows):
            if rows[i][2] not in ("k_copy<pack>", "k_self"):
                i += 1
                continue
            first = i - 1 if i > 0 and rows[i - 1][2] == "k_epoch_open" else i
            j = i
            data = 0.0
            n_ep = 1 if first < i else 0
            while j < len(rows) and rows[j][2] != "k_copy<unpack>":
                if rows[j][2].startswith("k_epoch"):
                    n_ep += 1
                elif rows[j][2] in ("k_copy<pack>", "k_self"):
                    data += (rows[j][1] - rows[j][0]) / 1e3
                j += 1
            if j == len(rows):
                break
            data += (rows[j][1] - rows[j][0]) / 1e3
            span = (rows[j][1] - rows[first][0]) / 1e3
            spans.append(span)
            extra.append(span - data)
            launches.append(n_ep)
            i = j + 1
        out["ranks"][str(r)] = {
            "kernels": kern, "exchanges": len(spans),
            "epoch_launches_per_exchange": sorted(set(launches)),
            "span_us_median": round(statistics.median(spans), 2) if spans else None,
            "span_minus_data_kernels_us_median": round(statistics.median(extra), 2) if extra else None,
            "span_minus_data_kernels_us_min": round(min(extra), 2) if extra else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_direct",
         sys.argv[2] if len(sys.argv) > 2 else "directloop")
