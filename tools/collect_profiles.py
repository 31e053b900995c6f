#!/usr/bin/env python3
"""Copy the judged rocprofv3 summaries of a round from gpurun_out/prof_<round>/ into profiles/:

  profiles/<round>_bench_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `python3 bench.py`
  profiles/<round>_bench_kernels_by_grid.csv  the same trace per (kernel, workgroup count)
  profiles/<round>_h{1,3}_kernel_stats.csv  the same at halo 1 / 3
  profiles/<round>_pmc.json                 per-kernel counters + corrected HBM bytes per launch
  profiles/pmc_traffic.json                 what bench.py reads for roofline.traffic
  profiles/<round>_bench.json               the bench JSON line printed under the profiler
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from parse_pmc import main as parse_pmc  # noqa: E402


def main(rn):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rn}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    p = os.path.join(src, "bench", "kt_kernel_stats.csv")
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, f"{rn}_bench_kernel_stats.csv"))
    for h in (1, 3):
        p = os.path.join(src, f"h{h}", "kt_kernel_stats.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, f"{rn}_h{h}_kernel_stats.csv"))
    blog = os.path.join(src, "bench.log")
    line = [l for l in open(blog) if l.startswith("{")] if os.path.exists(blog) else []
    if line:
        with open(os.path.join(dst, f"{rn}_bench.json"), "w") as fh:
            fh.write(line[-1])
    # per (kernel, workgroups) durations from the kernel trace: the bench's extras launch the
    # same kernels on other plans (config 4, config 5, put), so the headline launch is the
    # k_self / k_copy row with the 512^3 plan's grid
    kt = os.path.join(src, "bench", "kt_kernel_trace.csv")
    if os.path.exists(kt):
        import collections
        import csv
        import re
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            m = re.search(r"(k_\w+<[^>]*>)", r["Kernel_Name"])
            if m:
                acc[(m.group(1), int(r["Grid_Size_X"]) // 256)].append(
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        with open(os.path.join(dst, f"{rn}_bench_kernels_by_grid.csv"), "w") as fh:
            fh.write("kernel,workgroups,calls,avg_ns,median_ns,min_ns,max_ns\n")
            for (k, wg), v in sorted(acc.items()):
                v.sort()
                fh.write(f"\"{k}\",{wg},{len(v)},{sum(v) / len(v):.0f},{v[len(v) // 2]},"
                         f"{v[0]},{v[-1]}\n")
    pmc, traffic = {}, {}
    for h in (1, 2, 3):
        d = os.path.join(src, f"pmc_h{h}")
        if os.path.isdir(d):
            r = parse_pmc(d)
            ds = os.path.join(src, f"pmc_h{h}_self")
            if os.path.isdir(ds):
                rs = parse_pmc(ds)
                if "self" in rs:
                    r["self"] = rs["self"]
            pmc[f"N512_H{h}"] = r
            traffic[f"N512_H{h}"] = {k: {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"]}
                                     for k, v in r.items()}
    if not pmc:  # kernel-trace-only round (SKIP_PMC=1): keep the last PMC summary
        print("collected", rn, "(no PMC passes)")
        return
    with open(os.path.join(dst, f"{rn}_pmc.json"), "w") as fh:
        json.dump(pmc, fh, indent=1)
    traffic["source"] = f"profiles/{rn}_pmc.json (rocprofv3 --pmc, tools/pmc.sh)"
    tp = os.path.join(dst, "pmc_traffic.json")
    if os.path.exists(tp):  # keep the per-rank-plan entries (N512_H2_w*, tools/pmc_emu.sh)
        old = json.load(open(tp))
        traffic = {**{k: v for k, v in old.items() if "_w" in k}, **traffic}
    with open(tp, "w") as fh:
        json.dump(traffic, fh, indent=1)
    print("collected", rn)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
