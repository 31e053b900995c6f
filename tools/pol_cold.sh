#!/bin/bash
# Warm and cold two-launch step under the short-row cache-policy knob (short_pol 0..3):
# one bench line per setting (no extras), summarised to gpurun_out/pol_cold.jsonl.
set -o pipefail
mkdir -p gpurun_out
for t in short_pol=0 short_pol=1 short_pol=2 short_pol=3 short_pol=0; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-extras --no-cpu-baseline --tune "$t" > gpurun_out/pol.json 2>/dev/null || exit 1
  python - "$t" <<'PY' >> gpurun_out/pol_cold.jsonl
import json, sys
d = json.load(open("gpurun_out/pol.json")); r = d["roofline"]
print(json.dumps({"tune": sys.argv[1], "value": d["value"], **{k: r[k] for k in (
    "pack_kernel_us", "unpack_kernel_us", "step_device_us", "cold_clean_pack_us",
    "cold_clean_unpack_us", "cold_clean_step_us", "cold_dirty_launch_us", "cold_dirty_step_us")}}))
PY
done
