#!/bin/bash
# Developer sweep: bench.py at each short-row cache policy (warm = bench value, cold = roofline
# cold_launch_us). Output: gpurun_out/pol_sweep.jsonl
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pol_sweep.jsonl
: > $OUT
for pol in 0 1 2 3; do
  timeout -k 10 180 python $R/bench.py --no-cpu-baseline --tune short_pol=$pol "$@" | tail -1 >> $OUT
done
