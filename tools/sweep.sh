#!/bin/bash
# Developer sweep of tuning knobs with tools/microbench.py (one process per setting).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sweep_$(date +%s).jsonl
mkdir -p $R/gpurun_out
for t in "" "unroll=8" "unroll=2" "nt=1" "nt=2" "tile_bytes=65536" "tile_bytes=4096" "grid_cap=2048" "tile_bytes=65536,unroll=8"; do
  timeout -k 10 120 python $R/tools/microbench.py --tune "$t" >> $OUT
done
for h in 1 3; do
  timeout -k 10 120 python $R/tools/microbench.py --halo $h >> $OUT
done
echo $OUT
