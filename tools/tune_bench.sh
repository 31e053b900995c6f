#!/bin/bash
# Developer sweep: bench.py (no extras) once per ghx_tune setting given as arguments, e.g.
#   bash tools/tune_bench.sh "" "unroll=8" "small_tile_rows=2048,unroll=2"
# Output: gpurun_out/tune_bench.jsonl (one bench line per setting, "tune" added)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/tune_bench.jsonl
: > $OUT
for t in "$@"; do
  line=$(timeout -k 10 120 python $R/bench.py --no-cpu-baseline --no-extras --tune "$t" | tail -1)
  echo "{\"tune\": \"$t\", \"bench\": $line}" >> $OUT
done
