#!/bin/bash
# Runs tools/ipc_worker_diag.py as 4 ranks for each mode (developer diagnosis, not product).
# Usage: bash tools/ipc_diag.sh <out> [N]
OUT=${1:-gpurun_out/ipc_diag}; N=${2:-256}
mkdir -p $OUT
port=$((20000 + RANDOM % 20000))
for mode in ${MODES:-plain barrier sync early}; do
  port=$((port + 1))
  pids=()
  for r in 0 1 2 3; do
    env RANK=$r WORLD_SIZE=4 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port LOCAL_RANK=0 \
      timeout -k 10 60 python tools/ipc_worker_diag.py $N $mode > $OUT/$mode.r$r.log 2>&1 &
    pids+=($!)
  done
  worst=0
  for p in "${pids[@]}"; do wait $p; rc=$?; [ $rc -gt $worst ] && worst=$rc; done
  grep -h '^{' $OUT/$mode.r*.log >> $OUT/summary.jsonl
  if [ $worst -gt 1 ]; then echo "mode $mode rc=$worst" >> $OUT/summary.jsonl; exit $worst; fi
done
cat $OUT/summary.jsonl
