#!/bin/bash
# Developer diagnosis (not product): ghx_ipc_export in 4 concurrent processes on the one GPU
# (tools/ipc_probe.py each), to tell a per-process from a concurrency effect in the dmabuf IPC
# export failures of tests/test_gpu_multiproc.py at 256^3. Usage: bash tools/ipc_multi.sh <out>
OUT=${1:-gpurun_out/ipc_multi}
mkdir -p $OUT
pids=()
for r in 0 1 2 3; do
  timeout -k 10 120 python tools/ipc_probe.py > $OUT/p$r.jsonl 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep -h '"rc": [^0]' $OUT/p*.jsonl | head -20 || true
exit $rc
