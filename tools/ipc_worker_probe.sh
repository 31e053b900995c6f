#!/bin/bash
# Developer diagnosis (not product): the multi-process bulk worker of tests/test_gpu_multiproc.py
# at 4 ranks (2,2,1) over several sizes, and tools/ipc_probe.py as a fresh process's first
# allocation. Diagnosis switches (env, passed to the worker): ALLOC(S) numpy|device|pinned,
# PROBE=1 (an export at start), DIAG_SYNC=1, DIAG_PRIME=small|big|self, DIAG_KEEPCO=1 (no
# teardown of the first bulk object), DIAG_BARRIER=1 (ordered teardown), DIAG_TEARDOWN=
# imports|puts|epochs|free (one part of the teardown, then an export probe). A step that exits 0 or 1 (Python error) lets the next run; anything else (abort,
# fault, time limit) ends the script. Usage: bash tools/ipc_worker_probe.sh <out> [N ...]
OUT=${1:-gpurun_out/ipc_worker}
shift
mkdir -p $OUT
port=$((20000 + RANDOM % 20000))
step_world() {  # name px py pz N mode
  local name=$1; shift
  local w=$(($1 * $2 * $3))
  port=$((port + 1))
  local pids=()
  for ((r = 0; r < w; r++)); do
    env RANK=$r WORLD_SIZE=$w MASTER_ADDR=127.0.0.1 MASTER_PORT=$port LOCAL_RANK=0 AMD_LOG_LEVEL=1 \
      GHX_TEST_FIELD_ALLOC=${ALLOC:-numpy} GHX_WORKER_EXPORT_PROBE=${PROBE:-0} GHX_DIAG_SYNC=${DIAG_SYNC:-0} \
      GHX_DIAG_PRIME=${DIAG_PRIME:-0} \
      GHX_DIAG_KEEPCO=${DIAG_KEEPCO:-0} GHX_DIAG_BARRIER=${DIAG_BARRIER:-0} \
      GHX_DIAG_TEARDOWN=${DIAG_TEARDOWN:-} \
      timeout -k 10 150 python tests/mp_exchange_worker.py $1 $2 $3 $4 2 1 $5 > $OUT/${name}_r$r.log 2>&1 &
    pids+=($!)
  done
  local worst=0
  for p in "${pids[@]}"; do wait $p; rc=$?; [ $rc -gt $worst ] && worst=$rc; done
  echo "$name rc=$worst $(grep -h 'bad cells' $OUT/${name}_r0.log)" >> $OUT/status
  grep -h "hipIpcGetMemHandle\|IPC memory creation\|export_probe\|ipc_trace" $OUT/${name}_r*.log | head -40 >> $OUT/status
  if [ $worst -gt 1 ]; then exit $worst; fi
}
for a in ${ALLOCS:-numpy}; do
  for n in "${@:-192 256 320}"; do
    ALLOC=$a step_world w4_n${n}_bulk_$a 2 2 1 $n bulk
  done
done
cat $OUT/status
