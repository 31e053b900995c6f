#!/bin/bash
# One GPU-box pass for a round's checkpoint: the -m gpu suite, then (unless it crashed) the
# cold/warm PMC passes (tools/cold_pmc.sh) and the bench at the driver's settings. Each step
# under its own time limit; a fault, abort or timeout ends the call (no further GPU steps).
# Usage: bash tools/gpu_round.sh <tag> [skip-tests]
T=${1:-r03}
O=gpurun_out/$T
mkdir -p $O
stop() { echo "$1 rc=$2: stopping" >> $O/status; cat $O/status; exit $2; }
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
  [ $rc -gt 1 ] && stop tests $rc
fi
timeout -k 10 520 bash tools/cold_pmc.sh $O/cold; rc=$?; echo "cold rc=$rc" >> $O/status
[ $rc -ne 0 ] && stop cold $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc" >> $O/status
cat $O/status
