#!/bin/bash
# One GPU-box pass: the -m gpu suite, the bench at the driver's settings and at the defaults,
# and the N>1 rehearsal. Each step under its own time limit; stops at the first failing step.
# Usage: bash tools/gpu_check.sh <tag>
set -o pipefail
T=${1:-c}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
  > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status
tail -3 $O/tests.log
# 0 = passed, 1 = some tests failed: go on; anything else (timeout, abort, fault): stop here
if [ $rc -gt 1 ]; then cat $O/status; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err \
  && timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  && timeout -k 10 600 bash tools/rehearse_multi.sh $O/rehearse
echo "bench+rehearse rc=$?" >> $O/status
cat $O/status
