#!/bin/bash
# Kernel start/stop-event durations in the bench line against a rocprofv3 kernel trace of the
# same command, and the bench at the driver's settings without the profiler.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-timing}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest $R/tests/test_gpu_bench.py -q --timeout 120 --timeout-method thread -k launch_timing > $OUT/test.log 2>&1 || { tail -20 $OUT/test.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cold --no-extras --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.err || exit 1
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cold > $OUT/b.json 2> $OUT/b.err
