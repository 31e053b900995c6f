#!/bin/bash
# round-3 checkpoint f: the measured-engine staging copies (unit tests, multi-process staged /
# pipelined exchanges both ways), then the bench's host-staged leg
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_staging.py tests/test_gpu_multiproc.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/status
cat $O/status
