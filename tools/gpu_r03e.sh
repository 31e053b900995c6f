#!/bin/bash
# round-3 checkpoint e: host-staging copy forms (HIP stream kinds, chunked round trips, torch)
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 120 tools/bin/sdma_bench 25362944 15 > $O/sdma.jsonl 2>&1; rc=$?; echo "sdma rc=$rc" >> $O/status
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python tools/staged_bench.py > $O/staged.jsonl 2>&1; echo "staged rc=$?" >> $O/status
cat $O/status
