#!/bin/bash
# round-3 checkpoint h: mixed-host bulk exchange + staging tests, request ceilings, N>1 rehearsal
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_staging.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 tools/bin/req_ceiling 11 > $O/req_ceiling.jsonl 2>&1; rc=$?; echo "req rc=$rc" >> $O/status
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 bash tools/rehearse_multi.sh $O/rehearse; echo "rehearse rc=$?" >> $O/status
cat $O/status
