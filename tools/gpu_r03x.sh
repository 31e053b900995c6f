#!/bin/bash
# round-3 checkpoint x: pack/unpack floors at H=1/2/3, parity + random exchanges (incl. the
# unaligned-vector knob), then the field_unaligned16 A/B (tools/gpu_r03v.sh)
O=gpurun_out/r03x; mkdir -p $O
for h in 1 2 3; do timeout -k 10 100 tools/bin/pack_floor 21 512 $h || exit 1; done > $O/floors3.jsonl 2>&1
echo "floors rc=$?" >> $O/status
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_r03v.sh
cat $O/status
