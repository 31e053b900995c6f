#!/bin/bash
# round-3 ak: the direct exchange (pack into the receivers' buffers over IPC, device epochs):
# the multi-process tests, then the N=2/4 rehearsals whose isolated leg now also runs it.
O=gpurun_out/r03ak; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiproc.py -x -v --timeout 150 --timeout-method thread -k "direct" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status; tail -12 $O/tests.log
[ $rc -ne 0 ] && { cat $O/status; exit $rc; }
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --rehearse --steps 50 --warmup 5 > $O/n$n.json 2> $O/n$n.err; rc=$?
  echo "n$n rc=$rc" >> $O/status; [ $rc -ne 0 ] && { cat $O/status; exit $rc; }
done
cat $O/status
