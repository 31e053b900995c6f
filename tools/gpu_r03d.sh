#!/bin/bash
# round-3 checkpoint d: bulk epochs incl. graph replay (multi-process), config-5 / H=1 PMC, SDMA
# engine placement of the host-staging copies, bench bulk leg.
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiproc.py -k "bulk" -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 500 bash tools/config5_pmc.sh $O/c5; echo "c5 rc=$?" >> $O/status
timeout -k 10 120 tools/bin/sdma_bench 25362944 15 > $O/sdma.jsonl 2>&1; rc=$?; echo "sdma rc=$rc" >> $O/status
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/mct -o mct --output-format csv -- $GRAFT_REPO_ROOT/tools/bin/sdma_bench 25362944 5 > $GRAFT_REPO_ROOT/$O/sdma_traced.jsonl 2>&1; echo "mct rc=$?" >> $GRAFT_REPO_ROOT/$O/status
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/status
cat $O/status
