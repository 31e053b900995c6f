#!/bin/bash
# round-3 checkpoint al (direct exchange, C++ shm and direct tests): the whole -m gpu suite as the driver runs it, smoke(), the bench at the
# driver's settings. Each step under its own limit; a fault, abort or timeout ends the call.
O=gpurun_out/r03al; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -gt 1 ] && { cat $O/status; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" >> $O/status
[ $rc -ne 0 ] && { cat $O/status; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc" >> $O/status
cat $O/status
