O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_bulk.py tests/test_gpu_cpp_co.py tests/test_gpu_graph.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 tools/bin/granule_bench 4128 9 > $O/granule_4128.jsonl 2>&1 && timeout -k 10 120 tools/bin/granule_bench 4144 9 > $O/granule_4144.jsonl 2>&1; echo "granule rc=$?" >> $O/status
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/status
cat $O/status
