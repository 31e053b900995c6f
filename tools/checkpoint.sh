#!/bin/bash
# One GPU-box checkpoint, parameterised (replaces round 3's per-checkpoint gpu_r03*.sh scripts).
# Each step runs under its own time limit; the first failing step ends the call (no further GPU
# work after a fault, abort or timeout; pytest's "some tests failed" (rc 1) is recorded and the
# call goes on, any other status stops it).
#
# Usage: bash tools/checkpoint.sh <tag> <step> [<step> ...]
#   tests            the whole -m gpu suite, as the driver runs it
#   tests=<args>     pytest on <args>, shell-parsed (e.g. "tests=tests/test_gpu_bench.py -k 'a or b'")
#   smoke            __graft_entry__.smoke()
#   bench            bench.py at the driver's settings (--steps 20 --warmup 5)
#   bench=<args>     bench.py <args>  (e.g. "bench=--no-cold --no-extras")
#   rehearse=<n>     bench.py --gpus n --rehearse (n=2/4 through bench.py's own spawning, n=8
#                    through torch.distributed.run as the driver launches it)
#   bulkn=<n>        bench.py --bulk-only n: the N>1 isolated zero-copy leg alone (n children on
#                    the one GPU: puts + direct, verified)
#   prof             rocprofv3 kernel trace + stats of the bench (tools/profile_round.sh, no PMC)
#   pmc              the PMC passes of tools/profile_round.sh (halo 1/2/3)
#   profdirect       rocprofv3 kernel traces of the 2-process direct exchange (tools/prof_direct.sh)
#   run=<cmd>        any other command (one step, same limit)
# Results: gpurun_out/<tag>/ (status, one log per step).
T=${1:?tag}
shift
O=gpurun_out/$T
mkdir -p $O
LIM=${STEP_LIMIT:-600}
i=0
for s in "$@"; do
  i=$((i + 1))
  name=${s%%=*}
  arg=""
  [ "$s" != "$name" ] && arg=${s#*=}
  log=$O/$i-$name.log
  case $name in
    tests) eval "timeout -k 10 $LIM python -u -m pytest ${arg:-tests -m gpu} -x -v --timeout 150 \
             --timeout-method thread" > $log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
             > $log 2>&1 ;;
    bench) timeout -k 10 $LIM python bench.py ${arg:---steps 20 --warmup 5} > $O/$i-bench.json \
             2> $log ;;
    rehearse)
      if [ "$arg" = 8 ]; then
        timeout -k 10 $LIM python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
          --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --rehearse \
          --steps 50 --warmup 5 > $O/$i-rehearse$arg.json 2> $log
      else
        timeout -k 10 $LIM python bench.py --gpus $arg --rehearse --steps 50 --warmup 5 \
          > $O/$i-rehearse$arg.json 2> $log
      fi ;;
    bulkn) timeout -k 10 $LIM python bench.py --bulk-only $arg --steps 20 \
             > $O/$i-bulk$arg.json 2> $log ;;
    prof) SKIP_PMC=1 timeout -k 10 $LIM bash tools/profile_round.sh $T > $log 2>&1 ;;
    pmc) PMC_ONLY=1 timeout -k 10 $LIM bash tools/profile_round.sh $T > $log 2>&1 ;;
    profdirect) timeout -k 10 $LIM bash tools/prof_direct.sh > $log 2>&1 ;;
    run) timeout -k 10 $LIM bash -c "$arg" > $log 2>&1 ;;
    *) echo "unknown step $s" >> $O/status; exit 2 ;;
  esac
  rc=$?
  echo "$i $s rc=$rc" >> $O/status
  tail -3 $log
  if [ $rc -ne 0 ] && ! { [ $name = tests ] && [ $rc -eq 1 ]; }; then
    cat $O/status
    exit $rc
  fi
done
cat $O/status
