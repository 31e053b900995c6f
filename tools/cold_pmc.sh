#!/bin/bash
# Cold-vs-warm PMC passes over tools/cold_pmc.py: per mode (warm, cold_step, cold_pack,
# cold_unpack) one rocprofv3 --pmc pass per counter group, kernel trace only, each under its own
# time limit. Then the timing run without the profiler. Usage: tools/cold_pmc.sh <out> [args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/cold_pmc.py --time --iters 15 "$@" > $OUT/time.json 2> $OUT/time.err
GROUPS_=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE"
         "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum"
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum")
for m in warm cold_step cold_pack cold_unpack; do
  i=0
  mkdir -p $OUT/$m
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $OUT/$m/p$i -o pmc --output-format csv -- python3 $R/tools/cold_pmc.py --mode $m --iters 6 "$@" > $OUT/$m/p$i.log 2>&1 || { echo "pmc $m p$i failed" >> $OUT/status; exit 1; }
  done
done
echo done > $OUT/DONE
