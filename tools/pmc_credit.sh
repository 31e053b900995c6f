#!/bin/bash
# Read/write request occupancy of the pack/unpack launches per row class (tools/microbench.py:
# x faces, short rows, long rows, the whole plan, each as its own launch), at halo 1/2/3: one
# counter group per pass, kernel trace only, each pass under its own limit. The LEVEL counters
# accumulate the requests in flight per cycle, so LEVEL / GRBM_GUI_ACTIVE is the mean number of
# outstanding fabric requests and LEVEL / REQ the mean latency (Little's law).
# Usage: tools/pmc_credit.sh <out>
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GROUPS_=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE")
for h in 1 2 3; do
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1)); mkdir -p $OUT/h$h
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/h$h/p$i -o pmc --output-format csv -- python3 $R/tools/microbench.py --halo $h --iters 6 > $OUT/h$h/p$i.log 2>&1 || { echo "pmc h$h p$i failed" >> $OUT/status; exit 1; }
  done
  timeout -k 10 120 python3 $R/tools/microbench.py --halo $h --iters 30 > $OUT/h$h/time.json 2>&1
done
echo done > $OUT/DONE
