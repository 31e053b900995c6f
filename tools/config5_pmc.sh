#!/bin/bash
# PMC passes over tools/config5_probe.py (config 5's index-list gather/scatter, levels 1 and 8)
# and over tools/microbench.py at halo 1 (the 512^3 pack split by row class), one counter group
# per pass, kernel trace only, each pass under its own time limit. Usage: config5_pmc.sh <out>
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GROUPS_=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
         "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE"
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum"
         "TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_WRITE_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum")
for lv in 1 8; do
  timeout -k 10 120 python3 $R/tools/config5_probe.py --levels $lv --time > $OUT/time_l$lv.json
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1)); mkdir -p $OUT/l$lv
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $OUT/l$lv/p$i -o pmc --output-format csv -- python3 $R/tools/config5_probe.py --levels $lv --iters 6 > $OUT/l$lv/p$i.log 2>&1 || { echo "pmc l$lv p$i failed" >> $OUT/status; exit 1; }
  done
done
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1)); mkdir -p $OUT/h1
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/h1/p$i -o pmc --output-format csv -- python3 $R/tools/microbench.py --halo 1 --iters 6 > $OUT/h1/p$i.log 2>&1 || { echo "pmc h1 p$i failed" >> $OUT/status; exit 1; }
done
echo done > $OUT/DONE
