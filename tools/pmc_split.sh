#!/bin/bash
# PMC passes over tools/microbench.py (each iteration-space class of the 512^3 plan as its own
# launch: short rows / long rows / all, pack and unpack), one counter group per pass, kernel
# trace only. Rows are told apart by their grid (workgroup count). Usage: tools/pmc_split.sh <out>
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o pmc --output-format csv -- python3 $R/tools/microbench.py --iters 10 "$@" > $OUT/p$i.log 2>&1
done
echo done > $OUT/DONE
