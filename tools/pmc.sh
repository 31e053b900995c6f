#!/bin/bash
# Collect HBM/L2 counters for the bench's pack/unpack kernels, one rocprofv3 --pmc pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel-trace only.
# Usage: tools/pmc.sh <outdir> [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o pmc --output-format csv -- python3 $R/bench.py --no-graph --no-extras --no-cpu-baseline --no-cold "$@" > $OUT/p$i.log 2>&1
done
