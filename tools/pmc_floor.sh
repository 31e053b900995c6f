#!/bin/bash
# Counters of the unpack write-floor probes (tools/pack_floor.hip, one variant per run, warm):
# 2 = the halo pieces' writes alone, 3 = + the buffer streamed in first, 4 = + the buffer read
# interleaved with the writes. Same two passes as tools/pmc_credit.sh (requests + 64-B writes;
# LEVEL counters for latency and requests in flight), kernel trace only, each run under its own
# limit. Summarise with tools/parse_pmc_floor.py <out>. Usage: tools/pmc_floor.sh <out> [N H]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); N=${2:-512}; H=${3:-2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GROUPS_=("TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
         "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE")
for v in 2 3 4; do
  i=0
  mkdir -p $OUT/v$v
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --kernel-trace -d $OUT/v$v/p$i -o pmc --output-format csv -- $R/tools/bin/pack_floor 7 $N $H $v > $OUT/v$v/p$i.log 2>&1 || { echo "pmc v$v p$i failed" >> $OUT/status; exit 1; }
  done
done
echo done > $OUT/DONE
