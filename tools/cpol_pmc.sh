#!/bin/bash
# PMC passes of tools/bin/cpol_bench per cache policy (developer tool).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/cpol
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/bin/cpol_bench > $OUT/times.log 2>&1
for aux in 0 2 17 19; do
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $OUT/rd$aux -o pmc --output-format csv -- $R/tools/bin/cpol_bench $aux > $OUT/rd$aux.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $OUT/wr$aux -o pmc --output-format csv -- $R/tools/bin/cpol_bench $aux > $OUT/wr$aux.log 2>&1
done
