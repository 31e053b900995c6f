#!/bin/bash
# tools/bin/sector_bench timings + write-request counters (developer tool).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sector
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/bin/sector_bench > $OUT/times.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d $OUT/wr -o pmc --output-format csv -- $R/tools/bin/sector_bench > $OUT/wr.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $OUT/rd -o pmc --output-format csv -- $R/tools/bin/sector_bench > $OUT/rd.log 2>&1
