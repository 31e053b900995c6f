#!/bin/bash
# Instruction-fetch and wave-occupancy counters of the pack / unpack launches and of the pack's
# address-set probe (tools/launch_anatomy.py), one rocprofv3 --pmc pass per group, kernel-trace
# only. Usage: tools/pmc_ifetch.sh <outdir> N H [ghx_tune k=v,...] [counter group ...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); N=$2; H=$3; TUNE=${4:-}
shift 4 2>/dev/null || shift $#
GROUPS_=("$@")
[ ${#GROUPS_[@]} -eq 0 ] && GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY" "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU")
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o pmc --output-format csv -- python3 $R/tools/launch_anatomy.py $N $H 20 "$TUNE" > $OUT/p$i.log 2>&1
done
