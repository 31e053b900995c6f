#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace summaries of the bench command and
# per-counter PMC passes, at halo 1/2/3. Results land in gpurun_out/prof_<round>/; the
# summaries to commit are written by tools/collect_profiles.py into profiles/.
# Usage: bash tools/profile_round.sh r01   (PMC_ONLY=1 / SKIP_PMC=1 split it over two calls)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
RN=${1:-r01}
OUT=$R/gpurun_out/prof_$RN
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "${PMC_ONLY:-0}" != 1 ]; then
# 1) the bench command itself (defaults: N=1, 512^3, H=2, hipGraph, extras, cpu baseline) minus
#    the cold-cache legs and the padded-layout leg, whose extra launches of the same kernels
#    (same grids) would skew the per-kernel averages
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench -o kt --output-format csv -- python3 $R/bench.py --no-cold --no-layout > $OUT/bench.log 2>&1
# 2) kernel traces at halo 1 and 3
for h in 1 3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/h$h -o kt --output-format csv -- python3 $R/bench.py --halo $h --no-extras --no-cpu-baseline --no-cold > $OUT/h$h.log 2>&1
done
fi
# 3) PMC passes (one counter group per pass, kernel trace only), eager launches: the two-launch
#    pack/unpack path at halo 1/2/3 (the fused k_self of the extras is counted too)
if [ "${SKIP_PMC:-0}" != 1 ]; then
  for h in 1 2 3; do
    bash $R/tools/pmc.sh $OUT/pmc_h$h --steps 20 --warmup 5 --halo $h
  done
fi
echo done > $OUT/DONE
