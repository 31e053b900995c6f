#!/bin/bash
# PMC passes over tools/emu_rank_bench.py for rank 0 of the WORLD-rank decomposition (default 8:
# (2,2,2)): the fused pack/unpack of its peer buffers and, from its timeline, each peer buffer's
# own launch (told apart by grid size). Usage: tools/pmc_emu.sh <out> [world]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
W=${1:-8}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o pmc --output-format csv -- python3 $R/tools/emu_rank_bench.py $W > $OUT/p$i.log 2>&1
done
echo done > $OUT/DONE
