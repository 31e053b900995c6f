#!/bin/bash
# Per-L2-channel read requests of the x-face pack (tools/xface_probe.py): one rocprofv3 --pmc pass
# per tuning setting with the un-reduced TCC_EA0_RDREQ, JSON output (one value per TCC instance =
# (XCD, channel)); tools/parse_pmc_channels.py summarises. Usage:
#   tools/pmc_channels.sh <out> [pitches] [tune ...]      (tune: "key=v,key=v"; "" = defaults)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
P=${1:-516,518}; shift || true
[ $# -eq 0 ] && set -- ""
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for t in "$@"; do
  i=$((i+1))
  echo "$t" > $OUT/tune$i.txt
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ --kernel-trace --kernel-include-regex k_copy \
    -d $OUT/j$i -o pmc --output-format json -- python3 $R/tools/xface_probe.py --pitches $P --zs 512 --tune "$t" > $OUT/log$i 2>&1
done
echo done > $OUT/DONE
