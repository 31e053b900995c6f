#!/bin/bash
# Developer A/B of two builds of libghx (not product): ghex_amd/lib/libghx.so (A) against a
# variant prebuilt in the container (B, e.g. tools/lib/libghx_w8.so), interleaved A B A B, each
# run a tools/floor_sweep.py pass over SHAPES. The original library is restored on exit.
# Usage: bash tools/lib_ab.sh <variant.so> <out.jsonl> [shapes] [floor_sweep args, e.g. --tune k=v]
set -e
B=$1; OUT=$2; SHAPES=${3:-384:1,256:3,512:1,512:2,512:3,640:3}
shift 3 2>/dev/null || shift $#
EXTRA="$@"
LIB=ghex_amd/lib/libghx.so
cp $LIB /tmp/libghx_A.so
trap 'cp /tmp/libghx_A.so $LIB' EXIT
: > $OUT
for v in A B A B; do
  if [ $v = A ]; then cp /tmp/libghx_A.so $LIB; else cp $B $LIB; fi
  timeout -k 10 280 python tools/floor_sweep.py --no-floor --shapes $SHAPES $EXTRA | sed "s/^{/{\"lib\": \"$v\", /" >> $OUT
done
