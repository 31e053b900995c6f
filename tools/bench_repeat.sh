#!/bin/bash
# Run-to-run spread of the headline at the driver's settings and at the defaults (no extras, no
# cold legs), plus halo 1 and 3. Usage on the GPU box: bash tools/bench_repeat.sh <out-dir>
set -e
OUT=${1:-gpurun_out/repeat}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extras --no-cold --no-cpu-baseline >> $OUT/h2_20_5.jsonl
done
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-extras --no-cold --no-cpu-baseline >> $OUT/h2.jsonl
done
for h in 1 3; do
  timeout -k 10 120 python bench.py --no-extras --no-cold --no-cpu-baseline --halo $h >> $OUT/h$h.jsonl
done
echo done > $OUT/DONE
