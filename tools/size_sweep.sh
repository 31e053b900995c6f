#!/bin/bash
# The headline step (two launches, H=2) across cube sizes: bench lines without extras.
set -e
mkdir -p gpurun_out
for n in 128 256 384 512 640 768 1024; do
  timeout -k 10 120 python bench.py --N $n --no-extras --no-cold --no-cpu-baseline >> gpurun_out/size_sweep.jsonl 2>/dev/null
done
