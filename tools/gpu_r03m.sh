#!/bin/bash
# round-3 checkpoint m: the headline's start-up cost at the driver's K=20 — hipGraph of 20 steps
# (default), eager launches, one graph per step, and K=200 for reference
O=gpurun_out/r03m; mkdir -p $O
B="python bench.py --no-extras --no-cpu-baseline --no-cold"
for v in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-graph" "--steps 20 --warmup 5 --steps-per-graph 1" "--steps 200 --warmup 20" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-graph"; do
  timeout -k 10 200 $B $v > $O/tmp.json 2> $O/err.log || { echo "failed: $v" >> $O/status; exit 1; }
  python -c "
import json,sys; d=json.load(open('$O/tmp.json')); r=d['roofline']
print(json.dumps({'args': '$v', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'step_device_us': r['step_device_us'], 'launch': d['config']['launch']}))" >> $O/bubble.jsonl
done
cat $O/bubble.jsonl
