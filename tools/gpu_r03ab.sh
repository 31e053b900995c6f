#!/bin/bash
# round-3 checkpoint ab: steps per hipGraph at the driver's K=20 (graph launch start-up cost)
O=gpurun_out/r03ab; mkdir -p $O
for rep in 1 2 3; do for g in 20 10 5 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --steps-per-graph $g --no-extras --no-cold --no-cpu-baseline > $O/tmp.json 2>/dev/null || { echo "fail g$g" >> $O/status; exit 1; }
  python -c "
import json; d=json.load(open('$O/tmp.json')); r=d['roofline']
print(json.dumps({'rep': $rep, 'spg': $g, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'step_device_us': r['step_device_us']}))" >> $O/spg.jsonl
done; done
cat $O/spg.jsonl
