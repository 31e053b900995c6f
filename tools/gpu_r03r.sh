#!/bin/bash
# round-3 checkpoint r: short-row tile size, graph-timed two-launch step (bench.py) at halo 1/2/3
O=gpurun_out/r03r; mkdir -p $O
for rep in 1 2; do
for h in 1 3 2; do
  for t in 512 1024 2048 4096; do
    timeout -k 10 120 python bench.py --halo $h --steps 200 --warmup 20 --no-extras --no-cpu-baseline --no-cold --tune small_tile_rows=$t > $O/tmp.json 2>/dev/null || { echo "fail h$h t$t" >> $O/status; exit 1; }
    python -c "
import json; d=json.load(open('$O/tmp.json')); r=d['roofline']
print(json.dumps({'rep': $rep, 'halo': $h, 'small_tile_rows': $t, 'value': d['value'], 'step_us': r['step_device_us'], 'pack_us': r['pack_kernel_us'], 'unpack_us': r['unpack_kernel_us']}))" >> $O/sweep.jsonl
  done
done
done
cat $O/sweep.jsonl
