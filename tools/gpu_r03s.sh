#!/bin/bash
# round-3 checkpoint s: short-row tile size across cube sizes and halo widths (graph-timed step)
O=gpurun_out/r03s; mkdir -p $O
for n in 256 384 640 512; do
for h in 1 2 3; do
  for t in 1024 2048 3072 4096; do
    timeout -k 10 120 python bench.py --N $n --halo $h --steps 200 --warmup 20 --no-extras --no-cpu-baseline --no-cold --tune small_tile_rows=$t > $O/tmp.json 2>/dev/null || { echo "fail n$n h$h t$t" >> $O/status; exit 1; }
    python -c "
import json; d=json.load(open('$O/tmp.json')); r=d['roofline']
print(json.dumps({'N': $n, 'halo': $h, 'small_tile_rows': $t, 'value': d['value'], 'step_us': r['step_device_us'], 'pack_us': r['pack_kernel_us'], 'unpack_us': r['unpack_kernel_us']}))" >> $O/sweep.jsonl
  done
done
done
cat $O/sweep.jsonl
