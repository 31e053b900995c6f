#!/bin/bash
# round-3 checkpoint w: cube-size sweep at H=2 with the automatic short-row tiles (graph-timed
# two-launch step and the fused self launch)
O=gpurun_out/r03w; mkdir -p $O
for n in 128 256 384 512 640 768 1024; do
  timeout -k 10 180 python bench.py --N $n --halo 2 --steps 200 --warmup 20 --no-extras --no-cpu-baseline --no-cold > $O/tmp.json 2>/dev/null || { echo "fail n$n" >> $O/status; exit 1; }
  python -c "
import json; d=json.load(open('$O/tmp.json')); r=d['roofline']
print(json.dumps({'N': $n, 'value': d['value'], 'step_us': r['step_device_us'], 'pack_us': r['pack_kernel_us'], 'unpack_us': r['unpack_kernel_us'], 'pack_frac': r['frac'], 'fused_us': d.get('fused_self', {}).get('launch_us'), 'verified': d['verified']}))" >> $O/sizes.jsonl
done
cat $O/sizes.jsonl
