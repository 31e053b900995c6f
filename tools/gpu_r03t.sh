#!/bin/bash
# round-3 checkpoint t: automatic short-row tile rows vs the fixed choices (graph-timed step and
# the fused self launch), N = 256..640, H = 1..3
O=gpurun_out/r03t; mkdir -p $O
run() {  # n h tune-label tune-arg
  timeout -k 10 120 python bench.py --N $1 --halo $2 --steps 200 --warmup 20 --no-extras --no-cpu-baseline --no-cold $4 > $O/tmp.json 2>/dev/null || { echo "fail $*" >> $O/status; exit 1; }
  python -c "
import json; d=json.load(open('$O/tmp.json')); r=d['roofline']
print(json.dumps({'N': $1, 'halo': $2, 'tile_rows': '$3', 'value': d['value'], 'step_us': r['step_device_us'], 'pack_us': r['pack_kernel_us'], 'unpack_us': r['unpack_kernel_us'], 'fused_us': d.get('fused_self', {}).get('launch_us')}))" >> $O/sweep.jsonl
}
for n in 256 384 512 640; do for h in 1 2 3; do
  run $n $h auto ""
  run $n $h 4096 "--tune small_tile_rows=4096"
done; done
for n in 320 448; do for h in 1 2 3; do
  run $n $h auto ""
  for t in 512 1024 2048 4096; do run $n $h $t "--tune small_tile_rows=$t"; done
done; done
cat $O/sweep.jsonl
