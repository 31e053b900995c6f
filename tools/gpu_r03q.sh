#!/bin/bash
# round-3 checkpoint q: short-row tile size at halo 1/2/3 against the pack's read floor
O=gpurun_out/r03q; mkdir -p $O
for h in 1 2 3; do
  for t in 256 512 1024 2048 4096; do
    timeout -k 10 60 python tools/microbench.py --halo $h --iters 50 --tune small_tile_rows=$t > $O/h${h}_t$t.json 2>/dev/null || { echo "fail h$h t$t" >> $O/status; exit 1; }
    python -c "
import json; r=json.load(open('$O/h${h}_t$t.json'))['results']
print(json.dumps({'halo': $h, 'small_tile_rows': $t, 'all_pack': r['all_pack']['us'], 'all_unpack': r['all_unpack']['us'], 'short_pack': r['short_rows_pack']['us'], 'short_unpack': r['short_rows_unpack']['us'], 'tiles': r['all_pack']['tiles']}))" >> $O/sweep.jsonl
  done
done
cat $O/sweep.jsonl
