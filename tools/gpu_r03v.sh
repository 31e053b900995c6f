#!/bin/bash
# round-3 checkpoint v: 16-B vectors with unaligned field accesses (field_unaligned16) A/B on the
# bench line (H=1/3 legs, config 4), two interleaved repeats
O=gpurun_out/r03v; mkdir -p $O
for rep in 1 2; do for u in 0 1; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-cold --no-layout --tune field_unaligned16=$u > $O/b_${rep}_$u.json 2> $O/err.log || { echo "fail $rep $u" >> $O/status; exit 1; }
  python -c "
import json; d=json.load(open('$O/b_${rep}_$u.json')); h=d['halo_widths']; c=d['extra_configs']['config4_5fields_256^3_h3_f64f32']
print(json.dumps({'rep': $rep, 'u16': $u, 'h2': d['value'], 'h1': h['1']['value'], 'h1_pack': h['1']['pack_kernel_us'], 'h1_unpack': h['1']['unpack_kernel_us'], 'h3': h['3']['value'], 'h3_pack': h['3']['pack_kernel_us'], 'h3_unpack': h['3']['unpack_kernel_us'], 'cfg4': c['GBps'], 'cfg4_fused_us': c['fused_self']['us_per_exchange'], 'fused_h2': d['fused_self']['launch_us'], 'h1_ok': h['1']['verified'], 'h3_ok': h['3']['verified'], 'cfg4_ok': c['verified']}))" >> $O/ab.jsonl
done; done
cat $O/ab.jsonl
