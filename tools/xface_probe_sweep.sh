mkdir -p gpurun_out/s10
for t in "" small_tile_rows=256 small_tile_rows=512 small_tile_rows=1024 small_tile_rows=2048 small_tile_rows=8192 unroll=8 unroll=2 "unroll=8,small_tile_rows=1024" "unroll=8,small_tile_rows=2048" "unroll=2,small_tile_rows=512" "small_tile_rows=512,nt=3"; do
  timeout -k 10 60 python tools/xface_probe.py --pitches 516 --zs 512 --tune "$t" >> gpurun_out/s10/probe.jsonl || exit 1
done
