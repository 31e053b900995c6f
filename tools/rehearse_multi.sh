#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2, 4 and 8 ranks, all on cuda:0, gloo +
# host-staged transport (RCCL refuses two ranks on one GPU). Checks the decomposition, planning,
# mixed/unfused dispatch, verification, timing and JSON of the N>1 line; its numbers are not
# the metric. Usage: bash tools/rehearse_multi.sh <out-dir>
set -e
OUT=${1:-gpurun_out/rehearse}
mkdir -p $OUT
timeout -k 10 120 python bench.py --no-cpu-baseline > $OUT/n1.json 2> $OUT/n1.err
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --rehearse \
    --steps 50 --warmup 5 > $OUT/n$n.json 2> $OUT/n$n.err
done
echo done > $OUT/DONE
