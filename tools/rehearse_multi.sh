#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2, 4 and 8 ranks, all on cuda:0, gloo +
# host-staged transport (RCCL refuses two ranks on one GPU). Checks the decomposition, planning,
# dispatch, verification, the pipelined exchange (host-staged form), timing and JSON of the N>1
# line; its numbers are not the metric. n=2 and 4 go through bench.py's own spawning (no
# torchrun, as `python bench.py --gpus N`), n=8 through torch.distributed.run as the driver
# launches it. Usage: bash tools/rehearse_multi.sh <out-dir>
set -e
OUT=${1:-gpurun_out/rehearse}
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --rehearse --steps 50 --warmup 5 \
    > $OUT/n$n.json 2> $OUT/n$n.err
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --rehearse \
  --steps 50 --warmup 5 > $OUT/n8.json 2> $OUT/n8.err
echo done > $OUT/DONE
