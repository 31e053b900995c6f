#!/bin/bash
# round-3 checkpoint ah: the N=8 rehearsal through torchrun (all ranks on the one GPU; the
# isolated zero-copy leg skipped there, it ran at N=2/4 in r03_reh_ag), then a fuzz soak over
# seeds the suite and earlier soaks never drew. Each step under its own limit; a failure ends it.
O=gpurun_out/r03ah; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --rehearse \
  --steps 50 --warmup 5 > $O/n8.json 2> $O/n8.err; rc=$?; echo "n8 rc=$rc" >> $O/status
[ $rc -ne 0 ] && { cat $O/status; exit $rc; }
timeout -k 10 560 python -u tools/fuzz_soak.py --structured 2000:20000 --unstructured 2000:20000 \
  --seconds 480 > $O/soak.json 2> $O/soak.err; rc=$?; echo "soak rc=$rc" >> $O/status
cat $O/status; tail -c 1500 $O/soak.json
