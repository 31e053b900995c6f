#!/bin/bash
# Kernel trace of the direct exchange: 2 worker processes on the one GPU, each under its own
# rocprofv3 (kernel trace + stats only), 128^3 H=2, 40 exchanges per field layout, issued back to
# back on the stream (MODE=directloop, default: the devices stay in step through the epochs; MODE=
# direct waits on the host after each exchange, so the traces also carry the host-side skew).
O=gpurun_out/prof_direct; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats -d $O/r$r -o run --output-format csv -- python3 tests/mp_exchange_worker.py 2 1 1 128 2 40 ${MODE:-directloop} \
    > $O/log$r.txt 2>&1 &
done
wait
tail -2 $O/log0.txt
python3 tools/parse_prof_direct.py $O ${MODE:-directloop} > $O/summary.json && head -c 400 $O/summary.json
