#!/bin/bash
# Developer reproducer driver (not product): W processes of tools/bin/ipc_repro on GPU 0 sharing
# one shm block; prints each rank's line. Usage: bash tools/ipc_repro.sh [W] [MiB] [teardown 0|1] [inbox 0|1]
W=${1:-4}; MIB=${2:-136}; TD=${3:-1}; INBOX=${4:-0}
B=$(dirname "$0")/bin/ipc_repro
NAME=/ghx_ipc_repro_$$
$B init $NAME || exit 1
pids=()
for ((r = 0; r < W; r++)); do
  timeout -k 5 60 $B $W $r $MIB $TD $NAME $INBOX &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
$B unlink $NAME
exit $rc
