#!/bin/bash
# xcd_rotate A/B: per-channel skew of the x-face pack (PMC) and the two-launch step (tune_sweep).
set -e
bash tools/pmc_channels.sh gpurun_out/pmcch4 516 "" xcd_rotate=1 xcd_rotate=2 "xcd_rotate=2,small_tile_rows=2048" "xcd_rotate=2,small_tile_rows=1024"
timeout -k 10 200 python tools/tune_sweep.py --configs '[{}, {"xcd_rotate": 2}, {"xcd_rotate": 2, "small_tile_rows": 2048}, {}, {"xcd_rotate": 2}]' > gpurun_out/rot_sweep2.jsonl 2>/dev/null
