#!/bin/bash
# round-3 profiles part 2: PMC passes (one counter group per pass) at halo 1/2/3
mkdir -p gpurun_out/r03j
PMC_ONLY=1 timeout -k 10 1000 bash tools/profile_round.sh r03; echo "pmc rc=$?" >> gpurun_out/r03j/status
cat gpurun_out/r03j/status
