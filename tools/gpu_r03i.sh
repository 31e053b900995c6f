#!/bin/bash
# round-3 profiles part 1: rocprofv3 kernel traces of the bench (H=2 defaults, H=1/3)
mkdir -p gpurun_out/r03i
SKIP_PMC=1 timeout -k 10 900 bash tools/profile_round.sh r03; echo "profile rc=$?" >> gpurun_out/r03i/status
cat gpurun_out/r03i/status
