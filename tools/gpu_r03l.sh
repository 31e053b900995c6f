#!/bin/bash
# round-3 checkpoint l: request occupancy per row class at halo 1/2/3 (tools/pmc_credit.sh)
mkdir -p gpurun_out/r03l
timeout -k 10 900 bash tools/pmc_credit.sh gpurun_out/r03l/credit; echo "credit rc=$?" >> gpurun_out/r03l/status
cat gpurun_out/r03l/status
