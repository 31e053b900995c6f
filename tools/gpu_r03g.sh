#!/bin/bash
# round-3 profiles, part 1: rocprofv3 kernel traces of the bench (H=2 defaults, H=1/3), then the
# N>1 rehearsal through bench.py (2/4 spawned, 8 via torch.distributed.run; gloo + host staging)
O=gpurun_out; mkdir -p $O/r03g
SKIP_PMC=1 timeout -k 10 700 bash tools/profile_round.sh r03; rc=$?; echo "profile rc=$rc" >> $O/r03g/status
[ $rc -ne 0 ] && exit $rc
timeout -k 10 420 bash tools/rehearse_multi.sh $O/r03g/rehearse; echo "rehearse rc=$?" >> $O/r03g/status
cat $O/r03g/status
