#!/bin/bash
# r03ag: kernel stats of the 15-row decode step (3 windows x 5 beams) vs the 5-row step
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03ag_prof15 -o run -- python3 -u tools/decode_rows_bench.py large-v3 64 3 > gpurun_out/r03ag_prof15.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03ag_prof5 -o run -- python3 -u tools/decode_rows_bench.py large-v3 64 0 > gpurun_out/r03ag_prof5.txt 2>&1 || exit $?
cat gpurun_out/r03ag_prof15.txt gpurun_out/r03ag_prof5.txt | grep -v amdgpu.ids
