#!/bin/bash
# kernel stats of the fused similarity+stem vs the separate kernels (single scoring stream, no overlap)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1; do
  CBW_SIM_FUSION=$v CBW_KWS_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/simstem$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-x3-overlap --no-pipeline > $R/gpurun_out/simstem$v.log 2>&1
done
