#!/bin/bash
# A/B session: per-layer conv timings for two settings of an env knob, then the GPU kernel tests.
# usage: LB_VAR=CBW_CONV_RING LB_MODES=0,1 tools/gpu_ab.sh TAG [tests]
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python tools/layer_bench.py > gpurun_out/ab_${TAG}.log 2>&1; s=$?
grep -v amdgpu.ids gpurun_out/ab_${TAG}.log; [ $s -eq 0 ] || exit $s
if [[ " $* " == *" tests "* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_${TAG}_tests.log 2>&1; s=$?
  tail -15 gpurun_out/ab_${TAG}_tests.log; exit $s
fi
