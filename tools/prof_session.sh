#!/bin/bash
# Profiling session on the GPU box: per-layer conv timings, rocprofv3 kernel-trace stats of bench.py,
# and two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for the roofline traffic figure.
# usage: tools/prof_session.sh TAG [layers] [trace] [pmc]
TAG=$1; shift
mkdir -p gpurun_out
ARGS=" $* "
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [[ "$ARGS" == *" layers "* ]]; then
  LB_MODES=${LB_MODES:-1} timeout -k 10 300 python tools/layer_bench.py > gpurun_out/layers_${TAG}.log 2>&1; s=$?
  echo "layers=$s"; cat gpurun_out/layers_${TAG}.log | grep -v amdgpu.ids
  [ $s -eq 0 ] || exit $s
fi
if [[ "$ARGS" == *" trace "* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_${TAG}_bench.log 2>&1; s=$?
  echo "trace=$s"; tail -2 gpurun_out/prof_${TAG}_bench.log
  [ $s -eq 0 ] || exit $s
fi
if [[ "$ARGS" == *" pmc "* ]]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} > gpurun_out/pmc_${TAG}_$C.log 2>&1; s=$?
    echo "pmc $C=$s"; tail -2 gpurun_out/pmc_${TAG}_$C.log
    [ $s -eq 0 ] || exit $s
  done
fi
find gpurun_out -newer tools/prof_session.sh -name "*.csv" | head -20
