#!/bin/bash
# Paired bench.py runs for an env knob: VAR=NAME tools/ab_bench.sh VAL_A VAL_B [rounds]
mkdir -p gpurun_out
A=$1; B=$2; R=${3:-2}
for r in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/abb_$v.log 2> gpurun_out/abb_err.log || { tail -5 gpurun_out/abb_err.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abb_$v.log').read().strip().splitlines()[-1]); print('$VAR=$v', d['value'], d['ms_per_step'])"
  done
done
