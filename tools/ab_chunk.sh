#!/bin/bash
# Paired bench.py runs over keyword chunk sizes: tools/ab_chunk.sh "625 834 1000" [rounds]
mkdir -p gpurun_out
R=${2:-2}
for r in $(seq 1 $R); do
  for c in $1; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --chunk $c > gpurun_out/abc_$c.log 2> gpurun_out/abc_err.log || { tail -5 gpurun_out/abc_err.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abc_$c.log').read().strip().splitlines()[-1]); print('chunk=$c', d['value'], d['ms_per_step'])"
  done
done
