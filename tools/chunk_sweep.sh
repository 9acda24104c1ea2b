#!/bin/bash
# In-bench A/B of the scoring chunk size (pairs per ResNet chunk): one bench line per size, interleaved twice.
# usage (GPU box): bash tools/chunk_sweep.sh "625 834 770" > gpurun_out/chunk_sweep.log
set -o pipefail
sizes=${1:-"625 834"}
mkdir -p gpurun_out
for rep in 1 2; do
  for c in $sizes; do
    timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-companions --no-audit \
      --no-profile --chunk $c $EXTRA > gpurun_out/chunk_$c.json 2> gpurun_out/chunk_$c.err || { echo "chunk $c failed rc=$?"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('chunk', sys.argv[2], 'rep', sys.argv[3], d['value'], 'utt/s', d['ms_per_step'], 'ms')" gpurun_out/chunk_$c.json $c $rep
  done
done
