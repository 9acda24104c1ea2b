#!/bin/bash
# A/B of the early-stage sub-chunk schedule (CBW_SUBCHUNK pairs per slice, stages <= CBW_SUBCHUNK_STAGES)
mkdir -p gpurun_out/sub
for r in 1 2; do
  for cfg in "0 2" "64 2" "128 2" "208 2" "128 1" "312 2"; do
    set -- $cfg
    CBW_SUBCHUNK=$1 CBW_SUBCHUNK_STAGES=$2 timeout -k 10 300 python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/sub/s$1_$2_$r.json 2> gpurun_out/sub/s$1_$2_$r.err || { echo "sub $1 $2 failed"; tail -5 gpurun_out/sub/s$1_$2_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sub/s$1_$2_$r.json').read().strip().splitlines()[-1]); print('sub=$1 stages=$2 r$r', d['value'], d['ms_per_step'], d['breakdown_ms']['kws_score'], d['breakdown_ms']['band_rescore'], d['spotted_digest'])"
  done
done
