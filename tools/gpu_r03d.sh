#!/bin/bash
# r03d: one rank of the keyword-sharded path on its own GPU (C4: 12 500 of 100k over 8; C3: 1 250 of 10k over 8),
# then C5 at its stated audio length (30 min per rank, long-form seek loop + LEF 10k spotting per window)
mkdir -p gpurun_out
for K in 12500 1250; do
  timeout -k 10 300 python3 -u bench.py --mode kwshard --keywords $K --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03d_ks$K.json 2> gpurun_out/r03d_ks$K.err; s=$?
  echo "ks$K=$s"; python3 -c "import json,sys; d=json.loads(open('gpurun_out/r03d_ks$K.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['per_rank'], d['audit_flips'], d['roofline']['frac'])"; [ $s -eq 0 ] || { tail -20 gpurun_out/r03d_ks$K.err; exit $s; }
done
timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 1800 --steps 1 --warmup 1 > gpurun_out/r03d_lf1800.json 2> gpurun_out/r03d_lf1800.err; s=$?
echo "lf=$s"; cat gpurun_out/r03d_lf1800.json; tail -3 gpurun_out/r03d_lf1800.err; exit $s
