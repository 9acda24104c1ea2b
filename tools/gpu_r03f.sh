#!/bin/bash
# r03f: kernel trace of the fp8-first bench (realistic point), one rank of the keyword-sharded path (C4 / C3 shares),
# C5 at its stated audio length
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_r03f -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-audit --fp8-first --operating-point realistic > gpurun_out/r03f_trace.log 2>&1; s=$?
echo "trace=$s"; tail -1 gpurun_out/r03f_trace.log; [ $s -eq 0 ] || exit $s
for K in 12500 1250; do
  timeout -k 10 300 python3 -u bench.py --mode kwshard --keywords $K --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03d_ks$K.json 2> gpurun_out/r03d_ks$K.err; s=$?
  echo "ks$K=$s"; [ $s -eq 0 ] || { tail -20 gpurun_out/r03d_ks$K.err; exit $s; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r03d_ks$K.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['per_rank'], d['audit_flips'], d['roofline']['frac'])"
done
timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 1800 --steps 1 --warmup 1 > gpurun_out/r03d_lf1800.json 2> gpurun_out/r03d_lf1800.err; s=$?
echo "lf=$s"; cat gpurun_out/r03d_lf1800.json; tail -3 gpurun_out/r03d_lf1800.err; exit $s
