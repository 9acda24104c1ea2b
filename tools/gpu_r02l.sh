#!/bin/bash
# pool_fc load-parallel check (bench digest + time) and a kernel-stats profile of one long-form window
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err; s=$?
echo "bench=$s"; tail -2 gpurun_out/bench_l.err; cat gpurun_out/bench_l.json
[ $s -eq 0 ] || exit $s
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lfk -o run --output-format csv -- python3 bench.py --mode longform --steps 1 --warmup 0 --audio-seconds 30 > gpurun_out/lfk.log 2>&1; s=$?
echo "lfk=$s"; tail -2 gpurun_out/lfk.log
[ $s -eq 0 ] || exit $s
head -25 gpurun_out/lfk/run_kernel_stats.csv | cut -d, -f1-5
