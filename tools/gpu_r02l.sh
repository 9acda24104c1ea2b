#!/bin/bash
# short-form long-prompt test, the default bench, the long-form bench (calibrated band), a kernel-stats profile
# of one long-form audio
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoder.py -m gpu -q -x -k "shortform" -p no:cacheprovider > gpurun_out/l_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/l_tests.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err; s=$?
echo "bench=$s"; tail -2 gpurun_out/bench_l.err; cat gpurun_out/bench_l.json
[ $s -eq 0 ] || exit $s
timeout -k 10 400 python3 -u bench.py --mode longform --steps 2 --warmup 1 --audio-seconds 60 > gpurun_out/lf_l.json 2> gpurun_out/lf_l.err; s=$?
echo "lf=$s"; tail -2 gpurun_out/lf_l.err; cat gpurun_out/lf_l.json
[ $s -eq 0 ] || exit $s
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lfk -o run --output-format csv -- python3 bench.py --mode longform --steps 1 --warmup 0 --audio-seconds 60 > gpurun_out/lfk.log 2>&1; s=$?
echo "lfk=$s"; grep -v "^W20" gpurun_out/lfk.log | tail -3
[ $s -eq 0 ] || exit $s
head -25 gpurun_out/lfk/run_kernel_stats.csv | cut -d, -f1-5
