#!/bin/bash
# r03a: bench audit / algorithmic frac / kwshard pipeline / api mode + the re-targeted exactness tests
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err; s=$?
echo "bench=$s"; tail -c 3000 gpurun_out/r03a_bench.json; [ $s -eq 0 ] || { tail -30 gpurun_out/r03a_bench.err; exit $s; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench_modes.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a_modes.log 2>&1; s=$?
echo "modes=$s"; tail -30 gpurun_out/r03a_modes.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench_exact.py -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a_exact.log 2>&1; s=$?
echo "exact=$s"; tail -15 gpurun_out/r03a_exact.log; exit $s
