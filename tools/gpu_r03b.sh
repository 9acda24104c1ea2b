#!/bin/bash
# r03b: api / kwshard modes, the production-width decoder slice, the timed-clip + C4 exactness tests
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench_modes.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -k api > gpurun_out/r03b_modes.log 2>&1; s=$?
echo "modes=$s"; tail -15 gpurun_out/r03b_modes.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decoder.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k large_v3 > gpurun_out/r03b_dec.log 2>&1; s=$?
echo "dec=$s"; tail -15 gpurun_out/r03b_dec.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench_exact.py -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_exact.log 2>&1; s=$?
echo "exact=$s"; tail -15 gpurun_out/r03b_exact.log; exit $s
