#!/bin/bash
# r03aj: the 16-row fc2 with its rows staged in two K halves (CBW_GEMV_KS2, default 1): bit-exactness of the batched step,
# the batched long-form bench test once (faulthandler on), then the 15-row step with KS2 0 / 1 and fc2 on CPW 2
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decoder.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "step_rows or window_batcher" > gpurun_out/r03aj_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03aj_tests.log | tail -8; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bench_modes.py -m gpu -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "batched_windows" > gpurun_out/r03aj_bench_tests.log 2>&1; s=$?
echo "bench test=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03aj_bench_tests.log | tail -4
for v in "CBW_GEMV_KS2=0" "CBW_GEMV_KS2=1" "CBW_GEMV_CPW1=0"; do
  env $v timeout -k 10 200 python3 -u tools/decode_rows_bench.py large-v3 64 0,2,3 > gpurun_out/r03aj_rows_$v.txt 2>&1 || exit $?
  echo "$v"; grep step gpurun_out/r03aj_rows_$v.txt
done
