#!/bin/bash
# r03al: eight computing waves per workgroup for the 9..16-row decode GEMVs (CBW_GEMV_W8, default 1): bit-exactness of
# the batched step (every knob), the batcher, then the step at 5 / 10 / 15 rows with W8 0 / 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decoder.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "step_rows or window_batcher" > gpurun_out/r03al_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03al_tests.log | tail -8; [ $s -eq 0 ] || exit $s
for v in "CBW_GEMV_W8=0" "CBW_GEMV_W8=1"; do
  env $v timeout -k 10 200 python3 -u tools/decode_rows_bench.py large-v3 64 0,2,3 > gpurun_out/r03al_rows_$v.txt 2>&1 || exit $?
  echo "$v"; grep step gpurun_out/r03al_rows_$v.txt
done
