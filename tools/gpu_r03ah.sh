#!/bin/bash
# r03ah: 16-row GEMVs with two column groups per wave (CBW_GEMV_CG, default 2 at M > 8): bit-exactness of the batched
# step vs single-window steps, then the step cost at 5 / 10 / 15 rows with CG 1 vs 2
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decoder.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "step_rows or window_batcher or gemv" > gpurun_out/r03ah_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03ah_tests.log | tail -8; [ $s -eq 0 ] || exit $s
for cg in 1 2; do
  CBW_GEMV_CG=$cg timeout -k 10 200 python3 -u tools/decode_rows_bench.py large-v3 64 0,1,2,3 > gpurun_out/r03ah_rows_cg$cg.txt 2>&1 || exit $?
  echo "CG=$cg"; grep step gpurun_out/r03ah_rows_cg$cg.txt
done
