#!/bin/bash
# r03ai: HEAD validation after the GEMV column-group change (CG 1 default): the whole GPU suite, smoke, the bench;
# then the 15-row step with fc2 on two columns per wave (CBW_GEMV_CPW1=0)
mkdir -p gpurun_out
timeout -k 10 120 python3 -m pytest tests/test_host.py -q -p no:cacheprovider -k "matches_sources or exports" > gpurun_out/r03ai_host.log 2>&1 || { cat gpurun_out/r03ai_host.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ai_gpu_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/r03ai_gpu_tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ai_smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03ai_bench.json 2> gpurun_out/r03ai_bench.err || exit $?
tail -1 gpurun_out/r03ai_bench.json | cut -c1-400
CBW_GEMV_CPW1=0 timeout -k 10 200 python3 -u tools/decode_rows_bench.py large-v3 64 2,3 > gpurun_out/r03ai_rows_cpw2.txt 2>&1 || exit $?
grep step gpurun_out/r03ai_rows_cpw2.txt
