#!/bin/bash
# r03ab: fc2 (K 5120) GEMV with one column per wave (CBW_GEMV_CPW1) -- decoder tests, step A/B
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ab_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03ab_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for C in 0 1 0 1; do
  CBW_GEMV_CPW1=$C timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03ab_dec$C.log 2>&1; s=$?
  echo "dec CPW1=$C rc=$s"; tail -1 gpurun_out/r03ab_dec$C.log; [ $s -eq 0 ] || exit $s
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03ab_decprof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03ab_decprof.log 2>&1; s=$?
echo "decprof=$s"; exit $s
