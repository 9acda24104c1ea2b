#!/bin/bash
# r03x: decode-step GEMV -- fast full-wave reductions (softmax, LayerNorm prologue), split attention P.V without the xor-32 step
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03x_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03x_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for i in 1 2; do
  timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03x_dec.log 2>&1; s=$?
  echo "dec rc=$s"; tail -1 gpurun_out/r03x_dec.log; [ $s -eq 0 ] || exit $s
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03x_decprof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03x_decprof.log 2>&1; s=$?
echo "decprof=$s"; exit $s
