#!/bin/bash
# r03k: VALU dot GEMV for decoder steps -- decoder/whisper GPU tests, then step timing dot vs MFMA GEMV + a trace
mkdir -p gpurun_out
CBW_GEMV_DOT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py tests/test_gpu_kernels.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03k_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03k_tests.log | tail -15; [ $s -eq 0 ] || exit $s
CBW_GEMV_DOT=0 timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 > gpurun_out/r03k_dec_mfma.log 2>&1; s=$?
echo "dec_mfma=$s"; cat gpurun_out/r03k_dec_mfma.log; [ $s -eq 0 ] || exit $s
CBW_GEMV_DOT=1 timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 > gpurun_out/r03k_dec_dot.log 2>&1; s=$?
echo "dec_dot=$s"; cat gpurun_out/r03k_dec_dot.log; [ $s -eq 0 ] || exit $s
cd /tmp && export TMPDIR=/tmp CBW_GEMV_DOT=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03k_prof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03k_prof.log 2>&1; s=$?
echo "prof=$s"; exit $s
