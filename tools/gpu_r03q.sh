#!/bin/bash
# r03q: decode-step GEMV rework (activation rows by LDS-DMA, fifth-wave next-weight L2 prefetch) -- decoder GPU tests,
# step timing A/B (CBW_DEC_PF 0 / 1, alternating), kernel trace with the prefetch on
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03q_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for PF in 0 1 0 1; do
  CBW_DEC_PF=$PF timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03q_dec$PF.log 2>&1; s=$?
  echo "dec PF=$PF rc=$s"; tail -1 gpurun_out/r03q_dec$PF.log; [ $s -eq 0 ] || exit $s
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03q_decprof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03q_decprof.log 2>&1; s=$?
echo "decprof=$s"; exit $s
