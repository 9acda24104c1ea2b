#!/bin/bash
# r03s: split attention P.V summed in LDS (CBW_DEC_PVL) -- decoder GPU tests, step timing A/B, kernel trace
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03s_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03s_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for PV in 0 1 0 1; do
  CBW_DEC_PVL=$PV timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03s_dec$PV.log 2>&1; s=$?
  echo "dec PVL=$PV rc=$s"; tail -1 gpurun_out/r03s_dec$PV.log; [ $s -eq 0 ] || exit $s
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03s_decprof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03s_decprof.log 2>&1; s=$?
echo "decprof=$s"; [ $s -eq 0 ] || exit $s
cd $GRAFT_REPO_ROOT
for A in 6 8; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight $A > gpurun_out/r03s_lf$A.json 2> gpurun_out/r03s_lf$A.err; s=$?
  echo "lf$A=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03s_lf$A.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03s_lf$A.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'])"
done
