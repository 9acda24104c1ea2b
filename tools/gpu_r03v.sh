#!/bin/bash
# r03v: decode attention / combine / timestamp-rule kernels with their loads in flight together -- decoder GPU tests,
# step timing, kernel trace, long-form 300 s at 1 and 4 audios in flight
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03v_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03v_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for i in 1 2; do
  timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03v_dec.log 2>&1; s=$?
  echo "dec rc=$s"; tail -1 gpurun_out/r03v_dec.log; [ $s -eq 0 ] || exit $s
done
for A in 1 4; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight $A > gpurun_out/r03v_lf$A.json 2> gpurun_out/r03v_lf$A.err; s=$?
  echo "lf$A=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03v_lf$A.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03v_lf$A.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03v_decprof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03v_decprof.log 2>&1; s=$?
echo "decprof=$s"; exit $s
