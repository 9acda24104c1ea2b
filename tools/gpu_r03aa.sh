#!/bin/bash
# r03aa: Infinity-Cache warm-up of the next decoder layer on a side stream (CBW_DEC_MALL) -- decoder tests, step A/B,
# long-form 300 s at 1 and 4 lanes with the better setting
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "knobs or slice or split_key or beam" > gpurun_out/r03aa_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03aa_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for M in 0 1 0 1; do
  CBW_DEC_MALL=$M timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03aa_dec$M.log 2>&1; s=$?
  echo "dec MALL=$M rc=$s"; tail -1 gpurun_out/r03aa_dec$M.log; [ $s -eq 0 ] || exit $s
done
for A in 1 4; do
  CBW_DEC_MALL=1 timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight $A > gpurun_out/r03aa_lf$A.json 2> gpurun_out/r03aa_lf$A.err; s=$?
  echo "lf$A=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03aa_lf$A.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03aa_lf$A.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'])"
done
