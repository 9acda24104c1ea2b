#!/bin/bash
# r03ad: GEMV LayerNorm prologue staged through LDS (bit-exact vs the register prologue, decode step A/B), then the
# long-form lane-priority A/B (r03ac: its box was lost before starting)
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decoder.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03ad_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03ad_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for i in 1 2; do
  for L in 0 1; do
    CBW_GEMV_LDSLN=$L timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03ad_dec_ldsln$L.log 2>&1; s=$?
    echo "dec ldsln=$L rc=$s"; tail -1 gpurun_out/r03ad_dec_ldsln$L.log; [ $s -eq 0 ] || exit $s
  done
done
for P in --no-lane-priority --lane-priority; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight 4 $P > gpurun_out/r03ad_lf300$P.json 2> gpurun_out/r03ad_lf300$P.err; s=$?
  echo "lf300$P=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03ad_lf300$P.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03ad_lf300$P.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'], d['transcript_digests'])"
done
