#!/bin/bash
# r03r: bench-mode GPU tests (long-form lanes, fp8-first long-form, keyword-sharded sim), then C5 at full length:
# 1800 s audios, 4 in flight, realistic operating point, bf16-first and fp8-first spotting
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench_modes.py -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r03r_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03r_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for F in "" "--fp8-first"; do
  T=$([ -z "$F" ] && echo bf16 || echo fp8)
  timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 1800 --steps 1 --warmup 1 --audios-in-flight 4 --operating-point realistic $F > gpurun_out/r03r_lf1800_$T.json 2> gpurun_out/r03r_lf1800_$T.err; s=$?
  echo "lf1800_$T=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03r_lf1800_$T.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03r_lf1800_$T.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'], d['spotted_keywords_per_window'], d['config']['fp8_first'], d['transcript_digests'])"
done
