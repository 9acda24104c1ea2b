#!/bin/bash
# r03ae: C5 after the decoder work -- 1800 s audios, 4 in flight: realistic point fp8-first, and the synthetic point
mkdir -p gpurun_out
for OP in realistic synthetic; do
  F=$([ "$OP" = realistic ] && echo --fp8-first || echo "")
  timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 1800 --steps 1 --warmup 1 --audios-in-flight 4 --operating-point $OP $F > gpurun_out/r03ae_lf1800_$OP.json 2> gpurun_out/r03ae_lf1800_$OP.err; s=$?
  echo "lf1800_$OP=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03ae_lf1800_$OP.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03ae_lf1800_$OP.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'], d['spotted_keywords_per_window'], d['dtype'])"
done
