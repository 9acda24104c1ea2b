#!/bin/bash
# r03p: long-form audios in flight per GPU (3, 4 lanes at 300 s), then 1800 s audios (C5's length) at 1 and the best lanes
mkdir -p gpurun_out
for A in 3 4; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight $A > gpurun_out/r03p_lf$A.json 2> gpurun_out/r03p_lf$A.err; s=$?
  echo "lf$A=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03p_lf$A.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03p_lf$A.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'])"
done
B=$(python3 -c "
import json
v={a: json.loads(open(f'gpurun_out/r03p_lf{a}.json').read().strip().splitlines()[-1])['value'] for a in (3,4)}
print(max(v, key=v.get) if max(v.values()) > 45.5 else 2)")
echo "best lanes $B"
timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 1800 --steps 1 --warmup 1 --audios-in-flight $B > gpurun_out/r03p_lf1800_$B.json 2> gpurun_out/r03p_lf1800_$B.err; s=$?
echo "lf1800=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03p_lf1800_$B.err; exit $s; }
tail -c 1500 gpurun_out/r03p_lf1800_$B.json
