# bench.py A/B over one environment variable: VAR=name VALS="0 1" [ROUNDS=2]; prints value, ms/step, breakdown per run
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/ab/${VAR}_${v}_$r.json 2> gpurun_out/ab/${VAR}_${v}_$r.err || { echo "$VAR=$v failed"; tail -5 gpurun_out/ab/${VAR}_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/${VAR}_${v}_$r.json').read().strip().splitlines()[-1]); print('$VAR=$v r$r', d['value'], d['ms_per_step'], d['breakdown_ms']['kws_score'], d['breakdown_ms']['band_rescore'], d.get('roofline', {}).get('achieved'))"
  done
done
