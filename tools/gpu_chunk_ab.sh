# bench.py over --chunk values (two rounds, interleaved)
mkdir -p gpurun_out/cab
for r in 1 2; do for c in ${CHUNKS:-625 910 1250}; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --chunk $c > gpurun_out/cab/c$c.json 2> gpurun_out/cab/c$c.err || { echo "chunk $c failed"; tail -3 gpurun_out/cab/c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cab/c$c.json').read().strip().splitlines()[-1]); print('chunk $c r$r', d['value'], d['ms_per_step'], d['breakdown_ms']['kws_score'])"
done; done
