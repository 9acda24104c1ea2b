# compensated-tier chunk sweep: bench.py's band_rescore per CBW_X3_CHUNK value
mkdir -p gpurun_out/x3c
for c in ${CHUNKS:-128 256 512 1024}; do
  CBW_X3_CHUNK=$c timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/x3c/c$c.json 2> gpurun_out/x3c/c$c.err || { echo "chunk $c failed"; tail -5 gpurun_out/x3c/c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/x3c/c$c.json').read().strip().splitlines()[-1]); print($c, d['value'], d['ms_per_step'], d['breakdown_ms'])"
done
