#!/bin/bash
# final validation: smoke, full GPU suite, bench x2, long-form
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1; s=$?
echo "smoke=$s"; tail -1 gpurun_out/smoke_f.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/final_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/final_tests.log; [ $s -eq 0 ] || exit $s
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/final_bench_$r.json 2> gpurun_out/final_bench_$r.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/final_bench_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['breakdown_ms']['kws_score'], d['breakdown_ms']['band_rescore'], d['spotted_digest'], d['roofline']['frac'])"
done
timeout -k 10 400 python3 -u bench.py --mode longform --steps 2 --warmup 1 --audio-seconds 60 > gpurun_out/lf_f.json 2> gpurun_out/lf_f.err; s=$?
echo "lf=$s"; cat gpurun_out/lf_f.json
