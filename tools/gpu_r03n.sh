#!/bin/bash
# r03n (session re-entry): smoke + full GPU suite on HEAD, stage-3 image-bottleneck A/B in the bench
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03n_smoke.log 2>&1; s=$?
echo "smoke=$s"; tail -1 gpurun_out/r03n_smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r03n_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03n_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for M in 1 0; do
  CBW_BT3=$M timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-companions > gpurun_out/r03n_bench$M.json 2> gpurun_out/r03n_bench$M.err; s=$?
  echo "bench$M=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03n_bench$M.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03n_bench$M.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['audit_flips'], d['spotted_digest'], d['roofline']['frac'])"
done
