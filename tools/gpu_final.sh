#!/bin/bash
# final validation, two gpurun calls (each within gpurun's 1200 s): `bash tools/gpu_final.sh tests` -- smoke() and the
# full GPU suite; `bash tools/gpu_final.sh bench` -- the driver's default bench line (every companion).  Logs under
# gpurun_out/final_*.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ "$1" = tests ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1; s=$?
  echo "smoke=$s"; tail -2 gpurun_out/final_smoke.log; [ $s -eq 0 ] || exit $s
  timeout -k 10 1080 python3 -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/final_tests.log 2>&1; s=$?
  echo "tests=$s"; grep -cE "PASSED" gpurun_out/final_tests.log; tail -3 gpurun_out/final_tests.log; exit $s
fi
if [ "$1" = bench ]; then
  timeout -k 10 900 python3 -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err; s=$?
  echo "bench=$s"; tail -2 gpurun_out/final_bench.err; [ $s -eq 0 ] || exit $s
  python3 -c "import json; d=json.loads(open('gpurun_out/final_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['audit_flips'], d['spotted_digest'], d['roofline']['frac'], d['cpu_baseline'].get('value'))"
  exit 0
fi
echo "usage: bash tools/gpu_final.sh tests|bench"; exit 2
