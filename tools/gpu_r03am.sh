#!/bin/bash
# r03am: HEAD validation (W8 default for the 9..16-row GEMVs): host checks, the whole GPU suite, smoke, the bench;
# then the 300 s long-form with 3 audios: lanes vs --batch-windows
mkdir -p gpurun_out
timeout -k 10 120 python3 -m pytest tests/test_host.py -q -p no:cacheprovider -k "matches_sources or exports" > gpurun_out/r03am_host.log 2>&1 || { cat gpurun_out/r03am_host.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03am_gpu_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/r03am_gpu_tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03am_smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03am_bench.json 2> gpurun_out/r03am_bench.err || exit $?
tail -1 gpurun_out/r03am_bench.json | cut -c1-300
for B in "" --batch-windows; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight 3 $B > gpurun_out/r03am_lf300_a3$B.json 2> gpurun_out/r03am_lf300_a3$B.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r03am_lf300_a3$B.json').read().strip().splitlines()[-1]); print('$B', d['value'], d['ms_per_window'], d.get('window_batch'), d['transcript_digests'])"
done
