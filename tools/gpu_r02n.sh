#!/bin/bash
# full GPU suite, the default bench (side streams created as needed), the long-form bench (packed beam log)
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/n_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/n_tests.log
[ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_n.json 2> gpurun_out/bench_n.err; s=$?
echo "bench=$s"; tail -1 gpurun_out/bench_n.err; python3 -c "import json; d=json.loads(open('gpurun_out/bench_n.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['breakdown_ms'], d['spotted_digest'], d['roofline']['frac'])"
[ $s -eq 0 ] || exit $s
timeout -k 10 400 python3 -u bench.py --mode longform --steps 2 --warmup 1 --audio-seconds 60 > gpurun_out/lf_n.json 2> gpurun_out/lf_n.err; s=$?
echo "lf=$s"; tail -1 gpurun_out/lf_n.err; cat gpurun_out/lf_n.json
