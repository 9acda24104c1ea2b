#!/bin/bash
# r04g: end-of-round validation on the round's final library -- the whole GPU suite, smoke(), the driver's default
# bench command (with its CPU baseline and companions), and the kernel trace + roofline of a 3-step bench
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
O=gpurun_out/r04g
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; s=$?
echo "tests=$s"; tail -4 $O/gpu_tests.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; s=$?
echo "smoke=$s"; tail -3 $O/smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err; s=$?
echo "bench=$s"; [ $s -eq 0 ] || { tail -20 $O/bench.err; exit $s; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['audit_flips'], json.dumps(d.get('fp8_first_mode')), json.dumps({k: (v or {}).get('value') for k, v in (d.get('configs_companion') or {}).items()}))"
BA="--steps 3 --warmup 1 --no-cpu-baseline --no-companions"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u bench.py $BA --prof-dump $O/dump_trace.json > $O/trace.log 2>&1; s=$?
echo "trace=$s"; tail -2 $O/trace.log; [ $s -eq 0 ] || exit $s
python3 tools/roofline_from_trace.py $O/trace --dump $O/dump_trace.json --out $O/roofline.json > /dev/null; s=$?
echo "roofline=$s"; head -24 $O/roofline.json
