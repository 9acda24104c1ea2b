#!/bin/bash
# One GPU session: gpu tests, then (only if nothing crashed) bench + optional rocprof.
# usage: tools/gpu_session.sh [tests] [bench] [prof] [smoke]
mkdir -p gpurun_out
want() { [[ " $* " == *" $1 "* ]]; }
ARGS=" $* "
ok_status() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 pass, 1 test failures; anything else = crash/timeout
if [[ "$ARGS" == *" smoke "* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; s=$?
  echo "smoke=$s"; tail -3 gpurun_out/smoke.log
  [ $s -eq 0 ] || exit $s
fi
if [[ "$ARGS" == *" tests "* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; s=$?
  echo "tests=$s"; tail -25 gpurun_out/gpu_tests.log
  ok_status $s || exit $s
fi
if [[ "$ARGS" == *" bench "* ]]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2> gpurun_out/bench.err; s=$?
  echo "bench=$s"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.log
  [ $s -eq 0 ] || exit $s
fi
if [[ "$ARGS" == *" prof "* ]]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1; s=$?
  echo "prof=$s"; tail -3 gpurun_out/prof_bench.log
  find gpurun_out/prof -name "*stats*" | head
fi
