#!/bin/bash
# Round-2 measurement session: the default bench (with the CPU baseline and the per-launch dump), then
# rocprofv3 passes (a kernel trace + stats pass and two PMC passes) whose records are cut to the timed
# region by the CLOCK_MONOTONIC bounds bench.py --prof-dump writes, and the roofline recomputed from them.  usage: tools/prof_r02.sh TAG [bench] [trace] [pmc]
TAG=$1; shift
ARGS=" $* "
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BA="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
if [[ "$ARGS" == *" bench "* ]]; then
  timeout -k 10 600 python3 -u bench.py --prof-dump gpurun_out/dump_${TAG}_bench.json ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; s=$?
  echo "bench=$s"; tail -2 gpurun_out/bench_${TAG}.err; cat gpurun_out/bench_${TAG}.json
  [ $s -eq 0 ] || exit $s
fi
if [[ "$ARGS" == *" trace "* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG} -o run --output-format csv -- python3 bench.py ${BA} --prof-dump gpurun_out/dump_${TAG}_trace.json > gpurun_out/trace_${TAG}.log 2>&1; s=$?
  echo "trace=$s"; tail -2 gpurun_out/trace_${TAG}.log
  [ $s -eq 0 ] || exit $s
fi
if [[ "$ARGS" == *" pmc "* ]]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    # (the audit runs in host-synchronised passes, bench.py --audit-pass: ~19k dispatches enqueued in one call crash the
    # profiled process under counter collection, DESIGN.md §5, profiles/r05b_pmc_f32_*)
    timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv -- python3 bench.py ${BA} --prof-dump gpurun_out/dump_${TAG}_$C.json > gpurun_out/pmc_${TAG}_$C.log 2>&1; s=$?
    echo "pmc $C=$s"; tail -2 gpurun_out/pmc_${TAG}_$C.log
    [ $s -eq 0 ] || exit $s
  done
fi
if [[ "$ARGS" == *" trace "* ]]; then
  P=""
  [[ "$ARGS" == *" pmc "* ]] && P="--fetch gpurun_out/pmc_${TAG}_FETCH_SIZE --fetch-dump gpurun_out/dump_${TAG}_FETCH_SIZE.json --write gpurun_out/pmc_${TAG}_WRITE_SIZE --write-dump gpurun_out/dump_${TAG}_WRITE_SIZE.json"
  python3 tools/roofline_from_trace.py gpurun_out/trace_${TAG} --dump gpurun_out/dump_${TAG}_trace.json $P --out gpurun_out/roofline_${TAG}.json > /dev/null; s=$?
  echo "roofline=$s"; head -30 gpurun_out/roofline_${TAG}.json
fi
