# tests, then band statistics, then the bench (each step time-limited; stop at the first crash)
mkdir -p gpurun_out
T="${TESTS:-tests/test_gpu_exact.py tests/test_gpu_kernels.py}"
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T -p no:cacheprovider > gpurun_out/tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAIL|ERROR|passed|failed|x3 tier" gpurun_out/tests.log | tail -20
if [ $s -ne 0 ]; then tail -40 gpurun_out/tests.log; exit $s; fi
if [ -n "$BAND" ]; then
  timeout -k 10 400 python -u tools/band_stats.py > gpurun_out/band_stats.json 2> gpurun_out/band_stats.err; s=$?
  echo "band=$s"; cat gpurun_out/band_stats.json
  [ $s -eq 0 ] || exit $s
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err; s=$?
  echo "bench=$s"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
fi
