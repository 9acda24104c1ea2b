# round-2 GPU session: targeted tests then a short bench (each step time-limited; stop at the first crash)
mkdir -p gpurun_out
T="${TESTS:-tests/test_gpu_encoder.py tests/test_gpu_exact.py tests/test_gpu_kws.py}"
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T -p no:cacheprovider > gpurun_out/tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "PASS|FAIL|ERROR|passed|failed|band pairs" gpurun_out/tests.log | tail -40
if [ $s -ne 0 ] && [ $s -ne 1 ]; then exit $s; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err; s=$?
  echo "bench=$s"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
fi
