#!/bin/bash
# r03y: validation of HEAD -- smoke, the full GPU suite, then the default bench as the driver runs it
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.log 2>&1; s=$?
echo "smoke=$s"; tail -1 gpurun_out/r03y_smoke.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r03y_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03y_tests.log | tail -15; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r03y_bench.json 2> gpurun_out/r03y_bench.err; s=$?
echo "bench=$s"; tail -c 1200 gpurun_out/r03y_bench.json; exit $s
