#!/bin/bash
# r03m: whole-image fused stage-3 bottleneck -- parity test, then bench A/B and a kernel trace
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kws.py -k "image_bottleneck or bottleneck_fusion" -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03m_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r03m_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for M in 1 0; do
  CBW_BT3=$M timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-companions > gpurun_out/r03m_bench$M.json 2> gpurun_out/r03m_bench$M.err; s=$?
  echo "bench$M=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03m_bench$M.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03m_bench$M.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['audit_flips'], d['spotted_digest'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp CBW_BT3=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03m_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-companions --no-audit > $GRAFT_REPO_ROOT/gpurun_out/r03m_prof.log 2>&1; s=$?
echo "prof=$s"; exit $s
