#!/bin/bash
# r03g: the 8-wave fp8 kernel (Cout % 256) -- conv parity, then the realistic-point fp8 bench with / without it
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g_fp8.log 2>&1; s=$?
echo "fp8tests=$s"; grep -E "PASS|FAIL|fp8 \|p" gpurun_out/r03g_fp8.log | head -20; [ $s -eq 0 ] || { grep -E "^E " gpurun_out/r03g_fp8.log | head -30; exit $s; }
for p8 in 1 0; do
  CBW_FP8_P8=$p8 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --operating-point realistic --fp8-first > gpurun_out/r03g_p8$p8.json 2> gpurun_out/r03g_p8$p8.err; s=$?
  echo "p8=$p8 rc=$s"; [ $s -eq 0 ] || { tail -20 gpurun_out/r03g_p8$p8.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03g_p8$p8.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], 'bf16', d['bf16_pairs_per_step'], 'flips', d['audit_flips'], d.get('audit_max_fp8_err'), d['breakdown_ms'], d['roofline']['tiers'])"
done
