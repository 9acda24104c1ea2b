#!/bin/bash
# r03h: fp8 streaming 1x1 kernel + the 8-wave schedule restricted to >= 8 K-tiles -- parity, then A/B at the
# realistic point
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h_fp8.log 2>&1; s=$?
echo "fp8tests=$s"; grep -E "PASS|FAIL|fp8 \|p" gpurun_out/r03h_fp8.log | head -24; [ $s -eq 0 ] || { grep -E "^E " gpurun_out/r03h_fp8.log | head -30; exit $s; }
for cfg in "1 1" "0 1" "1 0"; do
  set -- $cfg
  CBW_FP8_STREAM=$1 CBW_FP8_P8=$2 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --operating-point realistic --fp8-first > gpurun_out/r03h_s$1p$2.json 2> gpurun_out/r03h_s$1p$2.err; s=$?
  echo "stream=$1 p8=$2 rc=$s"; [ $s -eq 0 ] || { tail -20 gpurun_out/r03h_s$1p$2.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03h_s$1p$2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], 'bf16', d['bf16_pairs_per_step'], 'flips', d['audit_flips'], d.get('audit_max_fp8_err'), d['breakdown_ms']['kws_score'], d['roofline']['tiers']['fp8_first_tier'])"
done
