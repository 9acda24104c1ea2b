#!/bin/bash
# r03i: fp8 bias correction + unrolled quantize -- parity, then A/B (bias correction on / off) at the realistic
# point, and the synthetic point with it
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03i_fp8.log 2>&1; s=$?
echo "fp8tests=$s"; grep -E "FAIL|fp8 \|p" gpurun_out/r03i_fp8.log | head -24; [ $s -eq 0 ] || { grep -E "^E " gpurun_out/r03i_fp8.log | head -30; exit $s; }
for cfg in "1 realistic" "0 realistic" "1 synthetic"; do
  set -- $cfg
  CBW_FP8_BIAS_CORR=$1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --operating-point $2 --fp8-first > gpurun_out/r03i_bc$1$2.json 2> gpurun_out/r03i_bc$1$2.err; s=$?
  echo "bc=$1 $2 rc=$s"; [ $s -eq 0 ] || { tail -20 gpurun_out/r03i_bc$1$2.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03i_bc$1$2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], 'bf16', d['bf16_pairs_per_step'], 'flips', d['audit_flips'], d.get('audit_max_fp8_err'), d['fp8_first'], d['breakdown_ms']['kws_score'], d['roofline']['tiers']['fp8_first_tier'])"
done
