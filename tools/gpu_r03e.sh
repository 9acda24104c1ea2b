#!/bin/bash
# r03e: the fp8 first tier -- instruction probes, conv kernel vs float64, network + cascade, then the bench at the
# synthetic and the realistic operating point with and without the fp8 tier
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fp8.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_fp8.log 2>&1; s=$?
echo "fp8tests=$s"; grep -E "PASS|FAIL|Error|assert|matching|fp8 \|p" gpurun_out/r03e_fp8.log | head -40; [ $s -eq 0 ] || { tail -40 gpurun_out/r03e_fp8.log; exit $s; }
for cfg in "synthetic:" "synthetic:--fp8-first" "realistic:" "realistic:--fp8-first"; do
  op=${cfg%%:*}; fl=${cfg#*:}; tag=${op}${fl:+_fp8}
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --operating-point $op $fl > gpurun_out/r03e_$tag.json 2> gpurun_out/r03e_$tag.err; s=$?
  echo "$tag=$s"; [ $s -eq 0 ] || { tail -30 gpurun_out/r03e_$tag.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03e_$tag.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], 'spotted', d['spotted_last_clip'], 'bf16', d['bf16_pairs_per_step'], 'band', d['rescored_pairs_per_step'], 'flips', d['audit_flips'], d.get('audit_max_fp8_err'), d['fp8_first'], d['operating_point'], d['breakdown_ms'])"
done
