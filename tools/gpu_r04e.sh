#!/bin/bash
# r04e: fp8 tier tests, beam-sample tests, a kernel profile of the fp8-first bench, the fp8 tier's two A/Bs in the
# fp8-first bench at the realistic operating point -- the stage-1 output quantized inside the last fused block
# (CBW_FP8_Q8=1) and the 8-wave e4m3 schedule on stage 3 only (CBW_FP8_P8=2) -- and the decode-step A/B of two-wave
# GEMV workgroups for the N <= 1280 Linears (CBW_GEMV_WV2 1: without, 2: with the LayerNorm GEMVs)
mkdir -p gpurun_out/r04e
export TMPDIR=/tmp
O=gpurun_out/r04e
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp8.py > $O/fp8_tests.log 2>&1; s=$?
echo "fp8_tests=$s"; grep -E "PASS|FAIL|Error|max \|dp" $O/fp8_tests.log | tail -12; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decoder.py -k "beam_sample or beam_search_matches_oracle" > $O/bs_tests.log 2>&1; s=$?
echo "bs_tests=$s"; grep -E "PASS|FAIL|Error|beam sample:" $O/bs_tests.log | tail -6; [ $s -eq 0 ] || exit $s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o fp8 -- python3 -u bench.py --steps 3 --warmup 2 --fp8-first --operating-point realistic --no-companions --no-audit > $O/prof8.json 2> $O/prof8.err; s=$?
echo "prof8=$s"; [ $s -eq 0 ] || { tail -5 $O/prof8.err; exit $s; }
for cfg in "0 0" "0 1" "2 0" "2 1" "0 0" "2 1"; do
  set -- $cfg
  tag=p$1q$2
  CBW_FP8_P8=$1 CBW_FP8_Q8=$2 timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --fp8-first --operating-point realistic --no-companions > $O/fp8_$tag.json 2> $O/fp8_$tag.err || { tail -5 $O/fp8_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/fp8_$tag.json').read().strip().splitlines()[-1]); t=(d.get('roofline') or {}).get('tiers') or {}; print('fp8 p8=$1 q8=$2', d['value'], d['ms_per_step'], (t.get('fp8_first_tier') or {}).get('union_ms_per_step'), d['audit_flips'], d['spotted_digest'])" || exit 1
done
for r in 1 2; do
  for M in 0 1 2; do
    CBW_GEMV_WV2=$M timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> $O/dec_wv2_$M.log 2>&1 || exit $?
  done
done
grep -h "decoder" $O/dec_wv2_0.log $O/dec_wv2_1.log $O/dec_wv2_2.log
