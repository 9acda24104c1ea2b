#!/bin/bash
# r04e: fp8 tier tests + fp8-first bench and kernel profile, beam-sample tests, decode-step A/B of two-wave GEMV
# workgroups for the N <= 1280 Linears (CBW_GEMV_WV2, alternating), the drop-in API path's number (--mode api), and
# the e4m3 8-wave schedule on stage 3 only (CBW_FP8_P8=2) against the 4-wave kernel (alternating)
mkdir -p gpurun_out/r04e
O=gpurun_out/r04e
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp8.py > $O/fp8_tests.log 2>&1; s=$?
echo "fp8_tests=$s"; grep -E "PASS|FAIL|Error|max \|dp" $O/fp8_tests.log | tail -12; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_decoder.py -k "beam_sample or beam_search_matches_oracle" > $O/bs_tests.log 2>&1; s=$?
echo "bs_tests=$s"; grep -E "PASS|FAIL|Error|beam sample:" $O/bs_tests.log | tail -6; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --fp8-first --operating-point realistic --no-companions > $O/fp8first.json 2> $O/fp8first.err; s=$?
echo "fp8first=$s"; python3 -c "import json; d=json.loads(open('$O/fp8first.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps((d.get('roofline') or {}).get('tiers')))" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o fp8 -- python3 -u bench.py --steps 3 --warmup 2 --fp8-first --operating-point realistic --no-companions --no-audit > $O/prof8.json 2> $O/prof8.err; s=$?
echo "prof8=$s"; [ $s -eq 0 ] || { tail -5 $O/prof8.err; exit $s; }
for r in 1 2; do
  for M in 0 1 2; do
    CBW_GEMV_WV2=$M timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> $O/dec_wv2_$M.log 2>&1 || exit $?
  done
done
grep -h "decoder" $O/dec_wv2_0.log $O/dec_wv2_1.log $O/dec_wv2_2.log
timeout -k 10 600 python3 -u bench.py --mode api --steps 5 --warmup 2 > $O/api.json 2> $O/api.err; s=$?
echo "api=$s"; tail -c 900 $O/api.json; [ $s -eq 0 ] || { tail -20 $O/api.err; exit $s; }
for r in 1 2; do
  for M in 0 2; do
    CBW_FP8_P8=$M timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --fp8-first --operating-point realistic --no-companions > $O/fp8p8_${M}_$r.json 2> $O/fp8p8_${M}_$r.err || { tail -5 $O/fp8p8_${M}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/fp8p8_${M}_$r.json').read().strip().splitlines()[-1]); t=(d.get('roofline') or {}).get('tiers') or {}; print('fp8_p8=$M', d['value'], d['ms_per_step'], (t.get('fp8_first_tier') or {}).get('union_ms_per_step'), d['audit_flips'])" || exit 1
  done
done
