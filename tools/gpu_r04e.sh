#!/bin/bash
# r04e: decode-step A/B of two-wave GEMV workgroups for the N <= 1280 Linears (CBW_GEMV_WV2, alternating), the
# drop-in API path's number (--mode api), and C5's long-form at 300 s: four lanes vs one lane of batched generate
# calls (--generate-batch 3) vs two lanes of them
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
  for M in 0 1; do
    CBW_GEMV_WV2=$M timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> $O/dec_wv2_$M.log 2>&1 || exit $?
  done
done
grep -h "decoder" $O/dec_wv2_0.log $O/dec_wv2_1.log
timeout -k 10 600 python3 -u bench.py --mode api --steps 5 --warmup 2 > $O/api.json 2> $O/api.err; s=$?
echo "api=$s"; tail -c 900 $O/api.json; [ $s -eq 0 ] || { tail -20 $O/api.err; exit $s; }
for cfg in "--audios-in-flight 4" "--generate-batch 3" "--audios-in-flight 2 --generate-batch 3"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --fp8-first --operating-point realistic $cfg > $O/lf_$tag.json 2> $O/lf_$tag.err; s=$?
  echo "lf $cfg=$s"; [ $s -eq 0 ] || { tail -20 $O/lf_$tag.err; exit $s; }
  python3 -c "import json; d=json.loads(open('$O/lf_$tag.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_window'], d['windows'], d['config']['generate_batch'], d['config']['audios_in_flight'])"
done
