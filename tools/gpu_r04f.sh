#!/bin/bash
# r04f: A/B of compensated-tier passes of 1024 pairs (CBW_X3_CHUNK) in the headline bench (alternating), the drop-in
# API path's number (--mode api), and C5's long-form at 300 s: four lanes vs one lane of batched generate calls
# (--generate-batch 3) vs two lanes of them
mkdir -p gpurun_out/r04f
O=gpurun_out/r04f
for r in 1 2; do
  for C in 512 1024; do
    CBW_X3_CHUNK=$C timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --no-companions > $O/x3c_${C}_$r.json 2> $O/x3c_${C}_$r.err || { tail -5 $O/x3c_${C}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/x3c_${C}_$r.json').read().strip().splitlines()[-1]); t=(d.get('roofline') or {}).get('tiers') or {}; print('x3_chunk=$C', d['value'], d['ms_per_step'], (t.get('compensated_rescoring') or {}).get('union_ms_per_step'), d['audit_flips'])" || exit 1
  done
done
timeout -k 10 600 python3 -u bench.py --mode api --steps 5 --warmup 2 > $O/api.json 2> $O/api.err; s=$?
echo "api=$s"; tail -c 900 $O/api.json; [ $s -eq 0 ] || { tail -20 $O/api.err; exit $s; }
for cfg in "--audios-in-flight 4" "--generate-batch 3" "--audios-in-flight 2 --generate-batch 3"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 600 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --fp8-first --operating-point realistic $cfg > $O/lf_$tag.json 2> $O/lf_$tag.err; s=$?
  echo "lf $cfg=$s"; [ $s -eq 0 ] || { tail -20 $O/lf_$tag.err; exit $s; }
  python3 -c "import json; d=json.loads(open('$O/lf_$tag.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_window'], d['windows'], d['config']['generate_batch'], d['config']['audios_in_flight'])"
done
