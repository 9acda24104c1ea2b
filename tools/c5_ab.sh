#!/bin/bash
# C5 companion A/B over an environment setting: bash tools/c5_ab.sh "CBW_KWS_STREAMS=2" "CBW_KWS_STREAMS=3"
mkdir -p gpurun_out
for e in "$@"; do
  for mode in "--audios-in-flight 4" "--generate-batch 4 --batch-length-step 0"; do
    env $e timeout -k 10 300 python3 bench.py --mode longform --audio-seconds 300 $mode --fp8-first \
      --operating-point realistic --steps 1 --warmup 1 > gpurun_out/c5_ab.json 2> gpurun_out/c5_ab.err || { echo "fail $e $mode"; tail -3 gpurun_out/c5_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5_ab.json').read().strip().splitlines()[-1]); print(sys.argv[1], sys.argv[2], d['value'], d.get('spotting_ms_per_window'), d.get('ms_per_window'))" "$e" "$mode"
  done
done
