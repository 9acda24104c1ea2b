#!/bin/bash
# r03an: four lanes sharing a 3-slot window batcher (lanes beyond the slots queue while their next window's encoder and
# spotting run) vs four lanes of separate steps, 300 s audios
mkdir -p gpurun_out
for B in "" --batch-windows; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight 4 $B > gpurun_out/r03an_lf300_a4$B.json 2> gpurun_out/r03an_lf300_a4$B.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r03an_lf300_a4$B.json').read().strip().splitlines()[-1]); print('$B', d['value'], d['ms_per_window'], d.get('window_batch'), d['transcript_digests'])"
done
