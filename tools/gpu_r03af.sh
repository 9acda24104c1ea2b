#!/bin/bash
# r03af: several windows in one decode step (cbw_decoder_step_rows, cbw.window_batch): bit-exact vs single-window
# steps, the batcher vs beam_search_dev, the long-form bench with --batch-windows vs one lane; then C5 300 s A/B
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decoder.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "step_rows or window_batcher or graph_replay or fused_layernorm or knobs" > gpurun_out/r03af_tests.log 2>&1; s=$?
echo "tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03af_tests.log | tail -15; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bench_modes.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "batched_windows" > gpurun_out/r03af_bench_tests.log 2>&1; s=$?
echo "bench tests=$s"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03af_bench_tests.log | tail -15; [ $s -eq 0 ] || exit $s
for B in "" --batch-windows; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight 3 $B > gpurun_out/r03af_lf300_a3$B.json 2> gpurun_out/r03af_lf300_a3$B.err; s=$?
  echo "lf300_a3$B=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03af_lf300_a3$B.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03af_lf300_a3$B.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'], d.get('window_batch'), d['transcript_digests'])"
done
