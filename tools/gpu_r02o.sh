#!/bin/bash
# decoder tests + long-form bench (KV reorder skips identity rows)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -q -x -p no:cacheprovider > gpurun_out/o_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/o_tests.log
[ $s -eq 0 ] || exit $s
timeout -k 10 400 python3 -u bench.py --mode longform --steps 2 --warmup 1 --audio-seconds 60 > gpurun_out/lf_o.json 2> gpurun_out/lf_o.err; s=$?
echo "lf=$s"; tail -1 gpurun_out/lf_o.err; cat gpurun_out/lf_o.json
