#!/bin/bash
# decoder bookkeeping kernels: GPU decoder tests, long-form bench, kernel stats of one long-form audio
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python -u -m pytest tests/test_gpu_decoder.py tests/test_gpu_cbwhisper.py -m gpu -q -x -p no:cacheprovider > gpurun_out/m_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/m_tests.log
[ $s -eq 0 ] || exit $s
timeout -k 10 400 python3 -u bench.py --mode longform --steps 2 --warmup 1 --audio-seconds 60 > gpurun_out/lf_m.json 2> gpurun_out/lf_m.err; s=$?
echo "lf=$s"; tail -2 gpurun_out/lf_m.err; cat gpurun_out/lf_m.json
[ $s -eq 0 ] || exit $s
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/lfm -o run --output-format csv -- python3 bench.py --mode longform --steps 1 --warmup 0 --audio-seconds 60 > gpurun_out/lfm.log 2>&1; s=$?
echo "lfm=$s"
[ $s -eq 0 ] || exit $s
grep -E "beam_select|timestamp_rules|copyBuffer|gemv_kernel|reorder" gpurun_out/lfm/run_kernel_stats.csv | cut -d, -f1-5
