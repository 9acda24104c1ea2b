#!/bin/bash
# scalar K-tile walk in p8 and the 4-wave tile kernel: full GPU suite, per-layer times, counters, bench x2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/sca_tests.log 2>&1; s=$?
echo "tests=$s"; tail -3 gpurun_out/sca_tests.log
[ $s -eq 0 ] || exit $s
LB_PAIRS=625 LB_MODES=1 timeout -k 10 300 python -u tools/layer_bench.py > gpurun_out/sca_layers.log 2>&1; s=$?
echo "layers=$s"; grep -v repeat gpurun_out/sca_layers.log | grep -E "b3|b4|b7|b8|b13|b14|TOTAL"
[ $s -eq 0 ] || exit $s
P8_SHAPE="625,5,47,256,256,3" timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/p8pmc3 -o run --output-format csv -- python3 tools/p8_pmc.py > gpurun_out/p8pmc3.log 2>&1; s=$?
echo "pmc=$s"; [ $s -eq 0 ] || exit $s
python3 tools/pmc_kernel.py gpurun_out/p8pmc3 conv_igemm_p8
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sca_bench_$r.json 2> gpurun_out/sca_bench_$r.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/sca_bench_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['breakdown_ms']['kws_score'], d['spotted_digest'], d['roofline']['frac'])"
done
