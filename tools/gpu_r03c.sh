#!/bin/bash
# r03c: kwshard rehearsal (2 gloo ranks on GPU 0) with the full log, then the decoder slice and the exactness tests
mkdir -p gpurun_out
CBW_BENCH_DEVICE=0 CBW_BENCH_DIST=gloo OMP_NUM_THREADS=4 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --model small --keywords 720 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --mode kwshard --gpus 2 > gpurun_out/r03c_ks.json 2> gpurun_out/r03c_ks.err; s=$?
echo "ks=$s"; cat gpurun_out/r03c_ks.json | tail -c 1500; grep -n "Error\|File \"" gpurun_out/r03c_ks.err | head -30; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decoder.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "large_v3 or fallback" > gpurun_out/r03c_dec.log 2>&1; s=$?
echo "dec=$s"; tail -15 gpurun_out/r03c_dec.log; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench_exact.py -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c_exact.log 2>&1; s=$?
echo "exact=$s"; tail -15 gpurun_out/r03c_exact.log; exit $s
