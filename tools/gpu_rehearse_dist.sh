#!/bin/bash
# Rehearsal of bench.py's N-rank code paths on a one-GPU box: two ranks pinned to GPU 0 over gloo (numbers are
# meaningless -- both ranks share the card; RCCL refuses two ranks on one device).  The driver's 8-GPU runs use
# one rank per GPU over RCCL.
mkdir -p gpurun_out
export CBW_BENCH_DIST=gloo CBW_BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dist_clip.json 2> gpurun_out/dist_clip.err; s=$?
echo "clip-parallel=$s"; tail -3 gpurun_out/dist_clip.err; cat gpurun_out/dist_clip.json
[ $s -eq 0 ] || exit $s
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --mode kwshard > gpurun_out/dist_kw.json 2> gpurun_out/dist_kw.err; s=$?
echo "kwshard=$s"; tail -3 gpurun_out/dist_kw.err; cat gpurun_out/dist_kw.json
