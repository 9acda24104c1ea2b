#!/bin/bash
# r03t: C4 at full size on one GPU -- the 100k-keyword database as 8 ranks (gloo, every rank on GPU 0: the N-rank code
# path with its round-robin front end, broadcasts and all-gathers; timing meaningless) against one process scoring all
# 100k keywords: the same spotted keywords for the last clip (digest), every rank's audit 0 flips.
mkdir -p gpurun_out
timeout -k 10 500 python3 -u bench.py --mode kwshard --keywords 100000 --steps 2 --warmup 1 --no-cpu-baseline --no-companions > gpurun_out/r03t_k100k_1.json 2> gpurun_out/r03t_k100k_1.err; s=$?
echo "one=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03t_k100k_1.err; exit $s; }
export CBW_BENCH_DIST=gloo CBW_BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1 OMP_NUM_THREADS=2
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --mode kwshard --keywords 100000 --steps 2 --warmup 1 --no-cpu-baseline --no-companions > gpurun_out/r03t_k100k_8.json 2> gpurun_out/r03t_k100k_8.err; s=$?
echo "eight=$s"; [ $s -eq 0 ] || { tail -8 gpurun_out/r03t_k100k_8.err; exit $s; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/r03t_k100k_1.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/r03t_k100k_8.json").read().strip().splitlines()[-1])
for d in (a, b):
    print(d["n_gpus"], d["spotted_last_clip"], d["spotted_digest"], d["audit_flips"], d["audit_pairs"], d["audit_index_lists_equal"],
          [r["keywords"] for r in d["per_rank"]])
print("digest equal:", a["spotted_digest"] == b["spotted_digest"])
PY
