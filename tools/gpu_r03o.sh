#!/bin/bash
# r03o: decoder step timing + kernel trace, keyword-sharded per-rank simulation, long-form with 1 vs 2 audios in flight
mkdir -p gpurun_out
for LA in 0 1 0 1; do
  CBW_DEC_LA=$LA timeout -k 10 180 python3 -u tools/decode_bench.py large-v3 5 64 >> gpurun_out/r03o_dec$LA.log 2>&1; s=$?
  echo "dec LA=$LA rc=$s"; tail -1 gpurun_out/r03o_dec$LA.log; [ $s -eq 0 ] || exit $s
done
for R in 0 3; do
  timeout -k 10 400 python3 -u bench.py --mode kwshard --shard-sim $R/8 --keywords 12500 --steps 16 --warmup 8 --no-cpu-baseline --no-companions > gpurun_out/r03o_kwsim$R.json 2> gpurun_out/r03o_kwsim$R.err; s=$?
  echo "kwsim$R=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03o_kwsim$R.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03o_kwsim$R.json').read().strip().splitlines()[-1]); print(d['value'], d['per_rank'], d['audit_flips'])"
done
for A in 1 2; do
  timeout -k 10 400 python3 -u bench.py --mode longform --audio-seconds 300 --steps 1 --warmup 1 --audios-in-flight $A > gpurun_out/r03o_lf$A.json 2> gpurun_out/r03o_lf$A.err; s=$?
  echo "lf$A=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/r03o_lf$A.err; exit $s; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03o_lf$A.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_window'], d['windows'], d['spotting_ms_per_window'], d['transcript_digests'])"
done
cd /tmp && export TMPDIR=/tmp
CBW_DEC_LA=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03o_decprof -o dec --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py large-v3 5 64 > $GRAFT_REPO_ROOT/gpurun_out/r03o_decprof.log 2>&1; s=$?
echo "decprof=$s"; exit $s
