#!/bin/bash
# r04a: the r03 PMC crash -- the FETCH_SIZE and WRITE_SIZE passes of the 3-step bench
# under rocprofv3 --pmc with bench.py's faulthandler on (all threads), every log kept; then the kernel-trace pass and
# the roofline recomputed from the three passes (tools/prof_r02.sh's recipe).  The library check runs first.
mkdir -p gpurun_out/r04a
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04a
timeout -k 10 120 python3 -m pytest tests/test_host.py -q -p no:cacheprovider -k "matches_sources or exports" > $O/host.log 2>&1 || { cat $O/host.log; exit 1; }
BA="--steps 3 --warmup 1 --no-cpu-baseline --no-companions"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- python3 -u bench.py $BA --prof-dump $O/dump_$C.json > $O/pmc_$C.log 2>&1; s=$?
  echo "pmc $C=$s"; tail -4 $O/pmc_$C.log
  [ $s -eq 0 ] || exit $s
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u bench.py $BA --prof-dump $O/dump_trace.json > $O/trace.log 2>&1; s=$?
echo "trace=$s"; tail -2 $O/trace.log; [ $s -eq 0 ] || exit $s
python3 tools/roofline_from_trace.py $O/trace --dump $O/dump_trace.json --fetch $O/pmc_FETCH_SIZE --fetch-dump $O/dump_FETCH_SIZE.json --write $O/pmc_WRITE_SIZE --write-dump $O/dump_WRITE_SIZE.json --out $O/roofline.json > /dev/null; s=$?
echo "roofline=$s"; head -40 $O/roofline.json
