#!/bin/bash
# r04b: the PMC passes of the 3-step bench without the post-run audit (r04a: the SIGSEGV is in the main thread, inside
# hipLaunchKernel under the profiler's counter collection, at the audit's fp32 re-scoring of all 10 000 pairs -- after
# the timed region), then the kernel-trace pass and the roofline; last, a diagnostic: the audit on again with counters
# collected only for the bf16 conv family (--kernel-include-regex), which tells whether counting the audit's
# conv_f32 dispatches is what crashes.
mkdir -p gpurun_out/r04b
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04b
BA="--steps 3 --warmup 1 --no-cpu-baseline --no-companions"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- python3 -u bench.py $BA --no-audit --prof-dump $O/dump_$C.json > $O/pmc_$C.log 2>&1; s=$?
  echo "pmc $C=$s"; tail -2 $O/pmc_$C.log
  [ $s -eq 0 ] || exit $s
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u bench.py $BA --prof-dump $O/dump_trace.json > $O/trace.log 2>&1; s=$?
echo "trace=$s"; tail -2 $O/trace.log; [ $s -eq 0 ] || exit $s
python3 tools/roofline_from_trace.py $O/trace --dump $O/dump_trace.json --fetch $O/pmc_FETCH_SIZE --fetch-dump $O/dump_FETCH_SIZE.json --write $O/pmc_WRITE_SIZE --write-dump $O/dump_WRITE_SIZE.json --out $O/roofline.json > /dev/null; s=$?
echo "roofline=$s"; head -40 $O/roofline.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'conv_igemm|conv_ring|conv_stream|bottleneck' -d $O/pmc_diag -o run --output-format csv -- python3 -u bench.py $BA --prof-dump $O/dump_diag.json > $O/pmc_diag.log 2>&1; s=$?
echo "diag (audit on, counters on the bf16 family only)=$s"; grep -v "^    @" $O/pmc_diag.log | tail -12
exit 0
