#!/bin/bash
# r04d: the round-4 GPU tests (C5 at large-v3 widths, batched long-form, the decoder tests after the pruning, the bench
# modes incl. --generate-batch), then C2 / C1 through bench.py --variant
mkdir -p gpurun_out/r04d
O=gpurun_out/r04d
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batched.py tests/test_gpu_decoder.py tests/test_gpu_c5.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests_a.log 2>&1; s=$?
echo "tests_a=$s"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests_a.log | tail -40; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kws.py tests/test_host.py -k "checksum or matches_sources" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_k.log 2>&1; s=$?
echo "tests_k=$s"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests_k.log | tail -5; [ $s -eq 0 ] || exit $s
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_bench_modes.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests_b.log 2>&1; s=$?
echo "tests_b=$s"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests_b.log | tail -10; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python3 -u bench.py --model small --variant LE --keywords 1000 --chunk 250 --steps 5 --warmup 1 --no-cpu-baseline --no-companions > $O/c2.json 2> $O/c2.err; s=$?
echo "c2=$s"; tail -c 1500 $O/c2.json; [ $s -eq 0 ] || { tail -20 $O/c2.err; exit $s; }
timeout -k 10 400 python3 -u bench.py --model tiny.en --variant L --keywords 32 --chunk 32 --steps 5 --warmup 1 --no-cpu-baseline --no-companions > $O/c1.json 2> $O/c1.err; s=$?
echo "c1=$s"; tail -c 1500 $O/c1.json; [ $s -eq 0 ] || { tail -20 $O/c1.err; exit $s; }
