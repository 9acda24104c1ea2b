timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decoder.py -p no:cacheprovider > gpurun_out/dec_tests.log 2>&1; s=$?; tail -3 gpurun_out/dec_tests.log; [ $s -eq 0 ] || { tail -30 gpurun_out/dec_tests.log; exit $s; }
CBW_DEC_GRAPH=0 timeout -k 10 120 python tools/decode_bench.py large-v3 5 64 2>&1 | grep decoder
CBW_DEC_GRAPH=1 timeout -k 10 120 python tools/decode_bench.py large-v3 5 64 2>&1 | grep decoder
