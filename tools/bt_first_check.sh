export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kws.py -q -x -k "bottleneck or cnn12 or golden" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bt1_tests.log 2>&1; s=$?; tail -3 gpurun_out/bt1_tests.log; [ $s -eq 0 ] || { tail -40 gpurun_out/bt1_tests.log; exit $s; }
CBW_KWS_STREAMS=1 CO_K=1250 CO_REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ct2 -o run --output-format csv -- python tools/classify_once.py > gpurun_out/ct2.log 2>&1
