# single-stream per-layer timing of one 625-pair chunk (rocprofv3 kernel trace) -> tools/chunk_trace.py
mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CBW_KWS_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/chunk_${TAG:-x} -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --exact-band 0 --no-pipeline ${BENCH_ARGS} > gpurun_out/chunk_${TAG:-x}.log 2>&1; s=$?
echo "trace=$s"; [ $s -eq 0 ] || { tail -5 gpurun_out/chunk_${TAG:-x}.log; exit $s; }
python3 tools/chunk_trace.py $(find gpurun_out/chunk_${TAG:-x} -name "*kernel_trace.csv")
