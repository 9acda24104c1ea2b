#!/bin/bash
# A/B of bottleneck variants built by tools/bt_exp.sh: parity test vs the three-conv path, then
# rocprofv3 kernel stats of tools/classify_once.py (CO_K pairs) per variant.  usage: tools/bt_ab.sh TAG...
mkdir -p gpurun_out/btab
export TMPDIR=/tmp CBW_KWS_STREAMS=1   # one scoring stream: kernel durations not inflated by co-running chunks
for tag in $([ -n "$BT_NOTEST" ] || echo "$@"); do   # BT_NOTEST=1: diagnostic variants, timing only
  lib=enhance-cb-whisper_amd/cbw/exp_$tag/libcbw.so
  CBW_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_kws.py -q -x -k bottleneck --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/btab/test_$tag.log 2>&1 || { echo "$tag test fail"; tail -20 gpurun_out/btab/test_$tag.log; exit 1; }
  echo "[$tag] tests: $(tail -1 gpurun_out/btab/test_$tag.log)"
done
for rep in 1; do
for tag in "$@"; do
  lib=$PWD/enhance-cb-whisper_amd/cbw/exp_$tag/libcbw.so
  CBW_LIB=$lib CO_K=${CO_K:-1250} CO_REPS=${CO_REPS:-3} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/btab/p_${tag}_$rep \
      -o run --output-format csv -- python tools/classify_once.py > gpurun_out/btab/prof_${tag}_$rep.log 2>&1 || { echo "$tag prof fail"; exit 1; }
  echo "[$tag rep$rep] $(python3 tools/bt_times.py $tag)"
done
done
