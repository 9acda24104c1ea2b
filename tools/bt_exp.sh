#!/bin/bash
# Diagnostic builds of the fused stage-1 bottleneck kernel (BT_EXP variants, see bottleneck.hip),
# each linked into its own libcbw copy under build/exp<N>/ and timed with tools/classify_once.py.
set -e
cd "$(dirname "$0")/../enhance-cb-whisper_amd/csrc"
for e in "$@"; do
  mkdir -p build/exp$e ../cbw/exp$e
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. -DBT_EXP=$e -x hip -c bottleneck.hip -o build/exp$e/bottleneck.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../cbw/exp$e/libcbw.so build/conv_igemm.hip.o build/exp$e/bottleneck.o build/kws_kernels.hip.o build/whisper_kernels.hip.o build/runtime.cpp.o
done
