#!/bin/bash
# Variant builds of conv_igemm.hip (compile-time knobs) linked with the other in-tree objects into
# enhance-cb-whisper_amd/cbw/exp_<tag>/libcbw.so.  usage: tools/ci_exp.sh TAG "-DKNOB=1" [TAG2 "FLAGS2" ...]
set -e
cd "$(dirname "$0")/../enhance-cb-whisper_amd/csrc"
OBJS=$(ls build/*.o | grep -v conv_igemm)
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  mkdir -p build/exp_$tag ../cbw/exp_$tag
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. $flags -x hip -c conv_igemm.hip \
      -o build/exp_$tag/conv_igemm.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../cbw/exp_$tag/libcbw.so $OBJS build/exp_$tag/conv_igemm.o
done
