#!/bin/bash
# Variant builds of the fused stage-1 bottleneck kernel (bottleneck.hip compile-time knobs), each linked
# with the in-tree objects into its own libcbw copy: enhance-cb-whisper_amd/cbw/exp_<tag>/libcbw.so.
# usage: tools/bt_exp.sh TAG "-DBT_RG=1 -DBT_MG=1" [TAG2 "FLAGS2" ...]   (CBW_LIB=<that path> selects it)
set -e
cd "$(dirname "$0")/../enhance-cb-whisper_amd/csrc"
OBJS=$(ls build/*.o | grep -v bottleneck)
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  mkdir -p build/exp_$tag ../cbw/exp_$tag
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. $flags -x hip -c bottleneck.hip \
      -o build/exp_$tag/bottleneck.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "VGPRs|AGPRs|Spill|Occupancy|LDS" | sed "s/^/[$tag] /"
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../cbw/exp_$tag/libcbw.so $OBJS build/exp_$tag/bottleneck.o
done
