#!/bin/bash
# Host-code sanitizer run of libcbw's runtime (CPU only; never on the GPU box): runtime.cpp rebuilt with
# AddressSanitizer + UndefinedBehaviorSanitizer on its HOST side only (-Xarch_host before each -fsanitize=; the device
# code and the kernel objects are the normal build's), linked with tests/sanitize/host_driver.cpp into one executable
# under $OUT (default /tmp/cbw_sanitize), then run with halt_on_error.  Needs the normal build's objects first
# (python -c "import __graft_entry__ as g; g.build()").  tests/test_host.py::test_runtime_host_sanitizers runs it.
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
CSRC="$REPO/enhance-cb-whisper_amd/csrc"
OUT="${OUT:-/tmp/cbw_sanitize}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
mkdir -p "$OUT"
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
     -Xarch_host -fno-sanitize-recover=undefined)
OBJS=()
for f in conv_fp8.hip conv_fp8_stream.hip conv_igemm.hip conv_ring.hip conv_stream.hip gemv.hip bottleneck.hip \
         kws_kernels.hip kws_exact.hip whisper_kernels.hip; do
  OBJS+=("$CSRC/build/$f.o")
  [ -f "$CSRC/build/$f.o" ] || { echo "missing $CSRC/build/$f.o: run the normal build first" >&2; exit 2; }
done
"$HIPCC" -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -I"$REPO/include" -I"$CSRC" -x hip "${SAN[@]}" \
  -c "$CSRC/runtime.cpp" -o "$OUT/runtime_san.o"
"$HIPCC" -O1 -g -std=c++17 -x c++ -I"$REPO/include" -fsanitize=address,undefined \
  -fno-omit-frame-pointer -fno-sanitize-recover=undefined -c "$REPO/tests/sanitize/host_driver.cpp" -o "$OUT/driver.o"
"$HIPCC" --offload-arch=gfx950 "${SAN[@]}" -o "$OUT/host_driver" "$OUT/driver.o" "$OUT/runtime_san.o" "${OBJS[@]}" \
  "$CSRC/build/source_id.o"
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1:abort_on_error=0 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  "$OUT/host_driver"
