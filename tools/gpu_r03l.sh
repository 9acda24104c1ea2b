#!/bin/bash
# r03l: grid-barrier probe (persistent kernel vs one launch per phase)
mkdir -p gpurun_out
for a in "256 288 0" "256 288 64" "256 288 192" "512 288 0" "512 288 32" "128 288 0"; do
  timeout -k 10 60 ./tools/barrier_probe $a >> gpurun_out/r03l_probe.log 2>&1; s=$?
  [ $s -eq 0 ] || { echo "probe $a rc=$s"; cat gpurun_out/r03l_probe.log; exit $s; }
done
cat gpurun_out/r03l_probe.log
