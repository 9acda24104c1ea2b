#!/bin/bash
# MFMA-busy / issue / wait counters of conv_igemm_p8 on the plain GEMM shape and on the stage-3 3x3 shape
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/p8pmc2
for S in "1,1,65536,2048,2048,1" "625,5,47,256,256,3"; do
  T=$(echo $S | tr ',' '_')
  P8_SHAPE=$S timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/p8pmc2/$T -o run --output-format csv -- python3 tools/p8_pmc.py > gpurun_out/p8pmc2/$T.log 2>&1; s=$?
  echo "$S rc=$s"; tail -2 gpurun_out/p8pmc2/$T.log
  [ $s -eq 0 ] || exit $s
  python3 tools/pmc_kernel.py gpurun_out/p8pmc2/$T conv_igemm_p8
done
