# PMC pass over tools/p8_pmc.py (one p8 GEMM shape): LDS conflicts, LDS activity, wave/busy cycles, waits
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/p8pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY -d gpurun_out/p8pmc/${TAG:-a} -o run --output-format csv -- python3 tools/p8_pmc.py > gpurun_out/p8pmc/${TAG:-a}.log 2>&1
echo "rc=$?"
python3 tools/pmc_kernel.py gpurun_out/p8pmc/${TAG:-a} conv_igemm_p8
