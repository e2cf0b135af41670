set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex estep_forward --output-format csv -d gpurun_out/pmc/p1 -o p -- python3 tools/estep_once.py > gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-include-regex estep_forward --output-format csv -d gpurun_out/pmc/p2 -o p -- python3 tools/estep_once.py > gpurun_out/pmc/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_ACTIVE_INST_SCA --kernel-include-regex estep_forward --output-format csv -d gpurun_out/pmc/p3 -o p -- python3 tools/estep_once.py > gpurun_out/pmc/p3.log 2>&1
