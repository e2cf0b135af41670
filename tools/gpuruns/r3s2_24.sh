set -o pipefail
mkdir -p gpurun_out/r24
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_u8.so timeout -k 10 300 python -u tools/chain_ab.py u8 3 > gpurun_out/r24/chain_u8.log 2>&1 && cat gpurun_out/r24/chain_u8.log
timeout -k 10 300 python -u tools/chain_ab.py u4 3 > gpurun_out/r24/chain_u4.log 2>&1 && cat gpurun_out/r24/chain_u4.log
