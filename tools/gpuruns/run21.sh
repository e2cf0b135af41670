set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r21
timeout -k 10 150 python -u tools/chain_ab.py base > gpurun_out/r21/ab_base.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_tw.so timeout -k 10 150 python -u tools/chain_ab.py tw > gpurun_out/r21/ab_tw.log 2>&1 && \
timeout -k 10 150 python -u tools/chain_ab.py base2 > gpurun_out/r21/ab_base2.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_tw.so timeout -k 10 150 python -u tools/chain_ab.py tw2 > gpurun_out/r21/ab_tw2.log 2>&1
