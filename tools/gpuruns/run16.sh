set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r16
timeout -k 10 150 python -u tools/chain_ab.py base > gpurun_out/r16/ab_base.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_sel.so timeout -k 10 150 python -u tools/chain_ab.py sel > gpurun_out/r16/ab_sel.log 2>&1 && \
timeout -k 10 150 python -u tools/chain_ab.py base2 > gpurun_out/r16/ab_base2.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_sel.so timeout -k 10 150 python -u tools/chain_ab.py sel2 > gpurun_out/r16/ab_sel2.log 2>&1
