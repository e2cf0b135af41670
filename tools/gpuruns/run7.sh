set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r7
timeout -k 10 300 python -u tools/chain_ab.py base > gpurun_out/r7/ab_base.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_pf.so timeout -k 10 300 python -u tools/chain_ab.py pf > gpurun_out/r7/ab_pf.log 2>&1 && \
timeout -k 10 300 python -u tools/chain_ab.py base2 > gpurun_out/r7/ab_base2.log 2>&1 && \
CFG=3 ITERS=2 timeout -k 10 400 python -u tools/stamps_split.py > gpurun_out/r7/stamps_split.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 600 python -u tools/cfg4_m0.py > gpurun_out/r7/cfg4_m0.log 2>&1
