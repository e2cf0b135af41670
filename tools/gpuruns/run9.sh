set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r9
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "sample_size or large_sample or pass_shapes or estep_on_reference or value_only" > gpurun_out/r9/tests.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_head.so timeout -k 10 300 python -u tools/chain_ab.py head > gpurun_out/r9/ab_head.log 2>&1 && \
timeout -k 10 300 python -u tools/chain_ab.py cur > gpurun_out/r9/ab_cur.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_cpf.so timeout -k 10 300 python -u tools/chain_ab.py cpf > gpurun_out/r9/ab_cpf.log 2>&1 && \
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_head.so timeout -k 10 300 python -u tools/chain_ab.py head2 > gpurun_out/r9/ab_head2.log 2>&1
