set -o pipefail
mkdir -p gpurun_out/r15
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "value_pair_layout" > gpurun_out/r15/tests.log 2>&1 || { tail -40 gpurun_out/r15/tests.log; exit 1; }
tail -2 gpurun_out/r15/tests.log
timeout -k 10 300 python -u tools/chain_ab.py pair 3 > gpurun_out/r15/chain_pair.log 2>&1 && cat gpurun_out/r15/chain_pair.log
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_base.so timeout -k 10 300 python -u tools/chain_ab.py base 3 > gpurun_out/r15/chain_base.log 2>&1 && cat gpurun_out/r15/chain_base.log
timeout -k 10 300 python -u tools/e1_shapes.py 3 0:0:0:0 0:0:4:4 0:0:8:2 0:0:6:2 > gpurun_out/r15/e1.log 2>&1 && cat gpurun_out/r15/e1.log
