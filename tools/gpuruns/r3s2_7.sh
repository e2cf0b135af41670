set -o pipefail
mkdir -p gpurun_out/r7
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "estep_on_reference_model or estep_pass_shapes or estep_sample_sizes or value_only or wide_frontier or cfg2_full_size or test_full_em or underflow or edge_cases" > gpurun_out/r7/tests.log 2>&1 || { tail -40 gpurun_out/r7/tests.log; exit 1; }
tail -2 gpurun_out/r7/tests.log
timeout -k 10 300 python -u tools/chain_ab.py fused 3 > gpurun_out/r7/chain_fused.log 2>&1 && cat gpurun_out/r7/chain_fused.log
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_base.so timeout -k 10 300 python -u tools/chain_ab.py base 3 > gpurun_out/r7/chain_base.log 2>&1 && cat gpurun_out/r7/chain_base.log
