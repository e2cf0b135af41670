set -o pipefail
mkdir -p gpurun_out/r23
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "estep_on_reference_model or value_pair_layout or estep_sample_sizes or value_only or estep_pass_shapes" > gpurun_out/r23/tests.log 2>&1 || { tail -40 gpurun_out/r23/tests.log; exit 1; }
tail -2 gpurun_out/r23/tests.log
timeout -k 10 300 python -u tools/chain_ab.py pf 3 > gpurun_out/r23/chain_pf.log 2>&1 && cat gpurun_out/r23/chain_pf.log
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_base.so timeout -k 10 300 python -u tools/chain_ab.py base 3 > gpurun_out/r23/chain_base.log 2>&1 && cat gpurun_out/r23/chain_base.log
