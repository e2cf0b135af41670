set -o pipefail
mkdir -p gpurun_out/r1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "segmented_nth" > gpurun_out/r1/sel.log 2>&1 || { tail -30 gpurun_out/r1/sel.log; exit 1; }
tail -2 gpurun_out/r1/sel.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "estep_on_reference_model or estep_sample_sizes or cfg2_full_size or test_full_em" > gpurun_out/r1/tests.log 2>&1 || { tail -30 gpurun_out/r1/tests.log; exit 1; }
tail -2 gpurun_out/r1/tests.log
timeout -k 10 240 python -u tools/chain_ab.py new 3 > gpurun_out/r1/chain_new.log 2>&1 && cat gpurun_out/r1/chain_new.log
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_base.so timeout -k 10 240 python -u tools/chain_ab.py base 3 > gpurun_out/r1/chain_base.log 2>&1 && cat gpurun_out/r1/chain_base.log
