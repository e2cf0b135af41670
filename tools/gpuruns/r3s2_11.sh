set -o pipefail
mkdir -p gpurun_out/r11
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "estep_pass_shapes or estep_shape_invariance or small_frontier" > gpurun_out/r11/tests.log 2>&1 || { tail -40 gpurun_out/r11/tests.log; exit 1; }
tail -2 gpurun_out/r11/tests.log
timeout -k 10 300 python -u tools/chain_ab.py staged 3 > gpurun_out/r11/chain_staged.log 2>&1 && cat gpurun_out/r11/chain_staged.log
HMC_AMD_LIB=$PWD/hmc_amd/libhmc_amd_base.so timeout -k 10 300 python -u tools/chain_ab.py base 3 > gpurun_out/r11/chain_base.log 2>&1 && cat gpurun_out/r11/chain_base.log
timeout -k 10 400 python -u tools/e1_shapes.py 3 0:0:0:0 8:1:0:0 8:2:0:0 16:1:0:0 > gpurun_out/r11/e1.log 2>&1 && cat gpurun_out/r11/e1.log
