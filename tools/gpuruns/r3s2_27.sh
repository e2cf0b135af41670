set -o pipefail
mkdir -p gpurun_out/r27
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r27/smoke.log 2>&1 || { tail -20 gpurun_out/r27/smoke.log; exit 1; }
tail -1 gpurun_out/r27/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "cfg2_full_size or segmented_nth or test_full_em or estep_on_reference_model" > gpurun_out/r27/tests.log 2>&1 || { tail -40 gpurun_out/r27/tests.log; exit 1; }
tail -2 gpurun_out/r27/tests.log
