set -o pipefail
mkdir -p gpurun_out/r26
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "value_one_link_layout" > gpurun_out/r26/tests.log 2>&1 || { tail -40 gpurun_out/r26/tests.log; exit 1; }
tail -2 gpurun_out/r26/tests.log
