set -o pipefail
mkdir -p gpurun_out/r17
timeout -k 10 1100 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu -k "not full_size and not cfg4 and not exact_em and not exact_mstep" > gpurun_out/r17/tests_a.log 2>&1 || { tail -40 gpurun_out/r17/tests_a.log; exit 1; }
tail -3 gpurun_out/r17/tests_a.log
