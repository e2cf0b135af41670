set -o pipefail
mkdir -p gpurun_out/r18
timeout -k 10 1100 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu -k "full_size or cfg4 or exact_em or exact_mstep" > gpurun_out/r18/tests_b.log 2>&1 || { tail -40 gpurun_out/r18/tests_b.log; exit 1; }
tail -3 gpurun_out/r18/tests_b.log
