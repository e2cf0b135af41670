set -o pipefail
mkdir -p gpurun_out/r14
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "estep_pass_shapes" > gpurun_out/r14/tests.log 2>&1 || { tail -40 gpurun_out/r14/tests.log; exit 1; }
tail -2 gpurun_out/r14/tests.log
timeout -k 10 300 python -u tools/steady_shapes.py 3 1:12:0:0 1:16:0:0 1:20:0:0 1:12:0:0 > gpurun_out/r14/steady.log 2>&1 && cat gpurun_out/r14/steady.log
timeout -k 10 300 python -u tools/e1_shapes.py 3 0:0:0:0 4:4:0:0 4:3:0:0 > gpurun_out/r14/e1.log 2>&1 && cat gpurun_out/r14/e1.log
