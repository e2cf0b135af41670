set -o pipefail
mkdir -p gpurun_out/r9
timeout -k 10 300 python -u tools/steady_shapes.py 3 0:0 1:24 1:20 2:12 0:0 > gpurun_out/r9/steady.log 2>&1 || { tail -20 gpurun_out/r9/steady.log; exit 1; }
cat gpurun_out/r9/steady.log
timeout -k 10 300 python -u tools/e1_shapes.py 3 0:0:0:0 0:0:8:3 0:0:4:6 0:0:0:0 > gpurun_out/r9/e1.log 2>&1 || { tail -20 gpurun_out/r9/e1.log; exit 1; }
cat gpurun_out/r9/e1.log
