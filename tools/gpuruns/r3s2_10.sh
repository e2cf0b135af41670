set -o pipefail
mkdir -p gpurun_out/r10
timeout -k 10 400 python -u tools/e1_shapes.py 3 0:0:0:0 8:1:0:0 8:2:0:0 16:1:0:0 4:2:0:0 > gpurun_out/r10/e1.log 2>&1 || { tail -20 gpurun_out/r10/e1.log; exit 1; }
cat gpurun_out/r10/e1.log
