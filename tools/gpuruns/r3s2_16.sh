set -o pipefail
mkdir -p gpurun_out/r16
LAYOUT=2 timeout -k 10 300 python -u tools/steady_shapes.py 3 0:0 1:16 2:8 3:8 0:0 > gpurun_out/r16/steady_pair.log 2>&1 && cat gpurun_out/r16/steady_pair.log
LAYOUT=1 timeout -k 10 300 python -u tools/steady_shapes.py 3 0:0 0:0 > gpurun_out/r16/steady_base.log 2>&1 && cat gpurun_out/r16/steady_base.log
