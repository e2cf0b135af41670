set -o pipefail
mkdir -p gpurun_out/r19
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r19/smoke.log 2>&1 || { tail -20 gpurun_out/r19/smoke.log; exit 1; }
tail -1 gpurun_out/r19/smoke.log
timeout -k 10 400 python -u tools/e1_shapes.py 3 0:0:0:0 0:0:10:2 0:0:5:4 0:0:16:1 0:0:4:5 0:0:0:0 > gpurun_out/r19/e1.log 2>&1 && cat gpurun_out/r19/e1.log
