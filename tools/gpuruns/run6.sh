set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r6/tests.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 600 python -u tools/e1_shapes.py 3 0:0:0:0 0:0:0:0 1:0:0:0 4:2:0:0 4:4:0:0 > gpurun_out/r6/e1.log 2> gpurun_out/r6/e1.err && \
timeout -k 10 400 python -u tools/s1_stamps.py 3 2 > gpurun_out/r6/s1_stamps.log 2> gpurun_out/r6/s1_stamps.err
