set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u tools/s1_stamps.py 3 2 > gpurun_out/r4/s1_stamps.log 2> gpurun_out/r4/s1_stamps.err && \
HMC_DEBUG_MEM=1 timeout -k 10 600 python -u tools/e1_shapes.py 3 0:0:0 0:0:0 0:4:3 0:4:2 0:3:4 0:4:4:150:100 > gpurun_out/r4/e1.log 2> gpurun_out/r4/e1.err
