set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r17
HMC_DEBUG_MEM=1 timeout -k 10 400 python -u tools/e1_shapes.py 3 0:0:0:0 8:2:0:0 8:1:0:0 4:2:0:0 0:0:12:1 0:0:6:2 0:0:8:2 8:2:0:0 > gpurun_out/r17/e1_sweep.log 2> gpurun_out/r17/e1_sweep.err
