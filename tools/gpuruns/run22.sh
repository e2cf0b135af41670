set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r22
HMC_DEBUG_MEM=1 timeout -k 10 300 python -u tools/e1_shapes.py 3 0:0:0:0 0:0:10:2 0:0:5:4 0:0:20:1 0:0:0:0 > gpurun_out/r22/e1_wpe5.log 2> gpurun_out/r22/e1_wpe5.err
