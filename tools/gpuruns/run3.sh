set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
HMC_DEBUG_MEM=1 timeout -k 10 900 python -u tools/e1_shapes.py 3 0:0:0 0:4:4 0:3:6 0:2:10 0:1:20 0:4:5 8:0:0 16:0:0 0:0:0:150:100 0:4:4:150:100 > gpurun_out/r3/e1.log 2> gpurun_out/r3/e1.err
