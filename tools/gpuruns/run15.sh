set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r15
HMC_DEBUG_MEM=1 timeout -k 10 300 python -u tools/e1_shapes.py 3 0:0:0:0 0:0:16:1 0:0:8:2 16:1:0:0 0:0:0:0 > gpurun_out/r15/e1_wide.log 2> gpurun_out/r15/e1_wide.err && \
CFG=3 HMC_DEBUG_MEM=1 timeout -k 10 800 python -u tools/exact_time.py > gpurun_out/r15/exact_cfg3.log 2> gpurun_out/r15/exact_cfg3.err
