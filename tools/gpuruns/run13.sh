set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r13
CFG=3 HMC_DEBUG_MEM=1 timeout -k 10 1000 python -u tools/exact_time.py > gpurun_out/r13/exact_cfg3.log 2> gpurun_out/r13/exact_cfg3.err
