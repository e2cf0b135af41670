set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r8
timeout -k 10 1500 python -u -m pytest -x -v --timeout 1100 --timeout-method thread tests -m gpu > gpurun_out/r8/tests.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 900 python -u tools/cfg4_m0.py > gpurun_out/r8/cfg4_m0.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 900 python -u tools/shard_mstep.py 4 8 > gpurun_out/r8/shard_cfg4_w8.log 2>&1
