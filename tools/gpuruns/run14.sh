set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r14
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r14/tests.log 2>&1 && \
timeout -k 10 150 python -u tools/chain_ab.py cur > gpurun_out/r14/ab_cur.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 330 python -u tools/shard_mstep.py 4 8 > gpurun_out/r14/shard_cfg4_w8.log 2>&1
