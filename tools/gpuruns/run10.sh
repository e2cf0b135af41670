set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r10
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r10/tests.log 2>&1 && \
CFG=2 timeout -k 10 200 python -u tools/exact_time.py > gpurun_out/r10/exact_cfg2.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 240 python -u tools/cfg4_m0.py > gpurun_out/r10/cfg4_m0.log 2>&1
