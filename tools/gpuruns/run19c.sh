set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r19
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -k "exact" > gpurun_out/r19/tests_fix.log 2>&1 && \
CFG=2 HMC_DEBUG_MEM=1 timeout -k 10 200 python -u tools/exact_time.py > gpurun_out/r19/exact_cfg2.log 2> gpurun_out/r19/exact_cfg2.err && \
CFG=3 HMC_DEBUG_MEM=1 timeout -k 10 600 python -u tools/exact_time.py > gpurun_out/r19/exact_cfg3.log 2> gpurun_out/r19/exact_cfg3.err
