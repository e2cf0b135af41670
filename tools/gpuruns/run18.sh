set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r18
timeout -k 10 750 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r18/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r18/bench.json 2> gpurun_out/r18/bench.err
