set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_em_rewind_repeats_the_chain" "tests/test_gpu_parity.py::test_small_frontier_capacity_retries" tests/test_bench_rehearsal.py > gpurun_out/r2/tests.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 700 python -u bench.py > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err
