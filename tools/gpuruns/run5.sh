set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "many_alleles or mining_in_start_blocks or rewind or mine_genotypes or mine_level or long_patterns or find_pattern_by_num or full_em_models or exact_mstep or full_em" > gpurun_out/r5/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/s1_stamps.py 3 2 > gpurun_out/r5/s1_stamps.log 2> gpurun_out/r5/s1_stamps.err && \
HMC_DEBUG_MEM=1 timeout -k 10 600 python -u tools/e1_shapes.py 3 0:0:0 0:0:0 0:4:3 0:4:2 0:3:4 0:4:4:150:100 > gpurun_out/r5/e1.log 2> gpurun_out/r5/e1.err &&
CFG=2 timeout -k 10 300 python -u tools/exact_time.py > gpurun_out/r5/exact_cfg2.log 2>&1
