set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r11
timeout -k 10 500 python -u bench.py > gpurun_out/r11/bench.json 2> gpurun_out/r11/bench.err && \
timeout -k 10 400 python -u tools/shard_mstep.py 3 1,2,4,8 > gpurun_out/r11/shard_cfg3.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 400 python -u tools/shard_mstep.py 4 8 > gpurun_out/r11/shard_cfg4_w8.log 2>&1 && \
HMC_DEBUG_MEM=1 timeout -k 10 300 python -u tools/e1_shapes.py 3 4:3:0:0 4:2:0:0 4:3:0:0 4:2:0:0 4:1:0:0 > gpurun_out/r11/e1_s1shapes.log 2> gpurun_out/r11/e1_s1shapes.err && \
CFG=2 HMC_DEBUG_MEM=1 timeout -k 10 200 python -u tools/exact_time.py > gpurun_out/r11/exact_cfg2.log 2> gpurun_out/r11/exact_cfg2.err
