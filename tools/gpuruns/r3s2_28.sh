set -o pipefail
mkdir -p gpurun_out/r28
timeout -k 10 900 python -u tools/shard_mstep.py 3 "1,2,4,8" > gpurun_out/r28/shard_cfg3.log 2>&1 || { tail -20 gpurun_out/r28/shard_cfg3.log; exit 1; }
grep -E "^W=|chain 1:" gpurun_out/r28/shard_cfg3.log
