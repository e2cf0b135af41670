set -o pipefail
mkdir -p gpurun_out/r5
CFG=3 ITERS=1 LANES=1 timeout -k 10 300 python -u tools/stamps_split.py > gpurun_out/r5/stamps_lane.log 2>&1 || { tail -20 gpurun_out/r5/stamps_lane.log; exit 1; }
cat gpurun_out/r5/stamps_lane.log
CFG=3 ITERS=1 LANES=0 timeout -k 10 300 python -u tools/stamps_split.py > gpurun_out/r5/stamps_seg.log 2>&1 || { tail -20 gpurun_out/r5/stamps_seg.log; exit 1; }
cat gpurun_out/r5/stamps_seg.log
