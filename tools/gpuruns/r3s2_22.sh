set -o pipefail
mkdir -p gpurun_out/r22
CFG=3 ITERS=3 timeout -k 10 400 python -u tools/stamps_split.py > gpurun_out/r22/stamps_pair.log 2>&1 || { tail -20 gpurun_out/r22/stamps_pair.log; exit 1; }
cat gpurun_out/r22/stamps_pair.log
