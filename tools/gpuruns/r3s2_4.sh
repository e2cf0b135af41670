set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "value_lane_mode" > gpurun_out/r4/lane.log 2>&1 || { tail -40 gpurun_out/r4/lane.log; exit 1; }
tail -2 gpurun_out/r4/lane.log
timeout -k 10 300 python -u tools/chain_ab.py lane 3 > gpurun_out/r4/chain_lane.log 2>&1 || { tail -20 gpurun_out/r4/chain_lane.log; exit 1; }
cat gpurun_out/r4/chain_lane.log
