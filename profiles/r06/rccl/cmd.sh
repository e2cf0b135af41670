set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6a; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "rccl" > $O/rccl.log 2>&1 || exit 11
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_windows.py -k "overflow_shrinks" > $O/win.log 2>&1 || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --rccl-trace --kernel-trace --stats --output-format csv -d $O/trace -o rccl -- python3 -m pytest -x -q -p no:cacheprovider $R/tests/test_gpu_parity.py -k "rccl_send_recv_chain_full_em and cfg1" > $O/trace.log 2>&1 || exit 13
echo ok
