set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r20
timeout -k 10 1100 bash tools/profile_round.sh gpurun_out/r20/prof r03 3 > gpurun_out/r20/profile.log 2>&1
