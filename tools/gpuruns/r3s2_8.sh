set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r8
SKIP_SQ= timeout -k 10 1000 bash tools/profile_round.sh gpurun_out/r8/prof r03 3 > gpurun_out/r8/profile.log 2>&1 || { tail -20 gpurun_out/r8/profile.log; exit 1; }
cp gpurun_out/r8/prof/commit/r03/pmc_estep_values_cfg3.json profiles/r03/pmc_estep_values_cfg3.json
timeout -k 10 400 python -u bench.py > gpurun_out/r8/bench.json 2> gpurun_out/r8/bench.err || { tail -20 gpurun_out/r8/bench.err; exit 1; }
tail -1 gpurun_out/r8/bench.json
