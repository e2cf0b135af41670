#!/bin/bash
# Profile set for one round (run on the GPU box from the repo root):
#   PMC FETCH_SIZE / WRITE_SIZE passes on estep_forward, kernel-trace stats, bench line.
# usage: bash tools/profile_round.sh OUTDIR
set -euo pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex estep_forward --output-format csv \
  -d "$OUT/pmc_fetch" -o f -- python3 bench.py --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex estep_forward --output-format csv \
  -d "$OUT/pmc_write" -o w -- python3 bench.py --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT/pmc_fetch/f_counter_collection.csv" "$OUT/pmc_write/w_counter_collection.csv" \
  estep_forward "$OUT/pmc_estep_forward.json" "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) --kernel-include-regex estep_forward -- $CMD"
cp "$OUT/pmc_estep_forward.json" profiles/pmc_estep_forward.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --no-cpu-baseline > "$OUT/trace.log" 2>&1
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -1 "$OUT/bench.json"
