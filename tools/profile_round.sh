#!/bin/bash
# Profile set for one round (run on the GPU box from the repo root):
#   PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) on the dominant kernel
#   estep_values, kernel-trace stats, and the bench line, all of the same
#   command.  Summaries are copied to profiles/<TAG>/ and
#   profiles/pmc_estep_values.json (read by bench.py for roofline.traffic).
# usage: bash tools/profile_round.sh OUTDIR TAG   (copy OUTDIR/commit/TAG to profiles/TAG afterwards)
set -euo pipefail
OUT=${1:-gpurun_out/prof}
TAG=${2:-r01}
DEST=$OUT/commit/$TAG
mkdir -p "$OUT" "$DEST"
export TMPDIR=/tmp
K=estep_values
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv \
  -d "$OUT/pmc_fetch" -o f -- python3 bench.py --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv \
  -d "$OUT/pmc_write" -o w -- python3 bench.py --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
FC=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" | head -n 1)
WC=$(find "$OUT/pmc_write" -name "*counter_collection.csv" | head -n 1)
python3 tools/pmc_traffic.py "$FC" "$WC" \
  $K "$OUT/pmc_$K.json" "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) --kernel-include-regex $K -- python3 bench.py --no-cpu-baseline"
cp "$OUT/pmc_$K.json" profiles/pmc_$K.json
cp "$OUT/pmc_$K.json" "$DEST/"
cp "$FC" "$DEST/pmc_fetch_size.csv"
cp "$WC" "$DEST/pmc_write_size.csv"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --no-cpu-baseline > "$OUT/trace.log" 2>&1
cp "$(find "$OUT/trace" -name "*kernel_stats.csv" | head -n 1)" "$DEST/kernel_stats.csv"
tail -1 "$OUT/trace.log" > "$DEST/bench_under_rocprof.json"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -1 "$OUT/bench.json" > "$DEST/bench.json"
tail -1 "$OUT/bench.json"
