#!/bin/bash
# Counters of the exact M-step's trie walk (exact_walk) on a config (run on
# the GPU box from the repo root): the SQ instruction mix / wave states and
# LDS passes, the HBM fetch and write passes, each a separate rocprofv3 run of
# tools/exact_time.py, and the kernel-trace stats.
# usage: bash tools/profile_exact.sh OUTDIR CONFIG   -> OUTDIR/commit/
set -euo pipefail
OUT=${1:-gpurun_out/prof_exact}
CFG=${2:-2}
DEST=$OUT/commit
mkdir -p "$OUT" "$DEST"
export TMPDIR=/tmp CFG
K=exact_walk
P=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  P=$((P + 1))
  N=$(echo "$C" | awk '{print $1}')
  echo "[profile-exact] pass $P: $N" >&2
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$K" --output-format csv -d "$OUT/p$P" -o x -- \
    python3 tools/exact_time.py > "$OUT/p$P.log" 2> "$OUT/p$P.err"
  cp "$(find "$OUT/p$P" -name "*counter_collection.csv" | head -n 1)" "$DEST/exact_${N}_cfg$CFG.csv"
  cp "$OUT/p$P.log" "$DEST/exact_${N}_cfg$CFG.log"
done
echo "[profile-exact] kernel trace" >&2
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
  python3 tools/exact_time.py > "$OUT/trace.log" 2> "$OUT/trace.err"
cp "$(find "$OUT/trace" -name "*kernel_stats.csv" | head -n 1)" "$DEST/exact_kernel_stats_cfg$CFG.csv"
python3 tools/sq_summary.py "$DEST/exact_SQ_WAVES_cfg$CFG.csv" "$DEST/exact_SQ_INSTS_LDS_cfg$CFG.csv" "$K" > "$DEST/exact_sq_summary_cfg$CFG.md"
echo "[profile-exact] done" >&2
