#!/bin/bash
# Profile set for one round (run on the GPU box from the repo root):
#   HBM traffic of the dominant kernel estep_values from two separate PMC
#   passes (FETCH_SIZE, WRITE_SIZE) over the bench command itself, the
#   kernel-trace stats of the same command, and SQ counter passes (instruction
#   mix, LDS waits / bank conflicts, wave cycles, VALU issue busy incl. dual
#   issue, typed VALU mix) of both E-step passes on a short run.
# usage: bash tools/profile_round.sh OUTDIR TAG CONFIG
#   -> OUTDIR/commit/TAG/ (copy to profiles/TAG afterwards); the PMC summary is
#      profiles/TAG/pmc_estep_values_cfgCONFIG.json, which bench.py reads.
set -euo pipefail
OUT=${1:-gpurun_out/prof}
TAG=${2:-r02}
CFG=${3:-3}
DEST=$OUT/commit/$TAG
mkdir -p "$OUT" "$DEST"
export TMPDIR=/tmp
K=estep_values
BENCH="bench.py --config $CFG --no-cpu-baseline"
echo "[profile] FETCH_SIZE pass" >&2
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv \
  -d "$OUT/pmc_fetch" -o f -- python3 $BENCH > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
echo "[profile] WRITE_SIZE pass" >&2
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv \
  -d "$OUT/pmc_write" -o w -- python3 $BENCH > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
FC=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" | head -n 1)
WC=$(find "$OUT/pmc_write" -name "*counter_collection.csv" | head -n 1)
python3 tools/pmc_traffic.py "$FC" "$WC" $K "$DEST/pmc_${K}_cfg$CFG.json" \
  "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) --kernel-include-regex $K -- python3 $BENCH" \
  "$OUT/pmc_fetch.json" "$OUT/pmc_write.json"
cp "$FC" "$DEST/pmc_fetch_size_cfg$CFG.csv"
cp "$WC" "$DEST/pmc_write_size_cfg$CFG.csv"
echo "[profile] kernel trace" >&2
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 $BENCH > "$OUT/trace.json" 2> "$OUT/trace.err"
cp "$(find "$OUT/trace" -name "*kernel_stats.csv" | head -n 1)" "$DEST/kernel_stats_cfg$CFG.csv"
tail -1 "$OUT/trace.json" > "$DEST/bench_under_rocprof_cfg$CFG.json"
SHORT="bench.py --config $CFG --no-cpu-baseline --steps 2 --warmup 0"
[ -n "${SKIP_SQ:-}" ] && { echo "[profile] done (SQ passes skipped)" >&2; exit 0; }
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64"; do
  N=$(echo "$P" | awk '{print $1}')
  echo "[profile] SQ pass $N" >&2
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex "estep_values|estep_structure" --output-format csv -d "$OUT/sq_$N" -o s -- \
    python3 $SHORT > "$OUT/sq_$N.json" 2> "$OUT/sq_$N.err"
  cp "$(find "$OUT/sq_$N" -name "*counter_collection.csv" | head -n 1)" "$DEST/sq_${N}_cfg$CFG.csv"
done
python3 tools/sq_summary.py "$DEST/sq_SQ_WAVES_cfg$CFG.csv" "$DEST/sq_SQ_INSTS_LDS_cfg$CFG.csv" $K \
  "$DEST/sq_${K}_cfg$CFG.json" "$OUT/sq_SQ_WAVES.json" "$DEST/sq_SQ_ACTIVE_INST_VALU_cfg$CFG.csv" \
  "$DEST/sq_SQ_INSTS_VALU_INT32_cfg$CFG.csv"
echo "[profile] done" >&2
