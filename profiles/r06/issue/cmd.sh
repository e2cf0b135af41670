set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6b; mkdir -p $O
cd $R
export TMPDIR=/tmp
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64"
BUSY="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
MIX2="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
timeout -k 10 120 ./tools/diag/issue_bench 2048 > $O/issue_cpi.json 2> $O/issue.err || exit 11
echo issue done
for P in MIX BUSY MIX2; do
  timeout -s KILL 90 rocprofv3 --pmc ${!P} --output-format csv -d $O/ib_$P -o s -- ./tools/diag/issue_bench 1024 > $O/ib_$P.json 2> $O/ib_$P.err || exit 12
done
echo issue pmc done
timeout -k 10 120 ./tools/diag/coop_bench 32 2000 5 10 > $O/coop.txt 2>&1 || exit 13
for P in MIX BUSY MIX2; do
  timeout -s KILL 90 rocprofv3 --pmc ${!P} --kernel-include-regex bench_seg2e --output-format csv -d $O/cb_$P -o s -- ./tools/diag/coop_bench 32 2000 5 10 > $O/cb_$P.txt 2> $O/cb_$P.err || exit 14
done
echo coop pmc done
SHORT="bench.py --config 3 --no-cpu-baseline --steps 2 --warmup 0 --steady-steps 0"
for P in MIX BUSY MIX2; do
  timeout -s KILL 300 rocprofv3 --pmc ${!P} --kernel-include-regex "estep_values|estep_structure" --output-format csv -d $O/b3_$P -o s -- python3 $SHORT > $O/b3_$P.json 2> $O/b3_$P.err || exit 15
  echo "bench pass $P done"
done
timeout -k 10 600 python3 bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 16
echo ok
