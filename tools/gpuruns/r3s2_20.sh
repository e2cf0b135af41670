set -o pipefail
mkdir -p gpurun_out/r20
B=tools/diag/coop_bench
for w in 2 16 32 64; do
  for mode in 0 5 6; do
    timeout -k 5 60 $B $w 300 $mode 10 >> gpurun_out/r20/coop.log 2>&1 || { echo "fail w=$w mode=$mode"; cat gpurun_out/r20/coop.log; exit 1; }
  done
done
cat gpurun_out/r20/coop.log
