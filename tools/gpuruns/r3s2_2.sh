set -o pipefail
mkdir -p gpurun_out/r2
B=tools/diag/coop_bench
for w in 1 4 8; do
  for mode in 0 1 2 3; do
    timeout -k 5 60 $B $w 400 $mode 10 >> gpurun_out/r2/coop.log 2>&1 || { echo "fail w=$w mode=$mode"; cat gpurun_out/r2/coop.log; exit 1; }
  done
done
cat gpurun_out/r2/coop.log
