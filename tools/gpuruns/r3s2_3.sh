set -o pipefail
mkdir -p gpurun_out/r3
B=tools/diag/coop_bench
for w in 2 4 8 10; do
  for mode in 2 3; do
    timeout -k 5 60 $B $w 200 $mode 10 >> gpurun_out/r3/coop.log 2>&1 || { echo "fail w=$w mode=$mode"; cat gpurun_out/r3/coop.log; exit 1; }
  done
done
for w in 16 20; do timeout -k 5 60 $B $w 200 0 10 >> gpurun_out/r3/coop.log 2>&1 || exit 1; done
cat gpurun_out/r3/coop.log
