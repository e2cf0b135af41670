set -o pipefail
mkdir -p gpurun_out/r21
B=tools/diag/coop_bench
for w in 2 16 32 40; do
  for mode in 5 7; do
    timeout -k 5 60 $B $w 300 $mode 10 >> gpurun_out/r21/coop.log 2>&1 || { echo "fail w=$w mode=$mode"; cat gpurun_out/r21/coop.log; exit 1; }
  done
done
for S in 3 7 16; do for mode in 5 7; do timeout -k 5 60 $B 32 200 $mode $S >> gpurun_out/r21/coop.log 2>&1 || exit 1; done; done
cat gpurun_out/r21/coop.log
