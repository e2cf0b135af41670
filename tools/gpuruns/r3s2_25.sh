set -o pipefail
mkdir -p gpurun_out/r25
timeout -k 10 400 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/r25/bench_cfg2.json 2> gpurun_out/r25/bench_cfg2.err || { tail -20 gpurun_out/r25/bench_cfg2.err; exit 1; }
timeout -k 10 500 python -u bench.py --config 5 --no-cpu-baseline > gpurun_out/r25/bench_cfg5.json 2> gpurun_out/r25/bench_cfg5.err || { tail -20 gpurun_out/r25/bench_cfg5.err; exit 1; }
python3 -c "
import json
for c in (2,5):
    d=json.loads(open('gpurun_out/r25/bench_cfg%d.json'%c).read().strip().split(chr(10))[-1])
    print(c, d['value'], d['ms_per_step'], d.get('value_chain'), d['chain'], d['roofline']['frac'])
"
