# multi-rank rehearsal on the final library: cfg 2 with 1, 4 and 8 ranks on one GPU (gloo host collective),
# every step's LL and pattern count must equal the one-rank chain
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r8l
mkdir -p $D
C="--config 2 --steps 4 --warmup 1 --steady-steps 0 --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $C > $D/n1.json 2> $D/n1.err || { tail -5 $D/n1.err; exit 1; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 $C --trace-bytes 8000000000 --collective host > $D/n4.json 2> $D/n4.err || { tail -5 $D/n4.err; exit 2; }
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 8 $C --trace-bytes 4000000000 --collective host > $D/n8.json 2> $D/n8.err || { tail -5 $D/n8.err; exit 3; }
python3 - <<'PY'
import json
D="gpurun_out/r8l"
L={n: json.loads(open(f"{D}/n{n}.json").read().strip().splitlines()[-1]) for n in (1,4,8)}
ref=[(s["ll"], s["P"]) for s in L[1]["per_step"]]
for n in (4,8):
    got=[(s["ll"], s["P"]) for s in L[n]["per_step"]]
    print(n, "ranks: steps equal to one rank:", got == ref, "m0 patterns equal:", L[n]["m0"]["patterns"] == L[1]["m0"]["patterns"], L[n]["config"]["parallelism"])
print("one rank:", ref)
PY
