"""bench.py's multi-rank path end to end on one GPU: the driver's launch
(`torch.distributed.run --nproc-per-node N bench.py --gpus N`) with every rank
on device 0 and the gloo host collective in place of RCCL (`--collective
host`).  Sharded EM with the ordered reduction must reproduce the one-rank
chain exactly (LL and pattern count of every step)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--config", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--trace-bytes", "16000000000"]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out: str) -> dict:
    return json.loads(out.strip().splitlines()[-1])


def _run(cmd):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return _last_json(r.stdout)


def test_bench_two_ranks_equal_one():
    one = _run([sys.executable, "bench.py", *COMMON])
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                *COMMON, "--collective", "host"])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert "REHEARSAL" in two["config"]["parallelism"]
    assert [(s["ll"], s["P"]) for s in two["per_step"]] == [(s["ll"], s["P"]) for s in one["per_step"]]
    assert two["m0"]["patterns"] == one["m0"]["patterns"]
