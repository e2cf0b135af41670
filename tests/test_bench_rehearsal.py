"""bench.py's multi-rank path end to end on one GPU, with every rank on device
0 and the gloo host collective in place of RCCL (`--collective host`): the
driver's launch (`torch.distributed.run --nproc-per-node N bench.py --gpus N`)
and bench.py's own launch of N ranks when no launcher set WORLD_SIZE.  The
sharded EM with the ordered reduction must reproduce the one-rank chain
exactly (LL and pattern count of every step), and the timed steps must follow
the reference's converged chain (restart from M0 after the stop)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--config", "2", "--steps", "4", "--warmup", "1", "--steady-steps", "0", "--no-cpu-baseline",
          "--trace-bytes", "16000000000"]


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


@pytest.fixture(scope="module")
def one_rank():
    return _run([sys.executable, "bench.py", *COMMON])


def test_bench_steps_follow_the_converged_chain(one_rank):
    # cfg 2 stops after E3 (LL rises, then drops at iteration 3)
    assert [s["iteration"] for s in one_rank["per_step"]] == [1, 2, 3, 1]
    assert [s["go"] for s in one_rank["per_step"]] == [True, True, False, True]
    assert one_rank["per_step"][2]["mstep_ms"] == 0.0
    assert one_rank["per_step"][3]["ll"] == one_rank["per_step"][0]["ll"]  # the restart is E1 again
    assert one_rank["chain"]["iterations"] == [3]
    assert one_rank["library"]["path"].endswith("libhmc_amd.so")


def test_bench_two_ranks_equal_one(one_rank):
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                *COMMON, "--collective", "host"])
    assert one_rank["n_gpus"] == 1 and two["n_gpus"] == 2
    assert "REHEARSAL" in two["config"]["parallelism"]
    assert [(s["ll"], s["P"]) for s in two["per_step"]] == [(s["ll"], s["P"]) for s in one_rank["per_step"]]
    assert two["m0"]["patterns"] == one_rank["m0"]["patterns"]


def test_bench_spawns_ranks_without_launcher(one_rank):
    """`python bench.py --gpus 2` with no WORLD_SIZE: bench.py starts the two
    ranks itself (fresh processes, before any GPU call)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *COMMON, "--collective", "host"], cwd=ROOT,
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    two = _last_json(r.stdout)
    assert two["n_gpus"] == 2
    assert [(s["ll"], s["P"]) for s in two["per_step"]] == [(s["ll"], s["P"]) for s in one_rank["per_step"]]


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *COMMON], cwd=ROOT, capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2
