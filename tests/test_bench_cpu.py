"""bench.py's multi-rank contract on CPU (gloo, 2 ranks through torch.distributed.run, as the
driver launches it on a GPU node): one JSON line from rank 0 with the whole-job value, the
per-recipe parallelism string and the fields the driver reads."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("recipe,par", [("ddp", "dp2"), ("fsdp", "fsdp2"), ("pipe", "pp2"),
                                        ("pipe_ddp", "pp2xdp1")])
def test_bench_two_ranks_json_contract(recipe, par, tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--recipe", recipe, "--model", "ref",
           "--batch_size", "8", "--seq_len", "64"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == par
    assert out["value"] > 0 and out["ms_per_step"] > 0
    tok = out["config"]["tokens_per_step"]
    assert out["value"] == pytest.approx(tok * 2 / (2 * out["ms_per_step"] / 1000), rel=0.02)


@pytest.mark.parametrize("recipe,par", [("ddp", "dp2"), ("fsdp", "fsdp2"), ("pipe", "pp2"),
                                        ("pipe_ddp", "pp2xdp1")])
def test_bench_self_launches_n_ranks_without_torchrun(recipe, par, tmp_path):
    """`python bench.py --gpus 2` (no torchrun, WORLD_SIZE unset) must measure 2 ranks: the
    parent starts them as a torch.distributed.run child and relays rank 0's one line."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--recipe", recipe, "--model", "ref", "--batch_size", "8", "--seq_len", "64"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == par


def test_bench_refuses_world_size_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--model", "ref", "--batch_size", "2", "--seq_len", "32"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
