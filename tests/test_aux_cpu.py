"""Auxiliary subsystems on CPU: collective fingerprints, fault injection,
checkpoint layout and --resume."""
import os
import subprocess
import sys

import torch

from dist_helpers import ROOT, run_workers
from dist_workers import worker_coll_mismatch

TINY = ["--synthetic_data", "--batch_size", "4", "--epochs", "1", "--sequence_length", "32",
        "--dim", "32", "--heads", "2", "--head_dim", "16", "--num_layers", "2",
        "--train_samples", "64", "--val_samples", "8", "--num_workers", "0", "--no_generate", "--cpu"]


def test_collective_fingerprint_catches_mismatch():
    run_workers(worker_coll_mismatch, 2)


def test_fault_injection_then_resume(tmp_path):
    """DPC_FAULT_STEP kills the run mid-epoch; --save_every left a checkpoint behind, and
    --resume latest restores weights, AdamW moments and the step count from it."""
    ck = tmp_path / "ckpt"
    env = dict(os.environ, DPC_FAULT_STEP="5", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main-single.py"), *TINY, "--max_steps", "8",
                        "--save_every", "2", "--checkpoint_dir", str(ck)],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 13, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "[fault-injection]" in r.stdout

    from distributed_pytorch_cookbook_amd.recipes import run
    from distributed_pytorch_cookbook_amd.utils.checkpoint import latest_checkpoint, load_model_state, load_train_state

    path = latest_checkpoint(str(ck))
    assert path is not None
    sd = load_model_state(path)
    assert len(sd) == 13 * 2 + 5 and not any(k.startswith(("module.", "_orig_mod.")) for k in sd)
    st = load_train_state(path)
    assert st is not None and int(st["optimizer"]["step"]) == 4  # saved at steps 2 and 4
    assert st["optimizer"]["exp_avg"].abs().sum() > 0 and "rng" in st
    # --max_steps counts batches of the epoch: the resumed run skips the 4 already trained
    trainer, _ = run("single", [*TINY, "--max_steps", "6", "--resume", "latest", "--checkpoint_dir", str(ck),
                                "--no_save"])
    assert trainer.engine.step_count == 4 + 2
    w = dict(trainer.engine.lm().state_dict())["lm_head.weight"]
    assert torch.isfinite(w).all()


def test_resume_mid_epoch_matches_uninterrupted(tmp_path):
    """A run killed mid-epoch and resumed from its --save_every checkpoint trains the same
    batches, in the same order, as an uninterrupted run: identical final weights."""
    from distributed_pytorch_cookbook_amd.recipes import run

    full, _ = run("single", [*TINY, "--max_steps", "8", "--no_save"])
    w_full = {k: v.detach().clone() for k, v in full.engine.lm().state_dict().items()}
    ck = tmp_path / "ckpt"
    env = dict(os.environ, DPC_FAULT_STEP="5", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main-single.py"), *TINY, "--max_steps", "8",
                        "--save_every", "2", "--checkpoint_dir", str(ck)],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 13, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    resumed, _ = run("single", [*TINY, "--max_steps", "8", "--resume", "latest", "--checkpoint_dir", str(ck),
                                "--no_save"])
    assert resumed.skip_batches == 4 and resumed.engine.step_count == 8
    w_res = resumed.engine.lm().state_dict()
    for k, v in w_full.items():
        assert torch.equal(v, w_res[k]), k


def test_debug_switches_set_runtime_env(monkeypatch):
    """--serialize_kernels sets the HIP serialisation switches (before the
    runtime starts) and turns on per-launch synchronisation; --stream_check / --coll_check
    arm the transport and collective checks."""
    from distributed_pytorch_cookbook_amd import recipes
    from distributed_pytorch_cookbook_amd.config import parse
    from distributed_pytorch_cookbook_amd.ops import _lib
    from distributed_pytorch_cookbook_amd.parallel import comm, transport

    for k in ("AMD_SERIALIZE_KERNEL", "AMD_SERIALIZE_COPY", "HIP_LAUNCH_BLOCKING", "DPC_SERIALIZE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(_lib, "SERIALIZE", False)
    args = parse("ddp", ["--serialize_kernels", "--stream_check", "--coll_check"])
    try:
        recipes.apply_debug_switches(args)
        import os

        assert os.environ["AMD_SERIALIZE_KERNEL"] == "3" and os.environ["HIP_LAUNCH_BLOCKING"] == "1"
        assert _lib.SERIALIZE and transport.stream_check_enabled() and comm._CHECK
    finally:
        transport.set_stream_check(False)
        comm.set_coll_check(False)


def test_native_loader_seek_matches_stream(tmp_path):
    """Batches of the native token-file loader are a pure function of their index: seeking to
    batch k yields exactly what the k-th ``next`` of a fresh stream yields."""
    from distributed_pytorch_cookbook_amd.runtime import NativeBatchLoader, TokenFile, write_token_file

    path = str(tmp_path / "tok.bin")
    write_token_file(path, torch.randint(0, 50000, (20000,)).tolist())
    tf = TokenFile(path)
    a = NativeBatchLoader(tf, 4, 33, seed=5)
    stream = [next(a)["input_ids"] for _ in range(7)]
    b = NativeBatchLoader(tf, 4, 33, seed=5)
    b.seek(3)
    assert all(torch.equal(next(b)["input_ids"], stream[k]) for k in range(3, 7))
    b.seek(1)
    assert torch.equal(next(b)["input_ids"], stream[1])
    a.close(), b.close()


def test_data_path_resume_across_epochs_matches_uninterrupted(tmp_path):
    """--data_path (native loader) killed in epoch 2 and resumed: the resumed run seeks to the
    global batch it stopped at and ends with the uninterrupted run's weights."""
    from distributed_pytorch_cookbook_amd.recipes import run
    from distributed_pytorch_cookbook_amd.runtime import write_token_file

    tok = str(tmp_path / "corpus.bin")
    g = torch.Generator().manual_seed(0)
    write_token_file(tok, torch.randint(0, 50000, (40000,), generator=g).tolist())
    args = [*TINY, "--data_path", tok, "--train_samples", "32", "--epochs", "2", "--eval_steps", "1"]
    args[args.index("--epochs") + 1] = "2"  # (TINY's own --epochs 1 comes first; argparse keeps the last)
    full, _ = run("single", [*args, "--no_save"])  # 8 steps per epoch
    w_full = {k: v.detach().clone() for k, v in full.engine.lm().state_dict().items()}
    ck = tmp_path / "ckpt"
    env = dict(os.environ, DPC_FAULT_STEP="13", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main-single.py"), *args, "--save_every", "3",
                        "--checkpoint_dir", str(ck)], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 13, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    resumed, _ = run("single", [*args, "--resume", "latest", "--checkpoint_dir", str(ck), "--no_save"])
    assert resumed.start_epoch == 1 and resumed.skip_batches == 4 and resumed.engine.step_count == 16
    w_res = resumed.engine.lm().state_dict()
    for k, v in w_full.items():
        assert torch.equal(v, w_res[k]), k


def test_checkpoint_names_never_collide(tmp_path):
    from distributed_pytorch_cookbook_amd.utils.checkpoint import latest_checkpoint, save_model_state

    sd = {"w": torch.ones(2)}
    a = save_model_state(sd, str(tmp_path), stamp="2026-01-01_00-00-00")
    b = save_model_state({"w": torch.zeros(2)}, str(tmp_path), stamp="2026-01-01_00-00-00")
    c = save_model_state(sd, str(tmp_path), stamp="2026-01-01_00-00-00", step=6)
    assert len({a, b, c}) == 3 and a.name == "checkpoint-2026-01-01_00-00-00.pt"
    assert c.name == "checkpoint-2026-01-01_00-00-00_step6.pt"
    assert latest_checkpoint(str(tmp_path)) == c


def test_pipeline_default_microbatches_divide_the_batch():
    """Default micro-batch count: the largest divisor of the per-replica batch <= 4 x stages
    (batch 64 at pp 3 -> 8, not a ValueError)."""
    from types import SimpleNamespace

    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine

    f = PipelineEngine._micro_count
    assert f(SimpleNamespace(n_micro_req=0, pp=3), 64) == 8
    # the zero-bubble schedules: at most 2 x stages (profiles/r6_pp/)
    assert f(SimpleNamespace(n_micro_req=0, pp=8, _mfac=2), 512) == 16
    assert f(SimpleNamespace(n_micro_req=0, pp=8), 512) == 32
    assert f(SimpleNamespace(n_micro_req=0, pp=2), 128) == 8
    assert f(SimpleNamespace(n_micro_req=0, pp=5), 36) == 18
    assert f(SimpleNamespace(n_micro_req=0, pp=1), 64) == 1
    assert f(SimpleNamespace(n_micro_req=6, pp=2), 36) == 6


def test_phase_ranges_cover_every_engine(monkeypatch):
    """roctx ranges around the step phases (fwd / bwd / optim, comm waits) in
    every engine's eager step -- recorded here by replacing the range helper."""
    import contextlib

    from distributed_pytorch_cookbook_amd.engine import data_parallel, fsdp, pipeline
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine

    from dist_workers import full_batch, make_model

    seen = []

    @contextlib.contextmanager
    def rec(name):
        seen.append(name)
        yield

    for mod in (data_parallel, fsdp, pipeline):
        monkeypatch.setattr(mod, "mark", rec)
    for build in (lambda m: DataParallelEngine(m, "cpu", lr=1e-3),
                  lambda m: FSDPEngine(m, "cpu", lr=1e-3),
                  lambda m: PipelineEngine(m, "cpu", lr=1e-3, pp=1)):
        seen.clear()
        eng = build(make_model())
        eng.train_step(*full_batch())
        names = {n.split(" ")[0] for n in seen}
        assert {"fwd", "bwd", "optim"} <= names, seen


def test_attention_span_check_rejects_4gib_sequences():
    """The bf16 attention kernels use 32-bit row offsets per sequence (attention.hip:rows_rsrc):
    a sequence whose rows would span >= 4 GiB is refused with a clear error before any launch;
    the f32 kernels keep 64-bit offsets and are not limited."""
    import pytest

    from distributed_pytorch_cookbook_amd.ops.attention import _check_span

    bf = torch.empty(1, dtype=torch.bfloat16)
    _check_span(bf, 1023, 2304, 768)  # GPT-2 small: ~4.7 MB per sequence
    _check_span(bf, 131072, 3 * 4096, 4096)  # 128K tokens of a 4096-wide model: ~3.2 GB
    with pytest.raises(ValueError, match="4 GiB"):
        _check_span(bf, 200000, 3 * 4096, 4096)
    _check_span(torch.empty(1), 200000, 3 * 4096, 4096)
