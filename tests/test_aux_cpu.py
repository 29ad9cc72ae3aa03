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
