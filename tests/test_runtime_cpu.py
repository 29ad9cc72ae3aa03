"""Native host runtime (C++): loader, synthetic corpus, host AdamW; recipe with --data_path."""
import numpy as np
import torch

from distributed_pytorch_cookbook_amd import runtime as R


def test_synth_markov_deterministic_and_structured():
    a = R.synth_markov(8, 257, vocab=50257, seed=3)
    b = R.synth_markov(8, 257, vocab=50257, seed=3)
    c = R.synth_markov(2, 257, vocab=50257, seed=3, row0=4)
    assert torch.equal(a, b) and torch.equal(a[4:6], c)
    assert a.min() >= 0 and a.max() < 50257
    # a Markov chain with 4 successors per token: bigram diversity far below uniform
    pairs = set(zip(a[:, :-1].reshape(-1).tolist(), a[:, 1:].reshape(-1).tolist()))
    assert len(pairs) < 0.5 * a[:, 1:].numel()


def test_token_file_loader(tmp_path):
    toks = np.arange(100000, dtype=np.uint16) % 50000
    path = tmp_path / "c.bin"
    toks.tofile(path)
    tf = R.TokenFile(str(path))
    assert len(tf) == 100000
    l0 = R.NativeBatchLoader(tf, 4, 65, seed=1, rank=0, world=2, threads=3)
    l1 = R.NativeBatchLoader(tf, 4, 65, seed=1, rank=1, world=2, threads=2)
    b0 = [next(l0)["input_ids"] for _ in range(3)]
    b1 = next(l1)["input_ids"]
    for b in b0:
        assert b.shape == (4, 65)
        d = (b[:, 1:] - b[:, :-1]) % 50000
        assert bool((d == 1).all())  # contiguous windows of the file
    assert not torch.equal(b0[0], b1)  # ranks read different windows
    l2 = R.NativeBatchLoader(tf, 4, 65, seed=1, rank=0, world=2, threads=1)
    assert torch.equal(next(l2)["input_ids"], b0[0])  # deterministic, thread-count independent
    for l in (l0, l1, l2):
        l.close()
    tf.close()


def test_host_adamw_matches_torch():
    n = 5000
    p = torch.randn(n)
    g = torch.randn(n)
    m, v = torch.zeros(n), torch.zeros(n)
    sh = torch.empty(n, dtype=torch.bfloat16)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pr], lr=3e-3)
    for s in range(1, 5):
        g.normal_()
        pr.grad = g.clone()
        opt.step()
        R.adamw_host(p, g, m, v, 3e-3, 0.9, 0.999, 1e-8, 0.01, s, shadow=sh)
    assert (p - pr.detach()).abs().max().item() < 1e-6
    assert (sh.float() - p).abs().max().item() < 2e-2


def test_recipe_with_native_token_file(tmp_path, monkeypatch):
    from distributed_pytorch_cookbook_amd.recipes import run

    toks = R.synth_markov(64, 1024, vocab=50257, seed=5).numpy().astype(np.uint16) % 50257
    path = tmp_path / "corpus.bin"
    toks.reshape(-1).astype(np.uint16).tofile(path)
    monkeypatch.chdir(tmp_path)
    trainer, ckpt = run("single", ["--data_path", str(path), "--batch_size", "4", "--epochs", "1",
                                   "--sequence_length", "32", "--dim", "32", "--heads", "2",
                                   "--head_dim", "16", "--num_layers", "2", "--max_steps", "8",
                                   "--val_samples", "8", "--num_workers", "0", "--no_generate",
                                   "--cpu"])
    assert ckpt is not None and ckpt.exists()
    assert any("val_loss" in h for h in trainer.history)


def test_train_flops_per_token_matches_survey_table():
    """GPT-2 small 0.86, XL 10.28 GFLOP per trained token."""
    from distributed_pytorch_cookbook_amd.utils.metrics import mfu, train_flops_per_token

    assert abs(train_flops_per_token(768, 12, 64, 12, 50257, 1024) / 1e9 - 0.86) < 0.01
    assert abs(train_flops_per_token(1600, 25, 64, 48, 50257, 1024) / 1e9 - 10.28) < 0.05
    assert abs(mfu(1e6, 1e9) - 0.4) < 1e-9


def test_grad_scaler_cpu_semantics():
    """GradScaler on the host path: check / back-off / growth / skip (reference GradScaler)."""
    import torch

    from distributed_pytorch_cookbook_amd.ops.amp import GradScaler
    from distributed_pytorch_cookbook_amd.ops.optim import FlatAdamW

    sc = GradScaler("cpu", init_scale=8.0, growth_interval=2)
    p = torch.ones(16)
    g = torch.full((16,), 8.0)  # a scaled gradient of 1.0
    opt = FlatAdamW(p, g, lr=0.1, weight_decay=0.0)
    ref_p = torch.ones(16)
    ref = FlatAdamW(ref_p, torch.ones(16), lr=0.1, weight_decay=0.0)
    sc.check(g)
    opt.step(**sc.opt_kwargs(opt))
    sc.update()
    ref.step()
    assert torch.allclose(p, ref_p)
    g[3] = float("nan")
    sc.check(g)
    before = p.clone()
    opt.step(**sc.opt_kwargs(opt))
    sc.update()
    assert torch.equal(p, before) and float(sc.scale_t) == 4.0 and float(opt.step_t) == 1.0
    g[3] = 4.0
    for _ in range(2):
        sc.check(g)
        opt.step(**sc.opt_kwargs(opt))
        sc.update()
    assert float(sc.scale_t) == 8.0 and float(opt.step_t) == 3.0


def test_gemm_table_signature_and_file():
    """The measured GEMM table: signature format, and every entry names a real implementation."""
    import json
    import os

    from distributed_pytorch_cookbook_amd.ops import gemm as G
    sig = G._sig(65472, 3072, 768, True, False, False, None, 0, 2, None, None, object(), False)
    assert sig == "65472x3072x768:km:h:02:c"
    with open(G._TUNE_PATH) as f:
        table = json.load(f)["impl"]
    assert table and all(v in G._CANDIDATES for v in table.values())
    assert all(k.count(":") == 4 for k in table)
    assert os.path.dirname(G._TUNE_PATH).endswith("ops")


def test_gemm_table_nearest_token_dimension():
    """A product missing from the measured table takes the entry that differs only in its token
    dimension (M of a forward / dgrad, K of a weight gradient) by at most 25 %."""
    from distributed_pytorch_cookbook_amd.ops import gemm as G

    saved = (dict(G._table), dict(G._near_cache))
    try:
        G._table.clear()
        G._near_cache.clear()
        G._table.update({"65472x768x3072:kk:f:20:bxr": 6, "32736x768x3072:kk:f:20:bxr": 2,
                         "768x3072x65472:mm:f:00:a": 16, "65472x768x3072:kk:h:00:": 19})
        assert G._near("65528x768x3072:kk:f:20:bxr") == 6       # S = 8192: 8 x 8191 rows
        assert G._near("40000x768x3072:kk:f:20:bxr") == 2       # closer to 32736
        assert G._near("768x3072x65528:mm:f:00:a") == 16        # weight gradient: K = tokens
        assert G._near("65528x768x3072:kk:h:00:") == 19         # flags must match exactly
        assert G._near("65528x1024x3072:kk:f:20:bxr") is None   # another N
        assert G._near("16368x768x3072:kk:f:20:bxr") is None    # beyond 25 %
    finally:
        G._table.clear()
        G._table.update(saved[0])
        G._near_cache.clear()
        G._near_cache.update(saved[1])
