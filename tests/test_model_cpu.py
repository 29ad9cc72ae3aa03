"""Model contract + fused-path correctness on CPU (f32 torch-op implementations of the ops).

The fused autograd functions (manual backward, gradients written into the flat store)
must match autograd through the reference math (``reference_forward`` +
``F.cross_entropy``) -- this is the oracle for the hand-derived backward.
"""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_cookbook_amd.models.gpt import PRESETS, FeedForward, TransformerDecoderLM
from distributed_pytorch_cookbook_amd.parallel.store import LocalStore


def tiny(act="relu", L=2, seed=0, D=64, H=4, hd=16, V=97, S=24):
    torch.manual_seed(seed)
    return TransformerDecoderLM(dim=D, head_dim=hd, heads=H, num_layers=L, vocab_size=V,
                                max_position_embeddings=S, activation=act)


def batch(N=3, S=24, V=97, pad=True, seed=1):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (N, S), generator=g)
    pos = torch.arange(S).repeat(N, 1)
    tg = torch.randint(0, V, (N, S), generator=g)
    mask = None
    if pad:
        mask = torch.zeros(N, S, dtype=torch.bool)
        mask[0, S - 5:] = True
        tg[0, S - 5:] = -100
    return ids, pos, mask, tg


def test_state_dict_keys_match_reference_layout():
    m = tiny(L=2)
    keys = list(m.state_dict().keys())
    assert len(keys) == 13 * 2 + 5
    assert keys[0] == "embeddings.input_embeddings.weight"
    assert "decoder.layers.1.attn.to_q.weight" in keys
    assert "decoder.layers.0.fc.up_proj.bias" in keys
    assert "norm_out.weight" in keys and keys[-1] == "lm_head.weight"
    assert not any(k.startswith(("module.", "_orig_mod.")) for k in keys)


@pytest.mark.parametrize("name,params", [("ref", 32.1e6), ("gpt2-small", 163.0e6), ("gpt2-xl", 1637.8e6)])
def test_preset_param_counts(name, params):
    p = PRESETS[name]
    with torch.device("meta"):
        m = TransformerDecoderLM(p["dim"], p["head_dim"], p["heads"], p["num_layers"], 50257,
                                 p["sequence_length"])
    n = sum(x.numel() for x in m.parameters())
    assert abs(n - params) / params < 0.002


def test_feedforward_double_activation_quirk():
    ff = FeedForward(16)
    assert ff(torch.randn(4, 16)).min().item() >= 0.0


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_fused_logits_match_reference(act):
    m = tiny(act)
    ref = copy.deepcopy(m)
    ids, pos, mask, _ = batch()
    with torch.no_grad():
        want = ref.reference_forward(ids, pos, mask)
        got = m(ids, pos, mask)
    # rows whose query is padding differ only through the -1e9/finfo.min semantics; compare valid rows
    valid = ~mask
    assert torch.allclose(got[valid], want[valid], atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("pad", [False, True])
def test_fused_backward_matches_autograd(act, pad):
    m = tiny(act)
    ref = copy.deepcopy(m)
    ids, pos, mask, tg = batch(pad=pad)
    store = LocalStore(m, "cpu")
    store.zero_grad()
    out = m(ids, pos, mask, targets=tg)
    out.loss.backward()
    logits = ref.reference_forward(ids, pos, mask)
    loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), tg.reshape(-1), ignore_index=-100)
    loss.backward()
    assert abs(out.loss.item() - loss.item()) < 1e-5
    gp = dict(m.named_parameters())
    for n, p in ref.named_parameters():
        g_ref, g = p.grad, gp[n].grad
        err = (g - g_ref).norm() / g_ref.norm().clamp_min(1e-12)
        assert err < 1e-4, (n, err.item())


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("dropout", [0.0, 0.2])
def test_ffn_tail_fused_into_consumer_layernorm(monkeypatch, act, dropout):
    """Every layer's down-projection bias / act' / dropout backward runs inside the LayerNorm
    backward that consumes its output (the next layer's LN1, the final norm: models/fused.py
    _FfnTail) -- no separate bias_act_bwd pass -- with the gradients of the unfused path."""
    import distributed_pytorch_cookbook_amd.models.fused as fz

    calls = []
    real = fz.bias_act_bwd
    monkeypatch.setattr(fz, "bias_act_bwd", lambda *a, **k: calls.append(1) or real(*a, **k))

    def grads(fuse):
        monkeypatch.setattr(fz, "_FUSE_TAIL", fuse)
        torch.manual_seed(0)
        m = TransformerDecoderLM(dim=64, head_dim=16, heads=4, num_layers=3, vocab_size=97,
                                 max_position_embeddings=24, activation=act, dropout=dropout)
        m.train()
        ids, pos, mask, tg = batch(pad=True)
        store = LocalStore(m, "cpu")
        store.zero_grad()
        m(ids, pos, mask, targets=tg, dropout_seed=1234).loss.backward()
        return {n: p.grad.clone() for n, p in m.named_parameters()}

    calls.clear()
    fused = grads(True)
    assert calls == []  # all three layers fused
    plain = grads(False)
    assert len(calls) == 3
    for n in plain:
        err = (fused[n] - plain[n]).norm() / plain[n].norm().clamp_min(1e-12)
        assert err < 1e-5, (n, err.item())


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("dropout", [0.0, 0.2])
def test_ffn_residual_handoff_to_next_layernorm(monkeypatch, act, dropout):
    """The FFN down projection's residual add / act / dropout run in the NEXT LayerNorm's forward
    (models/fused.py _FfnTail.pending: the next layer's LN1, the final norm, or a materialising
    pass at a run boundary).  Same loss and gradients as the GEMM-epilogue form (DPC_FUSE_FFN_LN=0)
    to rounding, and the run output formed by the materialising pass equals, bit for bit, the one
    the final norm forms (a layer's position in a run never changes the math)."""
    import distributed_pytorch_cookbook_amd.models.fused as fz

    def run(handoff):
        monkeypatch.setattr(fz, "_FUSE_FFN_LN", handoff)
        torch.manual_seed(0)
        m = TransformerDecoderLM(dim=64, head_dim=16, heads=4, num_layers=3, vocab_size=97,
                                 max_position_embeddings=24, activation=act, dropout=dropout)
        m.train()
        ids, pos, mask, tg = batch(pad=True)
        store = LocalStore(m, "cpu")
        store.zero_grad()
        out = m(ids, pos, mask, targets=tg, dropout_seed=99)
        out.loss.backward()
        return out.loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}, m, store

    lh, gh, m, store = run(True)
    lp, gp, _, _ = run(False)
    assert abs(lh.item() - lp.item()) < 1e-5 * abs(lp.item())
    for n in gp:
        err = (gh[n] - gp[n]).norm() / gp[n].norm().clamp_min(1e-12)
        assert err < 1e-4, (n, err.item())
    # the run output through the final norm's fused add vs the materialising pass
    monkeypatch.setattr(fz, "_FUSE_FFN_LN", True)
    m.eval()
    ids, pos, _, _ = batch(pad=False)
    with torch.no_grad():
        N, S = ids.shape
        x0 = fz.run_embeddings(m, store, ids, pos, False)
        xa = fz.run_layers(m, store, x0, None, N, S, m.decoder.layers, False, head_next=True)
        la = fz.head_logits(m, xa, store, xa._dpc_tail)
        x0 = fz.run_embeddings(m, store, ids, pos, False)
        xb = fz.run_layers(m, store, x0, None, N, S, m.decoder.layers, False, head_next=False)
        lb = fz.head_logits(m, xb, store)
    assert torch.equal(xa, xb) and torch.equal(la, lb)


def test_causality():
    m = tiny()
    ids, pos, _, _ = batch(pad=False)
    with torch.no_grad():
        a = m(ids, pos)
        ids2 = ids.clone()
        ids2[:, 12:] = (ids2[:, 12:] + 1) % 97
        b = m(ids2, pos)
    assert torch.allclose(a[:, :12], b[:, :12], atol=1e-5)
    assert not torch.allclose(a[:, 12:], b[:, 12:])


def test_store_views_and_flat_layout():
    m = tiny()
    st = LocalStore(m, "cpu")
    # parameters are views into one flat buffer; q/k/v adjacent
    for l in m.decoder.layers:
        a = l.attn
        q, k, v = a.to_q.weight, a.to_k.weight, a.to_v.weight
        assert k.data_ptr() == q.data_ptr() + q.numel() * 4
        assert v.data_ptr() == k.data_ptr() + k.numel() * 4
    assert st.master.numel() >= sum(p.numel() for p in m.parameters())
    sd = st.state_dict()
    assert list(sd.keys()) == list(m.state_dict().keys())


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_fused_dropout_matches_pinned_reference(act):
    """Counter-based dropout: the fused path and the reference math (masks pinned to the same
    seed) agree on loss and gradients; eval mode disables it; seeds advance per forward."""
    torch.manual_seed(0)
    m = TransformerDecoderLM(dim=64, head_dim=16, heads=4, num_layers=2, vocab_size=97,
                             max_position_embeddings=24, activation=act, dropout=0.2)
    ref = copy.deepcopy(m)
    ids, pos, mask, tg = batch(pad=True)
    store = LocalStore(m, "cpu")
    store.zero_grad()
    seed = 1234567
    out = m(ids, pos, mask, targets=tg, dropout_seed=seed)
    out.loss.backward()
    logits = ref.reference_forward(ids, pos, mask, dropout_seed=seed)
    loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), tg.reshape(-1), ignore_index=-100)
    loss.backward()
    assert abs(out.loss.item() - loss.item()) < 1e-5
    gp = dict(m.named_parameters())
    for n, p in ref.named_parameters():
        err = (gp[n].grad - p.grad).norm() / p.grad.norm().clamp_min(1e-12)
        assert err < 1e-4, (n, err.item())
    # a different seed gives a different loss; eval mode is deterministic and dropout-free
    with torch.no_grad():
        l1 = m(ids, pos, mask, targets=tg).loss.item()
        l2 = m(ids, pos, mask, targets=tg).loss.item()
        assert l1 != l2
        m.eval()
        ref.eval()
        e1 = m(ids, pos, mask, targets=tg).loss.item()
        e2 = m(ids, pos, mask, targets=tg).loss.item()
        want = ref.reference_forward(ids, pos, mask)
        want = F.cross_entropy(want.reshape(-1, want.shape[-1]), tg.reshape(-1), ignore_index=-100)
    assert e1 == e2 and abs(e1 - want.item()) < 1e-5


def test_dropout_mask_statistics():
    from distributed_pytorch_cookbook_amd.ops.dropout import DropSpec, keep_mask

    spec = DropSpec.make(0.25, seed=99, site=3)
    k = keep_mask(spec, 512, 384)
    frac = (k == 0).float().mean().item()
    assert abs(frac - 0.25) < 0.01
    assert torch.allclose(k[k > 0], torch.full_like(k[k > 0], 1 / 0.75))
    # different sites / seeds decorrelate
    k2 = keep_mask(DropSpec.make(0.25, seed=99, site=4), 512, 384)
    both = ((k == 0) & (k2 == 0)).float().mean().item()
    assert abs(both - 0.0625) < 0.01
    assert DropSpec.make(0.0, 1, 1) is None


def test_activation_recompute_matches():
    """--recompute: identical loss and gradients (dropout masks regenerated from the seed)."""
    torch.manual_seed(0)
    base = TransformerDecoderLM(dim=64, head_dim=16, heads=4, num_layers=2, vocab_size=97,
                                max_position_embeddings=24, activation="gelu", dropout=0.1)
    ids, pos, mask, tg = batch(pad=True)
    grads = []
    for rc in (False, True):
        m = copy.deepcopy(base)
        m.recompute = rc
        st = LocalStore(m, "cpu")
        st.zero_grad()
        out = m(ids, pos, mask, targets=tg, dropout_seed=77)
        out.loss.backward()
        grads.append((out.loss.item(), st.grads.clone()))
    assert grads[0][0] == grads[1][0]
    assert torch.allclose(grads[0][1], grads[1][1], atol=1e-7, rtol=1e-5)


def test_last_only_logits_and_generate():
    """Decode path: the LM head on the last position only gives that position's logits, and
    greedy ``generate`` (which uses it) emits the same text as the full-logits forward."""
    from distributed_pytorch_cookbook_amd.utils.batch import generate
    from distributed_pytorch_cookbook_amd.utils.tokenizer import ByteTokenizer

    torch.manual_seed(0)
    m = TransformerDecoderLM(64, 32, 2, 2, 512, 64, activation="gelu")
    ids = torch.randint(0, 512, (2, 20))
    pos = torch.arange(20).expand(2, -1)
    with torch.no_grad():
        full = m(ids, pos)
        last = m(ids, pos, last_only=True)
    assert last.shape == (2, 1, 512)
    assert torch.allclose(full[:, -1:], last, atol=1e-5)
    tok = ByteTokenizer()
    full_only = lambda input_ids, position_ids: m(input_ids, position_ids)  # noqa: E731
    full_only.max_position_embeddings = m.max_position_embeddings
    cpu = torch.device("cpu")
    assert generate(m, "One day, ", tok, cpu, 6) == generate(full_only, "One day, ", tok, cpu, 6)


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_kv_cache_decode_matches_recompute(act):
    """KV-cache decode: prefill + one-token steps give the same logits as re-running the full
    sequence, and the same greedy text."""
    from distributed_pytorch_cookbook_amd.utils.batch import generate
    from distributed_pytorch_cookbook_amd.utils.tokenizer import ByteTokenizer

    torch.manual_seed(1)
    m = TransformerDecoderLM(64, 32, 2, 2, 512, 64, activation=act)
    ids = torch.randint(0, 512, (2, 24))
    with torch.no_grad():
        cache = m.new_kv_cache(2, 24)
        got = [m.decode(ids[:, :16], torch.arange(16).expand(2, -1), cache)]
        got.append(m.decode(ids[:, 16:19], torch.arange(16, 19).expand(2, -1), cache))  # 3-token block
        for t in range(19, 24):
            got.append(m.decode(ids[:, t:t + 1], torch.full((2, 1), t), cache))
        for lg, end in zip(got, [16, 19] + list(range(20, 25))):
            ref = m(ids[:, :end], torch.arange(end).expand(2, -1))[:, -1:]
            assert torch.allclose(lg, ref, atol=1e-4, rtol=1e-4), end
    tok, cpu = ByteTokenizer(), torch.device("cpu")
    assert generate(m, "One day, ", tok, cpu, 8) == generate(m, "One day, ", tok, cpu, 8, use_cache=False)


# ---------------------------------------------------------------- parity with the reference module
_REF_GPT = "/root/reference/models/gpt.py"


def _reference_module():
    """``/root/reference/models/gpt.py`` as shipped, with its two documented one-line crash
    fixes applied in memory (``self.dim`` read before it is set,
    ``:177-178``; undefined ``x`` in ``forward``, ``:227``)."""
    import types

    if not os.path.exists(_REF_GPT):
        pytest.skip("reference checkout not present")
    pytest.importorskip("einops")
    src = open(_REF_GPT).read()
    for bad, good in (("nn.Embedding(vocab_size, self.dim)", "nn.Embedding(vocab_size, dim)"),
                      ("nn.Embedding(max_position_embeddings, self.dim)", "nn.Embedding(max_position_embeddings, dim)"),
                      ("x = self.embeddings(x, position_ids)", "x = self.embeddings(input_ids, position_ids)")):
        assert src.count(bad) == 1, bad
        src = src.replace(bad, good)
    mod = types.ModuleType("reference_models_gpt")
    exec(compile(src, _REF_GPT, "exec"), mod.__dict__)
    return mod


def test_parity_with_reference_module():
    """The reference's own TransformerDecoderLM (bugs fixed) vs ours: identical state-dict
    keys and shapes, logits with and without a key-padding mask, and every parameter gradient
    of the cross-entropy loss (fused path, manual backward)."""
    ref_mod = _reference_module()
    D, hd, H, L, V, S = 64, 16, 4, 2, 97, 24
    torch.manual_seed(0)
    ref = ref_mod.TransformerDecoderLM(dim=D, head_dim=hd, heads=H, num_layers=L, vocab_size=V,
                                       max_position_embeddings=S).eval()
    ours = TransformerDecoderLM(dim=D, head_dim=hd, heads=H, num_layers=L, vocab_size=V,
                                max_position_embeddings=S)
    rsd = ref.state_dict()
    assert list(rsd) == list(ours.state_dict())
    assert all(rsd[k].shape == v.shape for k, v in ours.state_dict().items())
    ours.load_state_dict(rsd)
    for pad in (False, True):
        ids, pos, mask, tg = batch(pad=pad)
        with torch.no_grad():
            want = ref(ids, pos, mask)
            got = ours(ids, pos, mask)
        rows = ~mask if mask is not None else torch.ones(ids.shape, dtype=torch.bool)
        assert torch.allclose(got[rows], want[rows], atol=2e-5, rtol=1e-5), (got[rows] - want[rows]).abs().max()
    # gradients
    ids, pos, mask, tg = batch(pad=True)
    store = LocalStore(ours, "cpu")
    store.zero_grad()
    ours(ids, pos, mask, targets=tg).loss.backward()
    logits = ref(ids, pos, mask)
    F.cross_entropy(logits.reshape(-1, V), tg.reshape(-1), ignore_index=-100).backward()
    gp = dict(ours.named_parameters())
    for n, p in ref.named_parameters():
        err = (gp[n].grad - p.grad).norm() / p.grad.norm().clamp_min(1e-12)
        assert err < 1e-4, (n, err.item())


@pytest.mark.parametrize("prefix", ["module.", "_orig_mod.", "_orig_mod.module."])
def test_reference_checkpoint_prefixes_round_trip(tmp_path, prefix):
    """A state dict saved by the reference's recipes -- DDP (``module.``), torch.compile
    (``_orig_mod.``) or both (``main-ddp.py:179-185``) -- loads into an engine through the
    checkpoint reader, and our saved file has the canonical bare keys."""
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.utils.checkpoint import load_model_state, save_model_state

    ref_mod = _reference_module()
    torch.manual_seed(1)
    ref = ref_mod.TransformerDecoderLM(dim=32, head_dim=16, heads=2, num_layers=2, vocab_size=97,
                                       max_position_embeddings=24)
    path = tmp_path / "ref.pt"
    torch.save({prefix + k: v for k, v in ref.state_dict().items()}, path)
    eng = DataParallelEngine(tiny(D=32, H=2, hd=16), "cpu", lr=1e-3)
    eng.load_model_state(load_model_state(path))
    sd = eng.full_state_dict()
    for k, v in ref.state_dict().items():
        assert torch.equal(sd[k], v), k
    out = save_model_state(sd, str(tmp_path / "ck"))
    back = torch.load(out, weights_only=True)
    assert list(back) == list(ref.state_dict())
