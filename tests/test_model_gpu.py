"""End-to-end fused model on the GPU (bf16 kernels) vs the f32 CPU reference."""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM
from distributed_pytorch_cookbook_amd.ops import _lib
from distributed_pytorch_cookbook_amd.parallel.store import LocalStore

pytestmark = pytest.mark.gpu


def make(act, D=128, H=2, hd=64, L=2, V=1000, S=130, seed=0):
    torch.manual_seed(seed)
    return TransformerDecoderLM(dim=D, head_dim=hd, heads=H, num_layers=L, vocab_size=V,
                                max_position_embeddings=S, activation=act)


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("pad", [False, True])
def test_fused_gpu_matches_reference(act, pad):
    m_cpu = make(act)
    m_gpu = copy.deepcopy(m_cpu).cuda()
    N, S, V = 3, 129, 1000
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, V, (N, S), generator=g)
    tg = torch.randint(0, V, (N, S), generator=g)
    pos = torch.arange(S).repeat(N, 1)
    mask = None
    if pad:
        mask = torch.zeros(N, S, dtype=torch.bool)
        mask[1, 100:] = True
        tg[1, 100:] = -100
    logits = m_cpu.reference_forward(ids, pos, mask)
    loss = F.cross_entropy(logits.reshape(-1, V), tg.reshape(-1), ignore_index=-100)
    loss.backward()
    store = LocalStore(m_gpu, "cuda")
    store.zero_grad()
    out = m_gpu(ids.cuda(), pos.cuda(), mask.cuda() if mask is not None else None, targets=tg.cuda())
    out.loss.backward()
    torch.cuda.synchronize()
    assert abs(out.loss.item() - loss.item()) < 2e-2 * loss.item()
    gp = dict(m_gpu.named_parameters())
    for n, p in m_cpu.named_parameters():
        err = ((gp[n].grad.cpu() - p.grad).norm() / p.grad.norm().clamp_min(1e-12)).item()
        assert err < (1.2e-1 if act == "relu" else 6e-2), (n, err)
    assert _lib.is_loaded()


@pytest.mark.parametrize("act", ["relu", "gelu"])
def test_gpt2_width_gradients_match_fp32(act):
    """GPT-2-small width (D=768, 12 heads of 64, L=2): every parameter gradient of the fused
    bf16 GPU step against the f32 reference (/root/reference/models/gpt.py:10-41).  Weights and
    embeddings are rounded to bf16 first, so the remaining error is the kernels' own (bf16
    activations, f32 accumulation order)."""
    torch.manual_seed(0)
    D, H, hd, L, V, S, N = 768, 12, 64, 2, 2048, 257, 4
    m_cpu = TransformerDecoderLM(dim=D, head_dim=hd, heads=H, num_layers=L, vocab_size=V,
                                 max_position_embeddings=S, activation=act)
    with torch.no_grad():
        for p in m_cpu.parameters():
            p.copy_(p.bfloat16().float())
    m_gpu = copy.deepcopy(m_cpu).cuda()
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, V, (N, S), generator=g)
    tg = torch.randint(0, V, (N, S), generator=g)
    pos = torch.arange(S).repeat(N, 1)
    logits = m_cpu.reference_forward(ids, pos, None)
    loss = F.cross_entropy(logits.reshape(-1, V), tg.reshape(-1))
    loss.backward()
    store = LocalStore(m_gpu, "cuda")
    store.zero_grad()
    out = m_gpu(ids.cuda(), pos.cuda(), None, targets=tg.cuda())
    out.loss.backward()
    torch.cuda.synchronize()
    assert abs(out.loss.item() - loss.item()) < 5e-3 * loss.item()
    gp = dict(m_gpu.named_parameters())
    errs = {}
    for n, p in m_cpu.named_parameters():
        errs[n] = ((gp[n].grad.cpu() - p.grad).norm() / p.grad.norm().clamp_min(1e-12)).item()
    worst = max(errs.values())
    print(f"[{act}] worst relative gradient error {worst:.4f} ({max(errs, key=errs.get)})")
    assert worst < (GRAD_TOL_RELU if act == "relu" else GRAD_TOL_GELU), errs
    assert _lib.is_loaded()


GRAD_TOL_RELU = 7.5e-2  # measured 5.3 % (a layer-1 LayerNorm bias; ReLU kinks flip under bf16)
GRAD_TOL_GELU = 2e-2  # measured 0.54 %


def test_gpu_training_reduces_loss():
    m = make("gelu", V=512).cuda()
    eng = DataParallelEngine(m, "cuda", lr=3e-3)
    N, S = 8, 128
    ids = torch.randint(0, 512, (N, S + 1), device="cuda")
    b = dict(input_ids=ids[:, :-1], position_ids=torch.arange(S, device="cuda").expand(N, -1), mask=None)
    losses = [eng.train_step(b, ids[:, 1:]).item() for _ in range(30)]
    assert losses[-1] < 0.5 * losses[0], losses


def test_gpt2_small_step_and_generate():
    from distributed_pytorch_cookbook_amd.models.gpt import PRESETS
    from distributed_pytorch_cookbook_amd.utils.batch import generate
    from distributed_pytorch_cookbook_amd.utils.tokenizer import ByteTokenizer

    p = PRESETS["gpt2-small"]
    torch.manual_seed(0)
    with torch.device("cuda"):
        m = TransformerDecoderLM(p["dim"], p["head_dim"], p["heads"], p["num_layers"], 50257, 1024,
                                 activation="gelu")
    eng = DataParallelEngine(m, "cuda", lr=1e-4)
    N, S = 2, 1023
    ids = torch.randint(0, 50257, (N, S + 1), device="cuda")
    b = dict(input_ids=ids[:, :-1], position_ids=torch.arange(S, device="cuda").expand(N, -1), mask=None)
    l0 = eng.train_step(b, ids[:, 1:]).item()
    l1 = eng.train_step(b, ids[:, 1:]).item()
    assert 10.0 < l0 < 12.0 and l1 < l0
    s = generate(m, "One day, ", ByteTokenizer(), torch.device("cuda"), max_new_tokens=4)
    assert s.startswith("One day, ")


def test_long_context_train_step():
    """a full fused train step at S = 8191 (8x GPT-2's context) stays finite and learns."""
    torch.manual_seed(0)
    S = 8191
    with torch.device("cuda"):
        m = TransformerDecoderLM(256, 64, 4, 2, 50257, S + 1, activation="gelu")
    eng = DataParallelEngine(m, "cuda", lr=1e-3)
    ids = torch.randint(0, 50257, (1, S + 1), device="cuda")
    b = dict(input_ids=ids[:, :-1], position_ids=torch.arange(S, device="cuda").expand(1, -1), mask=None)
    losses = [eng.train_step(b, ids[:, 1:]).item() for _ in range(3)]
    assert all(math.isfinite(l) for l in losses) and losses[-1] < losses[0], losses


@pytest.mark.parametrize("head_dim", [64, 128])
def test_main_single_recipe_gpu(tmp_path, monkeypatch, head_dim):
    """main-single.py end to end on the GPU, including --head_dim 128 (the reference takes any
    head size: /root/reference/main-single.py:160)."""
    from distributed_pytorch_cookbook_amd.recipes import run

    monkeypatch.chdir(tmp_path)
    trainer, path = run("single", ["--synthetic_data", "--batch_size", "8", "--epochs", "1",
                                   "--sequence_length", "128", "--dim", "128", "--heads", "2",
                                   "--head_dim", str(head_dim), "--num_layers", "2", "--max_steps", "16",
                                   "--train_samples", "256", "--val_samples", "16", "--num_workers", "0",
                                   "--learning_rate", "1e-3"])
    assert path is not None and path.exists()
    sd = torch.load(path, weights_only=True)
    assert len(sd) == 13 * 2 + 5


@pytest.mark.parametrize("want_correct", [False, True])
def test_chunked_head_matches_whole_batch(monkeypatch, want_correct):
    """Row-chunked logits GEMM + cross-entropy (ragged last chunk, ignored targets) gives the
    same loss, accuracy and gradients as one pass over the whole batch."""
    import distributed_pytorch_cookbook_amd.models.fused as fused

    N, S, V = 3, 129, 1000
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, V, (N, S), generator=g).cuda()
    tg = torch.randint(0, V, (N, S), generator=g)
    tg[2, 50:70] = -100
    tg = tg.cuda()
    pos = torch.arange(S).repeat(N, 1).cuda()
    res = []
    for chunk in (0, 100):
        monkeypatch.setattr(fused, "_HEAD_CHUNK", chunk)
        m = make("gelu").cuda()
        store = LocalStore(m, "cuda")
        store.zero_grad()
        if want_correct:
            with torch.no_grad():
                out = m(ids, pos, None, targets=tg, want_correct=True)
            res.append((out.loss.item(), out.n_correct.item(), None))
            continue
        out = m(ids, pos, None, targets=tg)
        out.loss.backward()
        torch.cuda.synchronize()
        res.append((out.loss.item(), None, store.grads.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-5 * abs(res[0][0])
    if want_correct:
        assert res[0][1] == res[1][1]
    else:
        assert torch.allclose(res[0][2], res[1][2], rtol=1e-3, atol=1e-6)


def test_side_stream_wgrad_matches_single_stream(monkeypatch):
    """DPC_WGRAD_STREAM: weight gradients on a side stream give the same gradients as the
    single-stream backward (same kernels; split-K f32 atomics make the last bits run-dependent)."""
    from distributed_pytorch_cookbook_amd.models import fused
    N, S, V = 3, 129, 1000
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(0, V, (N, S), generator=g).cuda()
    tg = torch.randint(0, V, (N, S), generator=g).cuda()
    pos = torch.arange(S).repeat(N, 1).cuda()
    grads = []
    for on in (False, True):
        monkeypatch.setattr(fused, "_WGRAD_STREAM", on)
        m = make("gelu").cuda()
        store = LocalStore(m, "cuda")
        store.zero_grad()
        m(ids, pos, None, targets=tg).loss.backward()
        torch.cuda.synchronize()
        grads.append(store.grads.clone())
    assert ((grads[0] - grads[1]).norm() / grads[0].norm()).item() < 1e-5


@pytest.mark.parametrize("hd", [64, 32, 128])
def test_kv_cache_decode_gpu(hd):
    """KV-cache decode on the GPU kernels (flash-attention prefill, 1-row GEMMs) vs re-running
    the whole sequence through the fused forward."""
    torch.manual_seed(0)
    with torch.device("cuda"):
        m = TransformerDecoderLM(256, hd, 256 // hd, 2, 50257, 256, activation="gelu")
    m.eval()
    ids = torch.randint(0, 50257, (2, 40), device="cuda")
    pos = lambda a, b: torch.arange(a, b, device="cuda").expand(2, -1)  # noqa: E731
    with torch.no_grad():
        cache = m.new_kv_cache(2, 40)
        got = [(m.decode(ids[:, :33], pos(0, 33), cache), 33)]
        for t in range(33, 40):
            got.append((m.decode(ids[:, t:t + 1], pos(t, t + 1), cache), t + 1))
        for lg, end in got:
            ref = m(ids[:, :end], pos(0, end))[:, -1:]
            err = ((lg.float() - ref.float()).norm() / ref.float().norm()).item()
            assert err < 2e-2, (end, err)
    assert _lib.is_loaded()


@pytest.mark.parametrize("hd", [64, 128])
def test_graph_decoder_matches_eager_decode(hd):
    """The HIP-graph one-token decode step (static shapes over the cache capacity) gives the
    same logits as the eager cached decode and the full forward; greedy text is unchanged --
    at GPT-2's head size and at 128 (the decode kernel takes any multiple of 8 up to 256)."""
    from distributed_pytorch_cookbook_amd.utils.batch import generate
    from distributed_pytorch_cookbook_amd.utils.tokenizer import ByteTokenizer

    torch.manual_seed(0)
    with torch.device("cuda"):
        m = TransformerDecoderLM(256, hd, 256 // hd, 2, 50257, 128, activation="gelu")
    m.eval()
    ids = torch.randint(0, 50257, (1, 30), device="cuda")
    with torch.no_grad():
        cache = m.new_kv_cache(1, 40)
        m.decode(ids[:, :20], torch.arange(20, device="cuda")[None], cache)
        dec = m.graph_decoder(cache)
        assert dec is not None
        for t in range(20, 30):
            lg = dec.step(ids[:, t:t + 1]).clone()
            ref = m(ids[:, :t + 1], torch.arange(t + 1, device="cuda")[None])[:, -1:]
            err = ((lg.float() - ref.float()).norm() / ref.float().norm()).item()
            assert err < 2e-2, (t, err)
        assert cache.len == 30 and int(cache.len_t) == 30
    tok, dev = ByteTokenizer(), torch.device("cuda")
    a = generate(m, "One day, ", tok, dev, 12)
    b = generate(m, "One day, ", tok, dev, 12, use_cache=False)
    assert a == b
