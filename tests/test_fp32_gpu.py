"""The --disable_amp (f32 compute) path on HIP kernels: f32 MFMA GEMM (csrc/gemm_f32.hip), f32
flash attention (csrc/attention_f32.hip) and the whole fused f32 model against the f32
reference (/root/reference/main-single.py:88-90: with AMP off the reference trains in f32)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM
from distributed_pytorch_cookbook_amd.ops import _lib
from distributed_pytorch_cookbook_amd.ops.attention import attention_bwd, attention_fwd, attention_ref
from distributed_pytorch_cookbook_amd.ops.gemm import _gemm_ref, gemm
from distributed_pytorch_cookbook_amd.parallel.store import LocalStore

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel(x, ref):
    return float((x.float() - ref.float()).abs().max() / ref.float().abs().max().clamp_min(1e-30))


def _no_torch_fallback(monkeypatch):
    import distributed_pytorch_cookbook_amd.ops.attention as am
    import distributed_pytorch_cookbook_amd.ops.gemm as gm

    def boom(*a, **k):
        raise AssertionError("f32 path fell back to torch ops")

    monkeypatch.setattr(gm, "_gemm_ref", boom)
    monkeypatch.setattr(am, "attention_ref", boom)


@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
@pytest.mark.parametrize("shape", [(300, 264, 96), (257, 520, 1000), (1024, 768, 3072), (64, 50257, 130)])
def test_gemm_f32_plain(layout, shape):
    M, N, K = shape
    torch.manual_seed(0)
    ak, bk = layout[0] == "n", layout[1] == "t"
    A = torch.randn(M, K, device=dev) if ak else torch.randn(K, M, device=dev)
    B = torch.randn(N, K, device=dev) if bk else torch.randn(K, N, device=dev)
    out = gemm(A, B, a_kmaj=ak, b_kmaj=bk, out_dtype=torch.float32)
    ref = (A if ak else A.t()).double() @ (B if bk else B.t()).double().t()
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("aux_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [1, 2])
def test_gemm_f32_epilogues(act, aux_dtype):
    torch.manual_seed(1)
    M, N, K = 333, 200, 136
    A, W = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev)
    bias, res = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
    aux = torch.empty(M, N, device=dev, dtype=aux_dtype)
    out = gemm(A, W, bias=bias, act=act, residual=res, aux_out=aux, out_dtype=torch.float32)
    ref, ref_aux = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    _gemm_ref(A, W, True, True, ref, bias, act, 0, None, ref_aux, res, 1.0, None, False)
    assert rel(out, ref) < 1e-5 and rel(aux, ref_aux) < (1e-5 if aux_dtype == torch.float32 else 5e-3)
    # input-gradient form: act'(aux_in), column sums, accumulate into C
    z = torch.randn(M, N, device=dev).to(aux_dtype)
    cs, cs_ref = torch.zeros(N, device=dev), torch.zeros(N, device=dev)
    c0 = torch.randn(M, N, device=dev)
    out2 = c0.clone()
    gemm(A, W, act_bwd=act, aux_in=z, colsum=cs, out=out2, accumulate=True)
    ref2 = c0.clone()
    _gemm_ref(A, W, True, True, ref2, None, 0, act, z, None, None, 1.0, None, True, cs_ref)
    assert rel(out2, ref2) < 1e-5 and rel(cs, cs_ref) < 1e-5


@pytest.mark.parametrize("hd", [64, 32, 128])
@pytest.mark.parametrize("S,with_pad,causal", [(257, False, True), (200, True, True), (130, False, False)])
def test_attention_f32(S, with_pad, causal, hd):
    torch.manual_seed(2)
    N, H = 2, 3
    qkv = torch.randn(N * S, 3 * H * hd, device=dev)
    pad = None
    if with_pad:
        pad = torch.zeros(N, S, dtype=torch.bool, device=dev)
        pad[0, S - S // 4:] = True
        pad[1, 5:9] = True
    o, lse = attention_fwd(qkv, N, S, H, hd, pad, causal=causal)
    o_r, lse_r = attention_ref(qkv, N, S, H, hd, pad, causal=causal)
    assert o.dtype == torch.float32 and rel(o, o_r) < 1e-5
    fin = torch.isfinite(lse_r)
    assert torch.allclose(lse[fin], lse_r[fin], atol=1e-5, rtol=1e-5)
    do = torch.randn_like(o)
    g = attention_bwd(do, qkv, o, lse, N, S, H, hd, pad, causal=causal)
    x = qkv.clone().requires_grad_(True)
    (g_r,) = torch.autograd.grad(attention_ref(x, N, S, H, hd, pad, causal=causal)[0], x, do)
    assert rel(g, g_r) < 1e-4


def test_fp32_model_matches_reference(monkeypatch):
    """--disable_amp: the fused model in f32 on the HIP kernels (no torch GEMM / attention)."""
    torch.manual_seed(0)
    m_cpu = TransformerDecoderLM(dim=256, head_dim=32, heads=8, num_layers=2, vocab_size=1000,
                                 max_position_embeddings=130, activation="relu")
    m_gpu = copy.deepcopy(m_cpu).cuda()
    N, S, V = 3, 129, 1000
    g = torch.Generator().manual_seed(1)
    ids, tg = torch.randint(0, V, (N, S), generator=g), torch.randint(0, V, (N, S), generator=g)
    pos = torch.arange(S).repeat(N, 1)
    loss = F.cross_entropy(m_cpu.reference_forward(ids, pos, None).reshape(-1, V), tg.reshape(-1))
    loss.backward()
    store = LocalStore(m_gpu, "cuda", compute_dtype=torch.float32)
    store.zero_grad()
    _no_torch_fallback(monkeypatch)
    out = m_gpu(ids.cuda(), pos.cuda(), None, targets=tg.cuda())
    out.loss.backward()
    torch.cuda.synchronize()
    assert abs(out.loss.item() - loss.item()) < 1e-4 * loss.item()
    gp = dict(m_gpu.named_parameters())
    for n, p in m_cpu.named_parameters():
        err = ((gp[n].grad.cpu() - p.grad).norm() / p.grad.norm().clamp_min(1e-12)).item()
        assert err < 2e-3, (n, err)
    assert _lib.is_loaded()
