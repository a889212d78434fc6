"""Transformer HIP kernels (csrc/kernels/transformer.hip) vs fp32 PyTorch references of the same
ops on the same bf16 inputs: fused cross-entropy, LayerNorm / RMSNorm (+ residual add), QKV
split + RoPE, SwiGLU, bias-gradient column sums, and the fused BERT / Llama blocks end to end."""
import pytest
import torch
import torch.nn.functional as F

from consensusml_amd.ops import transformer as T

pytestmark = pytest.mark.gpu


def _leaf(t):
    return t.detach().clone().requires_grad_(True)


@pytest.mark.parametrize("R,V", [(7, 1000), (33, 30522), (5, 13), (4, 128256), (3, 3),
                                 (3000, 50)])
def test_cross_entropy(cuda, R, V):
    torch.manual_seed(R + V)
    x = (torch.randn(R, V, device=cuda) * 3).to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, V, (R,), device=cuda)
    if R > 4:
        y[1] = -100   # ignored row
    loss = T.cross_entropy(x, y)
    loss.backward(torch.tensor(1.7, device=cuda))
    xr = _leaf(x.float())
    lr = F.cross_entropy(xr, y, ignore_index=-100)
    lr.backward(torch.tensor(1.7, device=cuda))
    torch.testing.assert_close(loss.float(), lr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-4)
    if R > 4:
        assert x.grad[1].abs().max().item() == 0.0


def test_cross_entropy_all_ignored(cuda):
    """Every label ignored: loss 0 and a zero gradient (the valid count clamps to 1, as
    F.cross_entropy's reduction would divide by zero)."""
    x = torch.randn(9, 40, device=cuda).to(torch.bfloat16).requires_grad_(True)
    y = torch.full((9,), -100, device=cuda, dtype=torch.long)
    loss = T.cross_entropy(x, y)
    loss.backward()
    assert loss.item() == 0.0 and x.grad.abs().max().item() == 0.0


def test_cross_entropy_misaligned_view(cuda):
    """A logits view that is not 16-B aligned is copied, not read out of bounds."""
    base = torch.randn(6 * 37 + 1, device=cuda).to(torch.bfloat16)
    x = base[1:].view(6, 37).requires_grad_(False)
    y = torch.randint(0, 37, (6,), device=cuda)
    torch.testing.assert_close(T.cross_entropy(x, y).float(), F.cross_entropy(x.float(), y),
                               rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("D", [64, 768, 1024, 2048, 4096, 24])
@pytest.mark.parametrize("kind", ["ln", "rms"])
@pytest.mark.parametrize("res", [False, True])
def test_norms(cuda, D, kind, res):
    torch.manual_seed(D)
    M = 77
    x = (torch.randn(M, D, device=cuda) * 2 + 0.5).to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(M, D, device=cuda).to(torch.bfloat16).requires_grad_(True) if res else None
    w = (torch.rand(D, device=cuda) + 0.5).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(D, device=cuda).to(torch.bfloat16).requires_grad_(True) if kind == "ln" else None
    eps = 1e-5
    s, y = T.add_norm(x, r, w, b, eps)
    dy = torch.randn_like(y)
    ds = torch.randn_like(y) if res else None
    torch.autograd.backward([y, s] if res else [y], [dy, ds] if res else [dy])
    xr, wr = _leaf(x.float()), _leaf(w.float())
    rr = _leaf(r.float()) if res else None
    br = _leaf(b.float()) if b is not None else None
    sr = xr + rr if res else xr
    sr_b = sr.to(torch.bfloat16).float() if res else sr   # the kernel normalises the bf16 sum
    if kind == "ln":
        yr = F.layer_norm(sr_b, (D,), wr, br, eps)
    else:
        yr = sr_b * torch.rsqrt(sr_b.pow(2).mean(-1, keepdim=True) + eps) * wr
    torch.autograd.backward([yr, sr] if res else [yr], [dy.float(), ds.float()] if res else [dy.float()])
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    if res:
        torch.testing.assert_close(s.float(), sr, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(r.grad.float(), rr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=2e-2, atol=0.3)
    if b is not None:
        torch.testing.assert_close(b.grad.float(), br.grad, rtol=2e-2, atol=0.3)


@pytest.mark.parametrize("rot", [False, True])
@pytest.mark.parametrize("H,KV,hd", [(4, 2, 64), (12, 12, 64), (8, 2, 128)])
def test_qkv_split_rope(cuda, rot, H, KV, hd):
    torch.manual_seed(H * hd)
    B, S = 2, 19
    qkv = torch.randn(B, S, (H + 2 * KV) * hd, device=cuda).to(torch.bfloat16).requires_grad_(True)
    cos, sin = T.rope_tables(S, hd, 10000.0, cuda) if rot else (None, None)
    q, k, v = T.qkv_split(qkv, H, KV, hd, cos, sin)
    assert q.shape == (B, H, S, hd) and k.shape == (B, KV, S, hd) and q.is_contiguous()
    gq, gk, gv = torch.randn_like(q), torch.randn_like(k), torch.randn_like(v)
    torch.autograd.backward([q, k, v], [gq, gk, gv])
    xr = _leaf(qkv.float())
    x = xr.view(B, S, H + 2 * KV, hd).transpose(1, 2)
    qr, kr, vr = x[:, :H], x[:, H:H + KV], x[:, H + KV:]
    if rot:
        def rope(t):
            t1, t2 = t[..., 0::2], t[..., 1::2]
            c, s_ = cos[None, None], sin[None, None]
            return torch.stack((t1 * c - t2 * s_, t1 * s_ + t2 * c), -1).flatten(-2)
        qr, kr = rope(qr), rope(kr)
    torch.autograd.backward([qr, kr, vr], [gq.float(), gk.float(), gv.float()])
    torch.testing.assert_close(q.float(), qr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(k.float(), kr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(v.float(), vr, rtol=0, atol=0)
    torch.testing.assert_close(qkv.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,F_", [(33, 128), (7, 14336)])
def test_swiglu(cuda, M, F_):
    torch.manual_seed(M)
    h = (torch.randn(M, 2 * F_, device=cuda) * 2).to(torch.bfloat16).requires_grad_(True)
    y = T.swiglu(h)
    dy = torch.randn_like(y)
    y.backward(dy)
    hr = _leaf(h.float())
    a, b = hr.chunk(2, -1)
    yr = F.silu(a) * b
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(h.grad.float(), hr.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,N", [(4096, 768), (100, 3072), (1, 8), (65, 30528)])
def test_colsum_linear_bias(cuda, M, N):
    torch.manual_seed(N)
    x = torch.randn(M, 64, device=cuda).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(N, 64, device=cuda) * 0.1).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(N, device=cuda).to(torch.bfloat16).requires_grad_(True)
    y = T.linear(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    torch.testing.assert_close(b.grad.float(), dy.float().sum(0), rtol=1e-2, atol=0.15)
    xr, wr = _leaf(x.float()), _leaf(w.float())
    F.linear(xr, wr).backward(dy.float())
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=2e-2, atol=0.5)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=0.1)


@pytest.mark.parametrize("name", ["bert_tiny", "llama_tiny"])
def test_fused_model_matches_reference_path(cuda, name):
    """The fused-kernel forward / backward of a whole model agrees with the same model run on
    the PyTorch reference compositions (fp32 copies of the weights)."""
    from consensusml_amd.models import transformer as MT
    from consensusml_amd.ops.transformer import cross_entropy
    torch.manual_seed(0)
    m = getattr(MT, name)().to(cuda)
    ref = getattr(MT, name)().to(cuda)
    ref.load_state_dict(m.state_dict())
    m = m.to(torch.bfloat16)
    ids = torch.randint(0, 512, (2, 32), device=cuda)
    lab = torch.randint(0, 512, (2, 32), device=cuda)
    loss = cross_entropy(m(ids), lab)
    loss.backward()
    lr = cross_entropy(ref(ids), lab)   # fp32 -> reference path everywhere
    lr.backward()
    assert abs(loss.item() - lr.item()) < 0.05 * max(1.0, abs(lr.item()))
    gm = torch.cat([p.grad.float().flatten() for p in m.parameters()])
    gr = torch.cat([p.grad.float().flatten() for p in ref.parameters()])
    cos = F.cosine_similarity(gm, gr, dim=0).item()
    assert cos > 0.98, cos


def _attn_ref(qkv, H, hd):
    B, S, _ = qkv.shape
    x = qkv.float().view(B, S, 3, H, hd).permute(2, 0, 3, 1, 4)
    a = torch.softmax(x[0] @ x[1].transpose(-1, -2) / hd ** 0.5, -1) @ x[2]
    return a.transpose(1, 2).reshape(B, S, H * hd)


@pytest.mark.parametrize("S", [32, 64, 96, 128])
@pytest.mark.parametrize("B,H", [(3, 2), (2, 12)])
def test_mfma_attention(cuda, S, B, H):
    """csrc/kernels/attention.hip forward / backward vs fp32 softmax attention on the same bf16
    inputs (asymmetric random data: catches transposed fragments and k-permutation errors)."""
    torch.manual_seed(S * 7 + H)
    hd = 64
    qkv = (torch.randn(B, S, 3 * H * hd, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_(True)
    out = T.fused_qkv_attention(qkv, H, hd)
    assert out.shape == (B, S, H * hd)
    dout = torch.randn_like(out)
    out.backward(dout)
    xr = _leaf(qkv.float())
    ref = _attn_ref(xr, H, hd)
    ref.backward(dout.float())
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    g, gr = qkv.grad.float(), xr.grad

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()
    sec = H * hd
    for i, name in enumerate("qkv"):   # per-projection relative error (bf16 P / dS operands)
        e = rel(g[..., i * sec:(i + 1) * sec], gr[..., i * sec:(i + 1) * sec])
        assert e < 2e-2, (name, e)
    torch.testing.assert_close(g, gr, rtol=5e-2, atol=5e-2)


def test_mfma_attention_matches_sdpa_path(cuda):
    """The kernel path and the SDPA fallback path of fused_qkv_attention agree."""
    torch.manual_seed(11)
    qkv = torch.randn(4, 128, 3 * 12 * 64, device=cuda).to(torch.bfloat16)
    a = T.fused_qkv_attention(qkv, 12, 64)
    from consensusml_amd import perf
    with perf.use_policy(perf.policy().replace(attn_kernel=False)):
        b = T.fused_qkv_attention(qkv, 12, 64)
    torch.testing.assert_close(a.float(), b.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("Tn,N,K", [(8192, 768, 768), (4096, 3072, 768), (1024, 768, 3072),
                                    (1024, 256, 128)])
def test_linear_wgrad_on_wgrad1x1(cuda, Tn, N, K):
    """Transformer-linear weight gradient dY^T X on the 1x1-conv weight-gradient kernel
    (PerfPolicy.own_linear_wgrad) vs fp32, and through a linear's autograd with the policy on vs
    off (hipBLASLt)."""
    from consensusml_amd import perf
    g = torch.Generator(device=cuda).manual_seed(Tn + N)
    dy = torch.randn(Tn, N, device=cuda, generator=g).bfloat16()
    x = torch.randn(Tn, K, device=cuda, generator=g).bfloat16()
    ref = dy.float().t() @ x.float()
    with perf.use_policy(perf.policy().replace(own_linear_wgrad=True)):
        dw = T._linear_wgrad(dy, x)
    assert dw.shape == (N, K) and dw.dtype == torch.bfloat16
    assert float((dw.float() - ref).norm() / ref.norm()) < 5e-3
    w = (torch.randn(N, K, device=cuda, generator=g) * K ** -0.5).bfloat16()
    b = torch.zeros(N, device=cuda, dtype=torch.bfloat16)
    grads = []
    for on in (True, False):
        wi, bi_ = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        with perf.use_policy(perf.policy().replace(own_linear_wgrad=on)):
            T.linear(x, wi, bi_).backward(dy)
        grads.append(wi.grad.float())
    assert float((grads[0] - grads[1]).norm() / grads[1].norm()) < 5e-3
    assert float((grads[0] - ref).norm() / ref.norm()) < 5e-3


@pytest.mark.parametrize("M,N,K,own", [(1024, 768, 512, True), (512, 1152, 640, True),
                                       (2048, 512, 1024, False)])
def test_linear_nb_vs_fp32(cuda, M, N, K, own, monkeypatch):
    """Bias-free linear (Llama projections): hipBLASLt forward, own-or-library data gradient,
    weight gradient as an NT GEMM on transposed operands -- all against fp32."""
    from consensusml_amd.ops import transformer as T
    if not own:
        monkeypatch.setattr(T, "_NB_OWN_DGRAD_MAX", 0)
    torch.manual_seed(M + N)
    lin = T.LinearNB(K, N).to(cuda, torch.bfloat16)
    x = torch.randn(2, M // 2, K, device=cuda).bfloat16().requires_grad_(True)
    y = lin(x)
    assert "LinearNB" in type(y.grad_fn).__name__
    dy = torch.randn_like(y)
    y.backward(dy)
    xf = x.detach().float().requires_grad_(True)
    wf = lin.weight.detach().float().requires_grad_(True)
    yf = xf @ wf.t()
    yf.backward(dy.float())
    rel = lambda a, b: float((a.float() - b.float()).norm() / b.float().norm())  # noqa: E731
    assert rel(y, yf) < 1e-2
    assert rel(x.grad, xf.grad) < 1e-2
    assert rel(lin.weight.grad, wf.grad) < 1e-2
