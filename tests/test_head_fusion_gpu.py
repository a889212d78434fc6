"""BERT MLM-head fusions against fp32 PyTorch oracles:
* a biased linear whose width is not a multiple of 8 (V = 30522 in BERT) writes 16-B aligned
  padded rows; the cross-entropy reads them in place and its backward also emits the bias gradient
  (``ce_bwd_cs`` + ``ce_part_fold``), for plain and batched-virtual-worker (per-segment) gradients;
* the head transform gelu(x W^T + b) on gemm.hip with the GELU backward kernel."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("V", [510, 1003, 30522])
def test_padded_logits_ce_and_bias_grad(cuda, V):
    from consensusml_amd.ops import transformer as T
    torch.manual_seed(V)
    M, K = 256, 64
    x = (torch.randn(M, K, device=cuda)).bfloat16().requires_grad_(True)
    w = (torch.randn(V, K, device=cuda) * 0.2).bfloat16().requires_grad_(True)
    b = (torch.randn(V, device=cuda) * 0.1).bfloat16().requires_grad_(True)
    labels = torch.randint(0, V, (M,), device=cuda)
    labels[::7] = -100
    logits = T.linear(x, w, b, logits=True)
    assert logits.shape == (M, V) and logits.stride(0) % 8 == 0 and logits.stride(0) > V
    # any other biased linear of that width returns plain contiguous rows
    plain = T.linear(x.detach(), w.detach(), b.detach())
    assert plain.is_contiguous() and plain.view(-1).numel() == M * V
    loss = T.cross_entropy(logits, labels)
    loss.backward()
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    lr = F.cross_entropy(xr @ wr.t() + br, labels, ignore_index=-100)
    lr.backward()
    assert abs(float(loss) - float(lr)) < 2e-2 * max(1.0, abs(float(lr)))
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


def test_ce_bwd_cs_matches_plain_backward(cuda):
    """The fused backward's gradient equals the plain kernel's, and its column partials fold to the
    column sums of that stored gradient (per segment)."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(1)
    R, V, ld = 512, 1003, 1008
    buf = torch.randn(R, ld, device=cuda).bfloat16()
    logits = buf[:, :V]
    labels = torch.randint(0, V, (R,), device=cuda)
    lse, rows = lib().ce_fwd(logits, labels, -100)
    lse2, rows2 = lib().ce_fwd(logits.contiguous(), labels, -100)
    # (the contiguous rows are misaligned: another split between scalar edges and vector interior,
    # so another summation order)
    torch.testing.assert_close(lse, lse2, rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(rows, rows2, rtol=1e-6, atol=1e-5)
    scale = torch.tensor([0.5], device=cuda)
    g, part = lib().ce_bwd_cs(logits, labels, lse, scale, -100)
    g_ref = lib().ce_bwd(logits.contiguous(), labels, lse, scale, -100)
    assert torch.equal(g, g_ref)   # same lse: the elementwise formula is order-free
    for nseg in (1, 4):
        out = torch.empty(nseg, V, device=cuda, dtype=torch.float32)
        lib().ce_part_fold(part, V, nseg, out)
        ref = g.float().view(nseg, R // nseg, V).sum(1)
        assert (out - ref).abs().max().item() < 1e-4


def test_bert_tiny_uses_padded_logits(cuda):
    """bert_tiny's vocab (510) is not a multiple of 8, like BERT-base's: its logits come out as
    the padded view, so the batched-worker tests (test_batched_workers_gpu.py) run this path."""
    from consensusml_amd.models import transformer as MT
    m = MT.bert_tiny().to(cuda, torch.bfloat16)
    assert m.c.vocab % 8 != 0
    ids = torch.randint(0, m.c.vocab, (2, 32), device=cuda)
    out = m(ids)
    assert out.shape[-1] == m.c.vocab and out.stride(-2) % 8 == 0 and out.stride(-2) > m.c.vocab


def test_linear_gelu_vs_fp32(cuda):
    from consensusml_amd.ops import transformer as T
    torch.manual_seed(2)
    lin = torch.nn.Linear(256, 768).to(cuda, torch.bfloat16)
    x = torch.randn(2, 256, 256, device=cuda).bfloat16().requires_grad_(True)
    a = T.linear_gelu(x, lin)
    g = torch.randn_like(a)
    a.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().float().requires_grad_(True)
    br = lin.bias.detach().float().requires_grad_(True)
    ar = F.gelu(xr @ wr.t() + br)
    ar.backward(g.float())
    assert _rel(a, ar) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(lin.weight.grad, wr.grad) < 2e-2
    assert _rel(lin.bias.grad, br.grad) < 2e-2
