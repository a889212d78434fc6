"""Fused BERT FFN (ops.transformer.ffn_gelu on csrc/kernels/gemm.hip) against the fp32 PyTorch
composition fc2(gelu(fc1(x))): output and every gradient (x, W1, b1, W2, b2), plus the batched
virtual-worker path (per-worker weight / bias gradients into the engine's rows)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _layers(d, f, dev, seed=0):
    torch.manual_seed(seed)
    from consensusml_amd.ops.transformer import Linear
    fc1, fc2 = Linear(d, f), Linear(f, d)
    for m in (fc1, fc2):
        nn.init.normal_(m.weight, std=0.05)
        nn.init.normal_(m.bias, std=0.5)
    return fc1.to(dev, torch.bfloat16), fc2.to(dev, torch.bfloat16)


@pytest.mark.parametrize("B,S,d,f", [(4, 128, 256, 1024), (8, 128, 768, 3072)])
def test_ffn_gelu_vs_fp32(cuda, B, S, d, f):
    from consensusml_amd.ops.transformer import _FFNGeluFn, ffn_gelu
    fc1, fc2 = _layers(d, f, cuda)
    x = torch.randn(B, S, d, device=cuda).bfloat16().requires_grad_(True)
    y = ffn_gelu(x, fc1, fc2)
    assert y.grad_fn is not None and "FFNGelu" in type(y.grad_fn).__name__
    dy = torch.randn_like(y)
    y.backward(dy)
    # fp32 oracle
    xf = x.detach().float().requires_grad_(True)
    W1, b1, W2, b2 = (p.detach().float().requires_grad_(True)
                      for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias))
    yf = F.linear(F.gelu(F.linear(xf, W1, b1)), W2, b2)
    yf.backward(dy.float())
    assert _rel(y, yf) < 1e-2
    assert _rel(x.grad, xf.grad) < 1.5e-2
    assert _rel(fc1.weight.grad, W1.grad) < 1.5e-2
    assert _rel(fc1.bias.grad, b1.grad) < 1.5e-2
    assert _rel(fc2.weight.grad, W2.grad) < 1.5e-2
    assert _rel(fc2.bias.grad, b2.grad) < 1.5e-2


def test_ffn_gelu_matches_unfused_bf16(cuda):
    """Same rounding points as the bf16 composition: the fused and unfused paths agree to the
    GEMMs' summation-order differences."""
    from consensusml_amd import perf
    from consensusml_amd.ops.transformer import ffn_gelu
    fc1, fc2 = _layers(768, 3072, cuda, seed=3)
    x = torch.randn(4, 128, 768, device=cuda).bfloat16()
    outs = {}
    for fused in (True, False):
        with perf.use_policy(perf.policy().replace(fused_ffn=fused)):
            for p in (*fc1.parameters(), *fc2.parameters()):
                p.grad = None
            xi = x.clone().requires_grad_(True)
            y = ffn_gelu(xi, fc1, fc2)
            y.backward(torch.ones_like(y))
            outs[fused] = [y.detach(), xi.grad, fc1.weight.grad.clone(), fc1.bias.grad.clone(),
                           fc2.weight.grad.clone(), fc2.bias.grad.clone()]
    for a, b in zip(outs[True], outs[False]):
        assert _rel(a, b) < 6e-3


def test_linear_own_gemm_with_link(cuda):
    """ops.transformer.linear on gemm.hip (>= 128 tiles): forward with bias, data gradient against
    the transposed weight with the parked residual gradient added in place (ResidualLink)."""
    from consensusml_amd.ops.bn import ResidualLink
    from consensusml_amd.ops.transformer import _own_gemm, linear
    M, N, K = 16384, 3072, 768
    assert _own_gemm(M, N, K) and _own_gemm(M, K, N)
    torch.manual_seed(1)
    x = torch.randn(M, K, device=cuda).bfloat16().requires_grad_(True)
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16().requires_grad_(True)
    b = torch.randn(N, device=cuda).bfloat16().requires_grad_(True)
    link = ResidualLink()
    y = linear(x, w, b, link)
    g_res = torch.randn(M, K, device=cuda).bfloat16()
    link.grad = g_res.clone()
    dy = torch.randn_like(y)
    y.backward(dy)
    xf, wf, bf = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yf = F.linear(xf, wf, bf)
    yf.backward(dy.float())
    assert _rel(y, yf) < 4e-3
    assert _rel(x.grad, xf.grad + g_res.float()) < 6e-3
    assert _rel(w.grad, wf.grad) < 6e-3
    assert _rel(b.grad, bf.grad) < 1e-2


def test_ffn_batched_workers_unowned_biases(cuda):
    """a worker-gradients object owning W1 / W2 but NOT b1 / b2 -- the bias gradients
    must still reach autograd (summed over the batch), not vanish into a scratch row."""
    from consensusml_amd.ops import worker_grads as WG
    from consensusml_amd.ops.transformer import ffn_gelu
    V, S, d, f = 2, 128, 256, 1024
    fc1, fc2 = _layers(d, f, cuda, seed=5)
    views = {id(fc1.weight): torch.zeros(V, f, d, device=cuda, dtype=torch.bfloat16),
             id(fc2.weight): torch.zeros(V, d, f, device=cuda, dtype=torch.bfloat16)}
    wg = WG.WorkerGrads(V, views)
    x = torch.randn(V * 2, S, d, device=cuda).bfloat16()
    prev = WG.activate(wg)
    try:
        y = ffn_gelu(x, fc1, fc2)
        dy = torch.randn_like(y)
        y.backward(dy)
    finally:
        WG.activate(prev)
    assert fc1.bias.grad is not None and fc2.bias.grad is not None
    W1, b1, W2, b2 = (p.detach().float().requires_grad_(True)
                      for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias))
    yf = F.linear(F.gelu(F.linear(x.float(), W1, b1)), W2, b2)
    yf.backward(dy.float())
    assert _rel(fc1.bias.grad, b1.grad) < 1.5e-2
    assert _rel(fc2.bias.grad, b2.grad) < 1.5e-2
    # the owned weights got per-worker rows summing to the full gradient
    assert _rel(views[id(fc1.weight)].float().sum(0), W1.grad) < 2e-2
