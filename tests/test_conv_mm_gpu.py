"""1x1 convolutions that run as plain GEMMs (ResNet-50 layers 3-4: forward when cin >= 1024, data
gradient with the parked residual gradient added in place) on gemm.hip instead of hipBLASLt
(``ops.conv.conv_mm``), against fp32 PyTorch oracles."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,K,N", [(32768, 1024, 256), (32768, 256, 1024), (65536, 512, 2048),
                                   (12544, 2048, 512)])
def test_conv_mm_vs_fp32(cuda, M, K, N):
    """(12544, 2048, 512): a batch-256 layer-4 GEMM, 98 tiles of 256 x 256 -> the 128 x 128 kernel"""
    from consensusml_amd.ops import conv as fconv
    g = torch.Generator(device=cuda).manual_seed(0)
    a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    acc0 = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    ref = a.float() @ w.float().t()
    before = dict(fconv.CONV_MM_STATS)
    y = fconv.conv_mm(a, w)
    acc = acc0.clone()
    y2 = fconv.conv_mm(a, w, acc=acc)
    assert fconv.CONV_MM_STATS["own"] == before["own"] + 2
    small = (M // 256) * (N // 256) < 128
    assert fconv.CONV_MM_STATS["own128"] == before["own128"] + (2 if small else 0)
    assert y2.data_ptr() == acc.data_ptr()            # in place into the residual gradient
    assert _rel(y, ref) < 5e-3
    assert _rel(y2, ref + acc0.float()) < 5e-3
    # the transposed-weight form of the data gradient (w_nk = W^T, a strided view)
    wt = w.t()
    dy = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    d = fconv.conv_mm(dy, wt)
    assert d.shape == (M, K)
    assert _rel(d, dy.float() @ w.float()) < 5e-3


def test_conv1x1_module_on_own_gemm(cuda):
    """Conv1x1 (gemm policy) at a layer-3 shape: forward, data and weight gradients vs fp32 conv2d,
    and both GEMMs took gemm.hip."""
    from consensusml_amd import perf
    from consensusml_amd.models import resnet as R
    from consensusml_amd.ops import conv as fconv
    torch.manual_seed(0)
    m = R.Conv1x1(1024, 256).to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(128, 1024, 16, 16, device=cuda, dtype=torch.bfloat16)
    x = x.to(memory_format=torch.channels_last).requires_grad_(True)
    before = fconv.CONV_MM_STATS["own"]
    with perf.use_policy(perf.policy().replace(conv1x1_gemm="gemm")):
        y = m(x)
        g = torch.randn_like(y)
        y.backward(g)
    assert fconv.CONV_MM_STATS["own"] == before + 2
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr)
    yr.backward(g.float())
    assert _rel(y, yr) < 5e-3
    assert _rel(x.grad, xr.grad) < 5e-3
    assert _rel(m.weight.grad, wr.grad) < 1e-2


def test_conv_mm_policy_off_uses_hipblaslt(cuda):
    from consensusml_amd import perf
    from consensusml_amd.ops import conv as fconv
    a = torch.randn(32768, 1024, device=cuda).bfloat16()
    w = torch.randn(256, 1024, device=cuda).bfloat16()
    before = dict(fconv.CONV_MM_STATS)
    with perf.use_policy(perf.policy().replace(own_gemm_conv1x1=False)):
        y = fconv.conv_mm(a, w)
    assert fconv.CONV_MM_STATS["blas"] == before["blas"] + 1
    assert _rel(y, a.float() @ w.float().t()) < 5e-3
