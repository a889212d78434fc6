"""Stride-2 / padding-1 3x3 weight gradient on the wgrad DMA kernel (implicit im2col gather,
csrc/kernels/wgrad1x1.hip ``launch_wgrad3x3s2``) vs an fp32 PyTorch reference."""
import pytest
import torch

from consensusml_amd.ops.native import lib

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


# (N, Ci, Co, H, W): 128 x 128 / 256 x 256 / 256 x 128 / 128 x 256 tiles, non-square images,
# one 32-pixel chunk
@pytest.mark.parametrize("N,ci,co,H,W", [(8, 128, 128, 16, 16), (4, 256, 256, 8, 8),
                                         (8, 128, 256, 12, 12), (2, 512, 128, 8, 8),
                                         (4, 128, 128, 8, 16), (32, 256, 512, 14, 14)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad3x3s2_vs_fp32(cuda, N, ci, co, H, W, dtype):
    torch.manual_seed(N + ci + co + H + W)
    assert lib().wgrad3x3s2_ok(N, H, W, co, ci)
    x = torch.randn(N, ci, H, W, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, co, H // 2, W // 2, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dw = lib().wgrad3x3s2(dy, x, dtype)
    assert dw.shape == (co, ci, 3, 3) and dw.dtype == dtype
    ref = torch.nn.grad.conv2d_weight(x.float(), (co, ci, 3, 3), dy.float(), stride=2, padding=1)
    assert _rel(dw, ref) < (6e-3 if dtype == torch.bfloat16 else 1e-5)
    assert torch.equal(dw, lib().wgrad3x3s2(dy, x, dtype))


def test_wgrad3x3s2_plan_limits():
    assert not lib().wgrad3x3s2_ok(3, 7, 7, 128, 128)      # odd image
    assert not lib().wgrad3x3s2_ok(1, 10, 10, 128, 128)    # 25 output pixels: not % 32
    assert not lib().wgrad3x3s2_ok(8, 16, 16, 64, 128)     # Co not % 128
    assert lib().wgrad3x3s2_ok(2048, 56, 56, 128, 128)


def test_conv3x3_s2_module_own_wgrad_matches_miopen(cuda):
    """The ResNet stride-2 3x3 block conv's weight gradient with and without the own kernel."""
    from consensusml_amd import perf
    from consensusml_amd.ops import conv as C
    torch.manual_seed(5)
    x = torch.randn(32, 128, 16, 16, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(128, 128, 3, 3, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(32, 128, 8, 8, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = {}
    for own in (True, False):
        with perf.use_policy(perf.policy().replace(own_wgrad3x3_s2=own)):
            out[own] = C._wgrad3x3_s2(dy, x, w).float()
    assert _rel(out[True], out[False]) < 1e-2


# the 1x1 / stride 2 / padding 0 downsample (taps = 1: the single tap at (2 oh, 2 ow))
@pytest.mark.parametrize("N,ci,co,H,W", [(8, 128, 128, 16, 16), (4, 256, 512, 16, 16),
                                         (2, 1024, 256, 8, 8), (16, 128, 256, 8, 12)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad1x1s2_vs_fp32(cuda, N, ci, co, H, W, dtype):
    torch.manual_seed(N + ci + co + H + W + 1)
    assert lib().wgrad3x3s2_ok(N, H, W, co, ci, 1)
    x = torch.randn(N, ci, H, W, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, co, H // 2, W // 2, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dw = lib().wgrad3x3s2(dy, x, dtype, taps=1)
    assert dw.shape == (co, ci, 1, 1) and dw.dtype == dtype
    ref = torch.nn.grad.conv2d_weight(x.float(), (co, ci, 1, 1), dy.float(), stride=2, padding=0)
    assert _rel(dw, ref) < (6e-3 if dtype == torch.bfloat16 else 1e-5)


def test_downsample_s2_own_wgrad_matches_miopen(cuda):
    """ops.conv._wgrad for a stride-2 1x1 conv: own single-tap kernel vs MIOpen."""
    from consensusml_amd import perf
    from consensusml_amd.ops import conv as C
    torch.manual_seed(6)
    x = torch.randn(32, 256, 14, 14, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = torch.randn(512, 256, 1, 1, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(32, 512, 7, 7, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = {}
    for own in (True, False):
        with perf.use_policy(perf.policy().replace(own_wgrad1x1_s2=own)):
            out[own] = C._wgrad(dy, x, w, 2, True).float()
    assert out[True].shape == w.shape
    assert _rel(out[True], out[False]) < 1e-2
