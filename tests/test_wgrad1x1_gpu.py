"""1x1-conv weight gradient on csrc/kernels/wgrad1x1.hip vs an fp32 PyTorch reference."""
import pytest
import torch

from consensusml_amd.ops.native import lib

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N,ci,co,hw", [(3, 128, 256, 7), (8, 512, 128, 14), (2, 256, 1024, 5),
                                        (2, 2048, 512, 7), (64, 128, 128, 28)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad1x1_vs_fp32(cuda, N, ci, co, hw, dtype):
    torch.manual_seed(ci + co + hw)
    x = torch.randn(N, ci, hw, hw, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, co, hw, hw, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dw = lib().wgrad1x1(dy, x, dtype)
    assert dw.shape == (co, ci, 1, 1) and dw.dtype == dtype
    X = x.permute(0, 2, 3, 1).reshape(-1, ci).float()
    D = dy.permute(0, 2, 3, 1).reshape(-1, co).float()
    ref = (D.t() @ X).view(co, ci, 1, 1)
    assert _rel(dw, ref) < (6e-3 if dtype == torch.bfloat16 else 1e-5)


def test_conv1x1_module_own_wgrad_matches_miopen(cuda):
    import consensusml_amd.models.resnet as R
    torch.manual_seed(3)
    conv = R.Conv1x1(256, 1024).to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(16, 256, 14, 14, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    dy = torch.randn(16, 1024, 14, 14, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = {}
    for own in (True, False):
        from consensusml_amd import perf
        with perf.use_policy(perf.policy().replace(own_wgrad1x1=own)):
            conv.weight.grad = None
            x.grad = None
            conv(x).backward(dy)
            out[own] = (conv.weight.grad.float().clone(), x.grad.float().clone())
    assert _rel(out[True][0], out[False][0]) < 1e-2
    assert _rel(out[True][1], out[False][1]) < 1e-2


@pytest.mark.parametrize("S,n", [(1, 64), (7, 4096), (31, 256), (32, 256), (100, 4100),
                                 (2048, 4096), (2048, 64), (129, 65536), (8, 262144)])
@pytest.mark.parametrize("bf16", [False, True])
def test_split_fold_vs_fp64(cuda, S, n, bf16):
    """The split-K fold (narrow kernel below 32 splits, wide 16-lane kernel from 32) against an
    fp64 sum; bitwise repeatable."""
    torch.manual_seed(S * 7 + n)
    part = torch.randn(S, n, device=cuda)
    out = lib().split_fold(part, bf16)
    assert out.shape == (n,) and out.dtype == (torch.bfloat16 if bf16 else torch.float32)
    ref = part.double().sum(0)
    assert _rel(out, ref) < (6e-3 if bf16 else 1e-6)
    assert torch.equal(out, lib().split_fold(part, bf16))


@pytest.mark.parametrize("N,ci,co,hw", [(32, 1024, 256, 14), (16, 512, 128, 28), (32, 128, 512, 28),
                                        (32, 1024, 2048, 7), (64, 256, 256, 4), (2, 256, 256, 4)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_wgrad1x1_dma_vs_fp32(cuda, N, ci, co, hw, dtype):
    """The LDS-DMA variant (plain weight gradient, P % 32 == 0, 256 x 256 / 128 x 256 / 256 x 128
    tiles; down to one 32-pixel chunk) against fp32; bitwise repeatable."""
    torch.manual_seed(ci * 3 + co + hw)
    x = torch.randn(N, ci, hw, hw, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(N, co, hw, hw, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dw = lib().wgrad1x1(dy, x, dtype)
    X = x.permute(0, 2, 3, 1).reshape(-1, ci).float()
    D = dy.permute(0, 2, 3, 1).reshape(-1, co).float()
    ref = (D.t() @ X).view(co, ci, 1, 1)
    assert _rel(dw, ref) < (6e-3 if dtype == torch.bfloat16 else 1e-5)
    assert torch.equal(dw, lib().wgrad1x1(dy, x, dtype))
