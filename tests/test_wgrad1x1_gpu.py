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


def _rows(t):
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).float()


def _bits(mask, C):
    sh = torch.arange(8, device=mask.device, dtype=torch.uint8)
    return ((mask.unsqueeze(-1) >> sh) & 1).reshape(mask.shape[0], C).float()


@pytest.mark.parametrize("N,ci,co,hw", [(32, 256, 1024, 7), (8, 128, 512, 14), (32, 256, 256, 7),
                                        (8, 512, 128, 14), (2, 256, 256, 4)])
@pytest.mark.parametrize("pro", [False, True])
@pytest.mark.parametrize("colsum", [False, True])
def test_wgrad1x1_dma_prologues(cuda, N, ci, co, hw, pro, colsum):
    """The DMA kernel's in-LDS transforms: x prologue max(x sc + bi, 0) and the mode-2 dy
    prologue a (mask ? dy : 0) + c (Co % 256 == 0) with its column sums, against fp32 on the same
    bf16 rounding points; the plain and x-prologue calls at Co = 128 too (128 x 256 tile)."""
    g0 = torch.Generator(device=cuda).manual_seed(ci + co + hw + 7 * pro + colsum)
    dy = torch.randn(N, co, hw, hw, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    x = torch.randn(N, ci, hw, hw, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    M = N * hw * hw
    sc = torch.rand(ci, device=cuda, generator=g0) + 0.5
    bi = torch.randn(ci, device=cuda, generator=g0) * 0.1
    X = torch.relu(_rows(x) * sc + bi).bfloat16().float() if pro else _rows(x)
    if co % 256:
        if colsum:
            pytest.skip("mode 2 needs Co % 256 == 0 on the DMA kernel")
        dw = lib().wgrad1x1(dy, x, torch.float32, sc if pro else None, bi if pro else None)
        ref = _rows(dy).t() @ X
        assert _rel(dw.view(co, ci), ref) < 1e-5
        return
    mask = torch.randint(0, 256, (M, co // 8), device=cuda, generator=g0, dtype=torch.uint8)
    a = torch.randn(co, device=cuda, generator=g0)
    c = torch.randn(co, device=cuda, generator=g0) * 0.1
    dw, cs = lib().wgrad1x1_ex(dy, x, sc if pro else None, bi if pro else None, 2, mask, a, None,
                               c, colsum)
    D = (a * (_bits(mask, co) * _rows(dy)) + c).bfloat16().float()
    assert _rel(dw, D.t() @ X) < 2e-4   # (the reference rounds a * u + c unfused: 1-ulp bf16 ties)
    if colsum:
        torch.testing.assert_close(cs, D.sum(0), rtol=1e-4, atol=1e-3 * M ** 0.5)
    dw2, cs2 = lib().wgrad1x1_ex(dy, x, sc if pro else None, bi if pro else None, 2, mask, a,
                                 None, c, colsum)
    assert torch.equal(dw, dw2) and (not colsum or torch.equal(cs, cs2))


@pytest.mark.parametrize("T,N,K", [(8192, 4096, 4096), (4096, 6144, 4096), (2048, 4096, 7168),
                                   (8192, 2048, 4096)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("use_out", [False, True])
def test_wgrad1x1_one_split_direct(cuda, T, N, K, dtype, use_out):
    """Long-K transformer-linear shapes (>= 256 output tiles of 256 x 256: one split on the DMA
    kernel): dW is written by the kernel itself, no partial slab and no fold, optionally into a
    caller-given destination (a view of a flat gradient row)."""
    torch.manual_seed(T + N + K)
    dy = torch.randn(T, N, device=cuda).to(torch.bfloat16)
    x = torch.randn(T, K, device=cuda).to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = None
    if use_out:
        row = torch.full((N * K + 64,), float("nan"), device=cuda, dtype=dtype)
        out = row[64:64 + N * K]          # 16-B aligned view at an offset
    dw = lib().wgrad1x1(dy.view(T, 1, 1, N).permute(0, 3, 1, 2),
                        x.view(T, 1, 1, K).permute(0, 3, 1, 2), dtype, out=out)
    if use_out:
        assert dw.data_ptr() == out.data_ptr()
        assert torch.isnan(row[:64]).all()   # nothing written outside the destination
    assert _rel(dw.view(N, K), ref) < (6e-3 if dtype == torch.bfloat16 else 1e-5)
