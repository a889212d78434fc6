"""Patch-resident stride-1 3x3 conv (conv3x3p.hip: 64 -> 64 channels, 56-pixel-wide images, the
ResNet-50 layer-1 3x3 conv), which launch_conv_gemm / launch_conv_gemm_bnsums route to: plain
output, the BN-statistics epilogue and the BN + ReLU backward sums epilogue, against fp32 / fp64
PyTorch oracles. Heights cover one tile per image (4 rows), partial persistent ranges (tile
counts that do not divide by the grid) and the full 56 x 56 image; every image border (top /
bottom rows DMA'd from the zero buffer, left / right columns read from the LDS zero row)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from consensusml_amd.ops.native import lib
    return lib()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t):
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


# (images, H): W = 56 always; 4 x 14 = 56 tiles (grid = tiles), 37 x 14 = 518 tiles (uneven
# persistent ranges over 256 workgroups), 3 x 1, 5 x 3
SHAPES = [(4, 56), (37, 56), (3, 4), (5, 12)]


def _wf(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


@pytest.mark.parametrize("N,H", SHAPES)
def test_conv3x3p_forward_vs_fp32(cuda, N, H):
    g0 = torch.Generator(device=cuda).manual_seed(41)
    x = _nhwc((torch.randn(N, 64, H, 56, device=cuda, generator=g0) + 0.25).bfloat16())
    w = (torch.randn(64, 64, 3, 3, device=cuda, generator=g0) * 576 ** -0.5).bfloat16()
    y = _lib().conv_gemm(x, _wf(w), 9)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert _rel(y, ref) < 5e-3
    err = (y.float() - ref).abs()
    tol = 4 * float(err[:, :, 1:-1, 1:-1].amax()) + 1e-2
    # the borders (zero-row / zero-buffer taps) are as close as the interior
    for edge in (err[:, :, 0, :], err[:, :, -1, :], err[:, :, :, 0], err[:, :, :, -1]):
        assert float(edge.amax()) < tol


@pytest.mark.parametrize("N,H", SHAPES)
def test_conv3x3p_bn_stats(cuda, N, H):
    g0 = torch.Generator(device=cuda).manual_seed(42)
    x = _nhwc((torch.randn(N, 64, H, 56, device=cuda, generator=g0) + 0.3).bfloat16())
    w = (torch.randn(64, 64, 3, 3, device=cuda, generator=g0) * 576 ** -0.5).bfloat16()
    shift = torch.randn(64, device=cuda, generator=g0) * 0.1
    rm, rv = torch.zeros(64, device=cuda), torch.ones(64, device=cuda)
    y, mean, invstd = _lib().conv_gemm_bn(x, _wf(w), 9, None, shift, rm, rv, 1e-5, 0.1)
    assert _rel(y, F.conv2d(x.float(), w.float(), padding=1)) < 5e-3
    Y = _rows(y).double()
    torch.testing.assert_close(mean.double(), Y.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(invstd.double(), (Y.var(0, unbiased=False) + 1e-5).rsqrt(),
                               rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm.double(), 0.1 * Y.mean(0), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("N,H", SHAPES)
def test_conv3x3p_bnsums_vs_fp64(cuda, N, H):
    g0 = torch.Generator(device=cuda).manual_seed(43)
    x = _nhwc(torch.randn(N, 64, H, 56, device=cuda, generator=g0).bfloat16())
    z = _nhwc(torch.randn(N, 64, H, 56, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(64, 576, device=cuda, generator=g0) * 576 ** -0.5).bfloat16()
    zero = torch.zeros(64, device=cuda, dtype=torch.bfloat16)
    gam = (torch.rand(64, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = (torch.randn(64, device=cuda, generator=g0) * 0.1).bfloat16()
    Z = _rows(z).double()
    mean = Z.mean(0).float()
    invstd = (Z.var(0, unbiased=False) + 1e-5).rsqrt().float()
    sc = gam.float() * invstd
    bi = bet.float() - mean * sc
    y, s, q = _lib().conv_gemm_bnsums(x, w, 9, zero, z, sc, bi, mean, invstd)
    assert torch.equal(y, _lib().conv_gemm(x, w, 9, zero))
    m = (torch.addcmul(bi, _rows(z), sc) > 0).double()
    dyv = _rows(y).double() * m
    torch.testing.assert_close(s.double(), dyv.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(q.double(), (dyv * (Z - mean.double()) * invstd.double()).sum(0),
                               rtol=1e-5, atol=1e-3)


def test_conv3x3p_grads_through_model_op(cuda):
    """conv3x3_bn_stats forward + the data gradient through the rotated weights (both on the patch
    kernel at this shape) vs fp32 autograd."""
    from consensusml_amd.ops import conv as fconv
    g0 = torch.Generator(device=cuda).manual_seed(44)
    x = _nhwc((torch.randn(4, 64, 56, 56, device=cuda, generator=g0) + 0.3).bfloat16())
    w = (torch.randn(64, 64, 3, 3, device=cuda, generator=g0) * 576 ** -0.5).bfloat16()
    conv = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).to(cuda, torch.bfloat16)
    bn = torch.nn.BatchNorm2d(64).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(w)
    xi = x.clone().requires_grad_(True)
    z, (mean, invstd) = fconv.conv3x3_bn_stats(xi, conv, bn)
    assert _rel(z, F.conv2d(x.float(), w.float(), padding=1)) < 5e-3
    gy = _nhwc(torch.randn(z.shape, device=cuda, generator=g0).bfloat16())
    z.backward(gy)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(gy.float())
    assert _rel(xi.grad, xr.grad) < 5e-3
    assert _rel(conv.weight.grad, wr.grad) < 1e-2


def test_conv3x3p_deterministic(cuda):
    g0 = torch.Generator(device=cuda).manual_seed(45)
    x = _nhwc(torch.randn(37, 64, 56, 56, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(64, 576, device=cuda, generator=g0) * 0.04).bfloat16()
    a = _lib().conv_gemm_bn(x, w, 9)
    b = _lib().conv_gemm_bn(x, w, 9)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
