"""Stride-1 3x3 convolutions on gemm.hip's schedule (``launch_gemm_conv``: implicit-GEMM A
operand gathered per tap by the DMA path, 16x16x32 MFMAs, four staggered phases per k-tile), which
conv_gemm.hip routes to when the 256 x 256 tile grid applies and the pixel count is a multiple of
256: plain output, the BN-statistics epilogue and the BN + ReLU backward sums epilogue, against
fp32 / fp64 PyTorch oracles. Shapes: ResNet-50 layer-3 / layer-4 channel counts (256 / 512),
image borders on every side (padded taps read the zero row); and the 512 x 128 tall tile of the
128-channel (layer-2) convs, taken from 1024 such tiles (672 images of 28 x 28)."""
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


# (images, C, Co, H): M = images H H is a multiple of 256
SHAPES = [(4, 256, 256, 16), (16, 512, 512, 8), (4, 64, 256, 16), (64, 256, 512, 14),
          (672, 128, 128, 28), (672, 64, 128, 28), (256, 512, 512, 7)]
TALL = [(672, 128, 128, 28), (672, 64, 128, 28)]


@pytest.mark.parametrize("N,C,Co,H", TALL)
def test_tall_tile_taken(cuda, N, C, Co, H):
    assert _lib().gemm_conv_tm(N * H * H, Co, C) == 512
    assert _lib().gemm_conv_tm(N * H * H, 256, C) == 256
    assert _lib().gemm_conv_tm(256 * H * H, Co, C) == 0      # 392 tiles: conv_gemm.hip


@pytest.mark.parametrize("N,C,Co,H", SHAPES)
def test_gemm_conv_forward_vs_fp32(cuda, N, C, Co, H):
    g0 = torch.Generator(device=cuda).manual_seed(31)
    x = _nhwc((torch.randn(N, C, H, H, device=cuda, generator=g0) + 0.25).bfloat16())
    w = (torch.randn(Co, C, 3, 3, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    assert (N * H * H) % 256 == 0
    wf = w.permute(0, 2, 3, 1).reshape(Co, 9 * C).contiguous()
    y = _lib().conv_gemm(x, wf, 9)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert _rel(y, ref) < 5e-3
    # every pixel: the border rows / columns (padded taps) are as close as the interior
    err = (y.float() - ref).abs().amax(1)
    assert float(err[:, 0, :].max()) < 8 * float(err[:, H // 2, :].max()) + 1e-2


@pytest.mark.parametrize("N,C,Co,H", SHAPES[:6])
def test_gemm_conv_bn_stats_and_grads(cuda, N, C, Co, H):
    """conv3x3_bn_stats (forward + statistics epilogue) and the data gradient through the rotated
    weights (a plain gemm conv when C % 256 == 0) vs fp32 autograd."""
    from consensusml_amd.ops import conv as fconv
    g0 = torch.Generator(device=cuda).manual_seed(32)
    x = _nhwc((torch.randn(N, C, H, H, device=cuda, generator=g0) + 0.3).bfloat16())
    w = (torch.randn(Co, C, 3, 3, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    conv = torch.nn.Conv2d(C, Co, 3, padding=1, bias=False).to(cuda, torch.bfloat16)
    bn = torch.nn.BatchNorm2d(Co).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(w)
        bn.running_mean.copy_(torch.randn(Co, device=cuda, generator=g0) * 0.1)
    xi = x.clone().requires_grad_(True)
    z, (mean, invstd) = fconv.conv3x3_bn_stats(xi, conv, bn)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert _rel(z, ref) < 5e-3
    zb = z.float()
    torch.testing.assert_close(mean, zb.mean((0, 2, 3)), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(invstd, (zb.var((0, 2, 3), unbiased=False) + bn.eps).rsqrt(),
                               rtol=1e-3, atol=1e-3)
    gy = _nhwc(torch.randn(z.shape, device=cuda, generator=g0).bfloat16())
    z.backward(gy)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(gy.float())
    assert _rel(xi.grad, xr.grad) < 5e-3
    assert _rel(conv.weight.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("N,C,Co,H", SHAPES[:6])
def test_gemm_conv_bnsums_vs_fp64(cuda, N, C, Co, H):
    g0 = torch.Generator(device=cuda).manual_seed(33)
    x = _nhwc(torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16())
    z = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, 9 * C, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    zero = torch.zeros(64, device=cuda, dtype=torch.bfloat16)
    gam = (torch.rand(Co, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = (torch.randn(Co, device=cuda, generator=g0) * 0.1).bfloat16()
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


@pytest.mark.parametrize("N,C,Co,H", [(16, 256, 256, 14), (672, 128, 128, 28)])
def test_gemm_conv_deterministic(cuda, N, C, Co, H):
    g0 = torch.Generator(device=cuda).manual_seed(34)
    x = _nhwc(torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, 9 * C, device=cuda, generator=g0) * 0.02).bfloat16()
    a = _lib().conv_gemm(x, w, 9)
    b = _lib().conv_gemm(x, w, 9)
    assert torch.equal(a, b)


# stride-2 forwards on gemm.hip's gather (input grid IH x IW, output ((IH - 1) / 2 + 1)^2): the
# tall tile takes the 128-channel one (672 x 28 x 28 outputs); the 256-channel shape stays on
# conv_gemm.hip (the square tile was no faster there) and checks that route too
S2_SHAPES = [(672, 128, 128, 56), (768, 128, 256, 28)]


@pytest.mark.parametrize("N,C,Co,H", S2_SHAPES)
def test_gemm_conv_stride2_forward_and_stats(cuda, N, C, Co, H):
    g0 = torch.Generator(device=cuda).manual_seed(35)
    x = _nhwc((torch.randn(N, C, H, H, device=cuda, generator=g0) + 0.25).bfloat16())
    w = (torch.randn(Co, C, 3, 3, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    wf = w.permute(0, 2, 3, 1).reshape(Co, 9 * C).contiguous()
    Ho = (H - 1) // 2 + 1
    zero = torch.zeros(256, device=cuda, dtype=torch.bfloat16)
    y = _lib().conv_gemm(x, wf, 9, zero, 2)
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=1)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 5e-3
    err = (y.float() - ref).abs().amax(1)   # the padded top row / left column too
    assert float(err[:, 0, :].max()) < 8 * float(err[:, Ho // 2, :].max()) + 1e-2
    rm, rv = torch.zeros(Co, device=cuda), torch.ones(Co, device=cuda)
    y2, mean, invstd = _lib().conv_gemm_bn(x, wf, 9, zero, rm, rm, rv, 1e-5, 0.1, 2)
    assert torch.equal(y2, y)
    yb = y.float()
    torch.testing.assert_close(mean, yb.mean((0, 2, 3)), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(invstd, (yb.var((0, 2, 3), unbiased=False) + 1e-5).rsqrt(),
                               rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("N,C,Co,H", [(4, 256, 256, 16), (16, 64, 128, 28)])
def test_gemm_conv_bnsums_dgamma_dbeta(cuda, N, C, Co, H):
    """The BN parameter gradients from the sums' finalize launch equal bn_bwd_coeffs' values."""
    g0 = torch.Generator(device=cuda).manual_seed(36)
    x = _nhwc(torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16())
    z = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, 9 * C, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    zero = torch.zeros(64, device=cuda, dtype=torch.bfloat16)
    gam = (torch.rand(Co, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = (torch.randn(Co, device=cuda, generator=g0) * 0.1).bfloat16()
    Z = _rows(z).double()
    mean = Z.mean(0).float()
    invstd = (Z.var(0, unbiased=False) + 1e-5).rsqrt().float()
    sc = gam.float() * invstd
    bi = bet.float() - mean * sc
    dg, db = torch.empty_like(gam), torch.empty_like(bet)
    y, s, q = _lib().conv_gemm_bnsums(x, w, 9, zero, z, sc, bi, mean, invstd, dg, db)
    y2, s2, q2 = _lib().conv_gemm_bnsums(x, w, 9, zero, z, sc, bi, mean, invstd)
    assert torch.equal(y, y2) and torch.equal(s, s2) and torch.equal(q, q2)
    _, _, _, dg_ref, db_ref = _lib().bn_bwd_coeffs(s, q, gam, mean, invstd, N * H * H)
    assert torch.equal(dg, dg_ref) and torch.equal(db, db_ref)
