"""Fused 1x1 conv + BatchNorm statistics (csrc/kernels/conv1x1.hip) and the BN-ReLU prologue of
the MFMA weight gradient (wgrad1x1.hip) against fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

from consensusml_amd.ops import conv as C
from consensusml_amd.ops.native import lib

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _nhwc(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


SHAPES = [  # N, K (Cin), Cout, H (=W), stride
    (3, 64, 256, 7, 1),      # (1, 4) tile: ragged M = 147
    (2, 256, 64, 14, 1),     # W resident, K = 256
    (2, 128, 128, 9, 1),     # (2, 2) tile
    (4, 512, 128, 7, 1),     # streamed W
    (2, 128, 512, 8, 1),     # (4, 1) tile, 2 n-tiles
    (1, 1024, 2048, 5, 1),   # 8 n-tiles, K steps 16
    (2, 256, 512, 14, 2),    # downsample stride 2
    (2, 64, 256, 6, 2),
]


@pytest.mark.parametrize("N,K,Co,H,stride", SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_conv1x1_bn_fwd_vs_fp32(cuda, N, K, Co, H, stride, pro):
    if pro and stride == 2:
        pytest.skip("strided convs read a materialised input")
    torch.manual_seed(N * K + Co + H)
    x = _nhwc(torch.randn(N, K, H, H, device=cuda))
    w = (torch.randn(Co, K, 1, 1, device=cuda) / K ** 0.5).to(torch.bfloat16)
    sc = bi = None
    if pro:
        sc = torch.rand(K, device=cuda) + 0.5
        bi = torch.randn(K, device=cuda) * 0.3
    shift = torch.randn(Co, device=cuda) * 0.1
    rmean, rvar = shift.clone(), torch.ones(Co, device=cuda)
    y, mean, invstd = lib().conv1x1_bn_fwd(x, w, sc, bi, shift, rmean, rvar, stride, True,
                                           1e-5, 0.1)
    ref, rm, rv = C.reference_conv1x1_bn(x, w, stride, (sc, bi) if pro else None)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 8e-3
    torch.testing.assert_close(mean, rm, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(invstd, torch.rsqrt(rv + 1e-5), rtol=2e-3, atol=1e-4)
    M = ref.numel() // Co
    torch.testing.assert_close(rmean, 0.9 * shift + 0.1 * rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rvar, 0.9 + 0.1 * rv * M / (M - 1), rtol=2e-3, atol=1e-4)
    # statistics off: same output, no stats
    y2, m2, _ = lib().conv1x1_bn_fwd(x, w, sc, bi, None, None, None, stride, False, 1e-5, 0.1)
    assert torch.equal(y, y2) and m2 is None


def test_conv1x1_bn_stats_large_mean(cuda):
    """Shifted sums: a channel mean 100x its std still gives an accurate variance once the
    running mean (the shift) is near the batch mean."""
    torch.manual_seed(0)
    x = _nhwc(torch.randn(8, 64, 16, 16, device=cuda) * 0.05 + 1.0)
    w = torch.ones(128, 64, 1, 1, device=cuda).to(torch.bfloat16) / 8
    ref, rm, rv = C.reference_conv1x1_bn(x, w)
    shift = rm.clone()
    _, mean, invstd = lib().conv1x1_bn_fwd(x, w, None, None, shift, None, None, 1, True, 1e-5, 0.1)
    torch.testing.assert_close(mean, rm, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(invstd, torch.rsqrt(rv + 1e-5), rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("N,ci,co,hw", [(4, 64, 256, 14), (3, 128, 512, 7), (2, 256, 1024, 5),
                                        (2, 512, 2048, 7)])
def test_wgrad1x1_prologue_vs_fp32(cuda, N, ci, co, hw):
    torch.manual_seed(ci + co)
    z = _nhwc(torch.randn(N, ci, hw, hw, device=cuda))
    dy = _nhwc(torch.randn(N, co, hw, hw, device=cuda))
    sc = torch.rand(ci, device=cuda) + 0.5
    bi = torch.randn(ci, device=cuda) * 0.3
    dw = lib().wgrad1x1(dy, z, torch.float32, sc, bi)
    y = torch.relu(z.float() * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1)).to(torch.bfloat16)
    X = y.permute(0, 2, 3, 1).reshape(-1, ci).float()
    D = dy.permute(0, 2, 3, 1).reshape(-1, co).float()
    assert _rel(dw, (D.t() @ X).view(co, ci, 1, 1)) < 1e-4
    if ci == 64:   # the new 64-channel tile without prologue too
        dw0 = lib().wgrad1x1(dy, z, torch.float32)
        X0 = z.permute(0, 2, 3, 1).reshape(-1, ci).float()
        assert _rel(dw0, (D.t() @ X0).view(co, ci, 1, 1)) < 1e-4


def _bn_ref(z, g, b, eps=1e-5):
    m = z.mean((0, 2, 3), keepdim=True)
    v = z.var((0, 2, 3), unbiased=False, keepdim=True)
    return (z - m) / torch.sqrt(v + eps) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


@pytest.mark.parametrize("ci,co,hw", [(64, 256, 14), (128, 512, 7)])
def test_bnrelu_conv_autograd_vs_fp32(cuda, ci, co, hw):
    """z3 = conv(relu(bn2(z2))) and bn3's statistics, forward and backward (dz2, dgamma2,
    dbeta2, dW3) against the fp32 composition."""
    from consensusml_amd.ops.bn import BatchNormAct2d
    torch.manual_seed(ci)
    N = 4
    bn2 = BatchNormAct2d(ci).to(cuda, torch.bfloat16)
    bn3 = BatchNormAct2d(co).to(cuda, torch.bfloat16)
    with torch.no_grad():
        bn2.weight.copy_(torch.rand(ci) + 0.5)
        bn2.bias.copy_(torch.randn(ci) * 0.2)
    conv = torch.nn.Conv2d(ci, co, 1, bias=False).to(cuda, torch.bfloat16)
    z2 = _nhwc(torch.randn(N, ci, hw, hw, device=cuda)).requires_grad_(True)
    stats = C.bn_stats(z2.detach(), bn2)
    z3, m3, i3 = C.bnrelu_conv1x1_bn_stats(z2, bn2, stats, conv, bn3)
    g3 = _nhwc(torch.randn_like(z3.float()))
    z3.backward(g3)
    # fp32 reference
    zr = z2.detach().float().requires_grad_(True)
    gr = bn2.weight.detach().float().requires_grad_(True)
    br = bn2.bias.detach().float().requires_grad_(True)
    wr = conv.weight.detach().float().requires_grad_(True)
    yr = F.conv2d(torch.relu(_bn_ref(zr, gr, br)), wr)
    yr.backward(g3.float())
    assert _rel(z3, yr) < 1e-2
    torch.testing.assert_close(m3, yr.detach().mean((0, 2, 3)), rtol=2e-2, atol=2e-3)
    assert _rel(z2.grad, zr.grad) < 3e-2
    assert _rel(bn2.weight.grad, gr.grad) < 3e-2
    assert _rel(bn2.bias.grad, br.grad) < 3e-2
    assert _rel(conv.weight.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1x1_bn_stats_autograd(cuda, stride):
    from consensusml_amd.ops.bn import BatchNormAct2d
    torch.manual_seed(5 + stride)
    bn = BatchNormAct2d(256).to(cuda, torch.bfloat16)
    conv = torch.nn.Conv2d(128, 256, 1, stride=stride, bias=False).to(cuda, torch.bfloat16)
    x = _nhwc(torch.randn(4, 128, 12, 12, device=cuda)).requires_grad_(True)
    z, m, i = C.conv1x1_bn_stats(x, conv, bn, stride)
    g = _nhwc(torch.randn_like(z.float()))
    z.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().float().requires_grad_(True)
    zr = F.conv2d(xr, wr, stride=stride)
    zr.backward(g.float())
    assert _rel(z, zr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(conv.weight.grad, wr.grad) < 1e-2
    torch.testing.assert_close(m, zr.detach().to(torch.bfloat16).float().mean((0, 2, 3)),
                               rtol=1e-3, atol=1e-4)


def test_resnet50_fused_conv_bn_matches_unfused(cuda):
    """Whole ResNet-50 training step (64 x 64 images, batch 16): the fused 1x1 conv + BN path is
    as accurate as the unfused bf16 path, both measured against an fp32 copy of the model.
    (Per block the two bf16 paths agree to rounding, tools/diag/fused_block_diag.py; through 16
    blocks of 64-value BatchNorms both drift to a gradient cosine of ~0.94 vs fp32.)"""
    import copy
    import consensusml_amd.models.resnet as R
    torch.manual_seed(11)
    m32 = R.resnet50(num_classes=10).to(cuda)
    with torch.no_grad():   # bn3 is zero-initialised: give the residual branches some weight
        for mod in m32.modules():
            if isinstance(mod, R.Bottleneck):
                mod.bn3.weight.fill_(0.2)
    x = torch.randn(16, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (16,), device=cuda)
    out = {}
    for name in ("fp32", "fused", "unfused"):
        m = copy.deepcopy(m32)
        xx = x
        if name != "fp32":
            m = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
            xx = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        from consensusml_amd import perf
        with perf.use_policy(perf.policy().replace(fused_conv1x1=name == "fused")):
            loss = F.cross_entropy(m(xx).float(), y)
            loss.backward()
        out[name] = (loss.item(), torch.cat([p.grad.float().flatten() for p in m.parameters()]),
                     {k: b.float().clone() for k, b in m.named_buffers()})
    cf = F.cosine_similarity(out["fused"][1], out["fp32"][1], dim=0).item()
    cu = F.cosine_similarity(out["unfused"][1], out["fp32"][1], dim=0).item()
    assert cf > cu - 0.02 and cf > 0.85, (cf, cu)
    assert abs(out["fused"][0] - out["fp32"][0]) < 1e-2 * max(1.0, abs(out["fp32"][0]))
    for k in out["fp32"][2]:
        if "running" in k:
            torch.testing.assert_close(out["fused"][2][k], out["unfused"][2][k], rtol=2e-2,
                                       atol=2e-3)


@pytest.mark.parametrize("C,Co,H", [(64, 64, 9), (128, 128, 7), (256, 256, 5), (512, 512, 4),
                                    (64, 128, 6), (128, 64, 5)])
def test_conv_gemm_and_3x3_dgrad(cuda, C, Co, H):
    """conv_gemm.hip: forward 3x3 / 1x1 implicit GEMM vs fp32, and the 3x3 data gradient of
    ops.conv.conv3x3 vs the fp32 autograd gradient."""
    import torch.nn.functional as F
    from consensusml_amd.ops import conv as fconv
    from consensusml_amd.ops.native import lib
    g0 = torch.Generator(device=cuda).manual_seed(9)
    N = 3
    x = torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 3, 3, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    y = lib().conv_gemm(x, w.permute(0, 2, 3, 1).reshape(Co, 9 * C).contiguous(), 9)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert float((y.float() - ref).norm() / ref.norm()) < 5e-3
    y1 = lib().conv_gemm(x, w[:, :, 1, 1].contiguous(), 1)
    ref1 = F.conv2d(x.float(), w[:, :, 1:2, 1:2].float())
    assert float((y1.float() - ref1).norm() / ref1.norm()) < 5e-3
    conv = torch.nn.Conv2d(C, Co, 3, padding=1, bias=False).to(cuda, torch.bfloat16)
    with torch.no_grad():
        conv.weight.copy_(w)
    xi = x.clone().requires_grad_(True)
    out = fconv.conv3x3(xi, conv)
    gy = torch.randn(out.shape, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    out.backward(gy)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(gy.float())
    assert float((xi.grad.float() - xr.grad).norm() / xr.grad.norm()) < 5e-3
    assert float((conv.weight.grad.float() - wr.grad).norm() / wr.grad.norm()) < 1e-2


@pytest.mark.parametrize("C,Co,H,N", [(64, 64, 9, 3), (128, 128, 7, 3), (256, 256, 5, 3),
                                      (512, 512, 4, 5), (64, 192, 6, 2), (128, 512, 14, 4),
                                      (64, 64, 66, 4), (128, 128, 40, 12)])
def test_conv3x3_bn_stats_vs_fp32(cuda, C, Co, H, N):
    """conv_gemm_bn (ops.conv.conv3x3_bn_stats): the output, the BN batch statistics of the bf16
    output (epilogue partial sums, shifted by the running mean), the running-stat update and the
    gradients vs fp32 PyTorch. Odd M exercises partial tiles, the two largest M the two-level
    fold of the partial slab."""
    import torch.nn.functional as F
    from consensusml_amd.ops import conv as fconv
    g0 = torch.Generator(device=cuda).manual_seed(12)
    x = (torch.randn(N, C, H, H, device=cuda, generator=g0) + 0.3).bfloat16().contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 3, 3, device=cuda, generator=g0) * (9 * C) ** -0.5).bfloat16()
    conv = torch.nn.Conv2d(C, Co, 3, padding=1, bias=False).to(cuda, torch.bfloat16)
    bn = torch.nn.BatchNorm2d(Co).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(w)
        bn.running_mean.copy_(torch.randn(Co, device=cuda, generator=g0) * 0.1)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    xi = x.clone().requires_grad_(True)
    z, (mean, invstd) = fconv.conv3x3_bn_stats(xi, conv, bn)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert float((z.float() - ref).norm() / ref.norm()) < 5e-3
    zb = z.float()
    M = N * H * H
    m_ref, v_ref = zb.mean((0, 2, 3)), zb.var((0, 2, 3), unbiased=False)
    torch.testing.assert_close(mean, m_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(invstd, (v_ref + bn.eps).rsqrt(), rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(bn.running_mean, 0.9 * rm0 + 0.1 * m_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_var, 0.9 * rv0 + 0.1 * v_ref * M / (M - 1),
                               rtol=1e-3, atol=1e-4)
    gy = torch.randn(z.shape, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    z.backward(gy)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(gy.float())
    assert float((xi.grad.float() - xr.grad).norm() / xr.grad.norm()) < 5e-3
    assert float((conv.weight.grad.float() - wr.grad).norm() / wr.grad.norm()) < 1e-2


@pytest.mark.parametrize("C,Co,H,N", [(64, 64, 9, 4), (128, 128, 6, 4), (256, 256, 5, 4),
                                      (64, 256, 5, 4), (64, 64, 56, 2), (128, 128, 28, 2),
                                      (256, 256, 14, 3), (512, 512, 7, 4), (64, 128, 16, 3),
                                      (128, 256, 20, 2), (256, 128, 30, 1), (128, 64, 7, 3)])
def test_wgrad3x3_vs_fp32(cuda, C, Co, H, N):
    """3x3 weight gradient, nine taps per workgroup (wgrad3x3.hip: single-row to multi-image
    chunks, halo rows at image edges, channel tiles) vs the fp32 convolution weight gradient."""
    from consensusml_amd.ops.native import lib
    L = lib()
    assert L.wgrad3x3_direct_ok(N, H, H, Co, C), (N, H, Co, C)
    g0 = torch.Generator(device=cuda).manual_seed(12)
    x = torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    gy = torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16().contiguous(
        memory_format=torch.channels_last)
    zero = torch.zeros(64, dtype=torch.bfloat16, device=cuda)
    dw = L.wgrad3x3(gy, x, torch.float32, zero)
    w = torch.zeros(Co, C, 3, 3, device=cuda)
    ref = torch.ops.aten.convolution_backward(gy.float(), x.float(), w, None, [1, 1], [1, 1],
                                              [1, 1], False, [0, 0], 1, [False, True, False])[1]
    assert float((dw.float() - ref).norm() / ref.norm()) < 1e-5 * (N * H * H) ** 0.5 + 1e-4
    dwb = L.wgrad3x3(gy, x, torch.bfloat16, zero)
    assert dwb.dtype == torch.bfloat16
    assert float((dwb.float() - ref).norm() / ref.norm()) < 5e-3

