"""Stride-2 3x3 conv on conv_gemm.hip: the parity-class data gradient (``conv_gemm_s2dgrad``)
against PyTorch's fp32 transposed conv, its BN + ReLU backward sums against fp64, and a
downsample bottleneck's gradients with the own stride-2 path against the library path."""
import copy

import pytest
import torch

from consensusml_amd import perf
from consensusml_amd.ops.native import lib

pytestmark = pytest.mark.gpu


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t):
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).float()


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("N,Co,Ci,Ho", [(2, 128, 128, 7), (2, 256, 256, 7), (2, 512, 512, 4),
                                        (3, 64, 64, 5), (1, 64, 128, 3), (2, 128, 64, 6),
                                        (1, 256, 512, 1), (32, 256, 256, 64), (32, 128, 128, 64)])
def test_s2dgrad_vs_fp32(cuda, N, Co, Ci, Ho):
    """Small grids take the 128 x 128 tiles; the two 32 x 64 x 65 shapes (>= 512 tiles of 256 x
    256 per class) the 256 x 256 / 256 x 128 ones."""
    g0 = torch.Generator(device=cuda).manual_seed(31)
    dy = _nhwc(torch.randn(N, Co, Ho, Ho + 1, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, Ci, 3, 3, device=cuda, generator=g0) * (9 * Ci) ** -0.5).bfloat16()
    _, wr = lib().conv3x3_wlayouts(w, False)
    zero = torch.zeros(64, device=cuda, dtype=torch.bfloat16)
    dx = lib().conv_gemm_s2dgrad(dy, wr, zero)[0]
    assert dx.shape == (N, Ci, 2 * Ho, 2 * (Ho + 1))
    ref = torch.nn.grad.conv2d_input((N, Ci, 2 * Ho, 2 * (Ho + 1)), w.float(), dy.float(),
                                     stride=2, padding=1)
    assert _rel(dx.float(), ref) < 8e-3


@pytest.mark.parametrize("N,Co,Ci,Ho", [(2, 128, 128, 7), (2, 256, 256, 4), (2, 64, 64, 5)])
def test_s2dgrad_bnsums(cuda, N, Co, Ci, Ho):
    """With z: the sums of relu(bn(z))'s backward over dx, and bn_bwd_apply from them."""
    g0 = torch.Generator(device=cuda).manual_seed(32)
    dy = _nhwc(torch.randn(N, Co, Ho, Ho, device=cuda, generator=g0).bfloat16())
    z = _nhwc(torch.randn(N, Ci, 2 * Ho, 2 * Ho, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, Ci, 3, 3, device=cuda, generator=g0) * (9 * Ci) ** -0.5).bfloat16()
    _, wr = lib().conv3x3_wlayouts(w, False)
    zero = torch.zeros(64, device=cuda, dtype=torch.bfloat16)
    gam = (torch.rand(Ci, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = (torch.randn(Ci, device=cuda, generator=g0) * 0.1).bfloat16()
    Z = _rows(z).double()
    mean = Z.mean(0).float()
    invstd = (Z.var(0, unbiased=False) + 1e-5).rsqrt().float()
    sc = gam.float() * invstd
    bi = bet.float() - mean * sc
    y, s, q = lib().conv_gemm_s2dgrad(dy, wr, zero, z, sc, bi, mean, invstd)
    assert torch.equal(y, lib().conv_gemm_s2dgrad(dy, wr, zero)[0])
    m = (torch.addcmul(bi, _rows(z), sc) > 0).double()
    dyv = _rows(y).double() * m
    assert _rel(s, dyv.sum(0)) < 1e-5
    assert _rel(q, (dyv * (Z - mean.double()) * invstd.double()).sum(0)) < 1e-5
    dz = lib().bn_bwd_apply(y, z, gam, bet, mean, invstd, s, q)
    dz_ref, _, _, _ = lib().bn_bwd(y, None, z, None, gam, bet, mean, invstd, True, False)
    assert _rel(_rows(dz), _rows(dz_ref)) < 1e-2
    # the BN's parameter gradients from the sums' finalize launch == bn_bwd_coeffs' values
    dg, db = torch.empty_like(gam), torch.empty_like(bet)
    y2, s2, q2 = lib().conv_gemm_s2dgrad(dy, wr, zero, z, sc, bi, mean, invstd, dg, db)
    assert torch.equal(y2, y) and torch.equal(s2, s) and torch.equal(q2, q)
    _, _, _, dg_ref, db_ref = lib().bn_bwd_coeffs(s, q, gam, mean, invstd, Z.shape[0])
    assert torch.equal(dg, dg_ref) and torch.equal(db, db_ref)


@pytest.mark.parametrize("inplanes,planes,H", [(256, 128, 28), (512, 256, 14)])
def test_downsample_block_s2_matches_library_conv(cuda, monkeypatch, inplanes, planes, H):
    """A stride-2 downsample bottleneck: output and every gradient with the own stride-2 3x3 path
    (conv_gemm forward + statistics, parity-class dgrad + bn1 sums) vs MIOpen's conv2."""
    import consensusml_amd.models.resnet as R
    from consensusml_amd.ops import conv as fconv
    calls = []
    for name in ("bnrelu_conv3x3_s2_bn_stats", "conv3x3_s2_bn_stats"):
        fn = getattr(fconv, name)
        monkeypatch.setattr(fconv, name,
                            lambda *a, _fn=fn, _n=name, **k: (calls.append(_n), _fn(*a, **k))[1])
    torch.manual_seed(7)
    blk = R.Bottleneck(inplanes, planes, stride=2, downsample=True).to(cuda, torch.bfloat16)
    blk = blk.to(memory_format=torch.channels_last).train()
    x0 = _nhwc(torch.randn(4, inplanes, H, H, device=cuda).relu().bfloat16())
    gy = _nhwc(torch.randn(4, planes * 4, H // 2, H // 2, device=cuda).bfloat16())
    outs, grads = {}, {}
    for on in (True, False):
        with perf.use_policy(perf.policy().replace(own_conv3x3_s2=on)):
            b = copy.deepcopy(blk)
            x = x0.clone().requires_grad_(True)
            y = b(x)
            y.backward(gy)
        outs[on] = y.detach()
        grads[on] = [x.grad] + [p.grad for p in b.parameters()]
    assert calls, "the own stride-2 path did not run"
    assert _rel(outs[True].float(), outs[False].float()) < 2e-2
    for a, r in zip(grads[True], grads[False]):
        assert _rel(a.float(), r.float()) < 3e-2


def test_layer4_downsample_compact_matches_strided(cuda, monkeypatch):
    """Layer-4 downsample block (1024 -> 2048, 14 x 14 -> 7 x 7): the downsample conv as a stride-1
    GEMM of x[:, :, ::2, ::2] with its compact data gradient handed to conv1's data-gradient GEMM
    (PerfPolicy.down_s2_compact) vs MIOpen's stride-2 conv; output and every gradient."""
    import consensusml_amd.models.resnet as R
    calls = []
    orig = R.Bottleneck._down_conv_s2_compact
    monkeypatch.setattr(R.Bottleneck, "_down_conv_s2_compact",
                        lambda self, *a: (calls.append(1), orig(self, *a))[1])
    torch.manual_seed(8)
    blk = R.Bottleneck(1024, 512, stride=2, downsample=True).to(cuda, torch.bfloat16)
    blk = blk.to(memory_format=torch.channels_last).train()
    x0 = _nhwc(torch.randn(4, 1024, 14, 14, device=cuda).relu().bfloat16())
    gy = _nhwc(torch.randn(4, 2048, 7, 7, device=cuda).bfloat16())
    outs, grads = {}, {}
    for on in (True, False):
        with perf.use_policy(perf.policy().replace(down_s2_compact=on)):
            b = copy.deepcopy(blk)
            x = x0.clone().requires_grad_(True)
            y = b(x)
            y.backward(gy)
        outs[on] = y.detach()
        grads[on] = [x.grad] + [p.grad for p in b.parameters()]
    assert len(calls) == 1, "the compact downsample path did not run exactly once"
    assert _rel(outs[True].float(), outs[False].float()) < 2e-2
    for a, r in zip(grads[True], grads[False]):
        assert _rel(a.float(), r.float()) < 3e-2
