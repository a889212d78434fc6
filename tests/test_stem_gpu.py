"""ResNet stem on the HIP kernels of csrc/kernels/stem_conv.hip (MFMA conv with the BN statistics in
its epilogue; one-pass weight gradient through BN + ReLU + max-pool) vs an fp32 PyTorch reference,
with the library path (bf16 conv + fused BN-pool) as the yardstick for bf16 error."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from consensusml_amd.ops.bn import BatchNormAct2d
from consensusml_amd.ops.pool import bn_relu_max_pool2d
from consensusml_amd.ops.stem import pack_stem_weight, stem_conv_bn_relu_pool, stem_ok

pytestmark = pytest.mark.gpu


def _rel(p, q):
    return ((p.float() - q.float()).norm() / q.float().norm().clamp_min(1e-6)).item()


@pytest.mark.parametrize("N,C,H,W", [(4, 3, 64, 64), (3, 3, 50, 46), (2, 4, 40, 40),
                                     (600, 3, 16, 16)])
def test_stem_fused_vs_fp32(cuda, N, C, H, W):
    torch.manual_seed(N * 100 + H)
    x = torch.randn(N, C, H, W, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w0 = (torch.randn(64, C, 7, 7, device=cuda) * 0.1).to(torch.bfloat16)
    gam = torch.empty(64, device=cuda).uniform_(-0.5, 1.5)
    bet = torch.empty(64, device=cuda).uniform_(-0.5, 0.5)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    PH, PW = (OH - 1) // 2 + 1, (OW - 1) // 2 + 1
    dy = torch.randn(N, 64, PH, PW, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    res = []
    for fused in (True, False):
        conv = nn.Conv2d(C, 64, 7, 2, 3, bias=False).to(cuda, torch.bfloat16)
        bn = BatchNormAct2d(64, relu=True).to(cuda, torch.bfloat16)
        with torch.no_grad():
            conv.weight.copy_(w0)
            bn.weight.copy_(gam)
            bn.bias.copy_(bet)
        if fused:
            assert stem_ok(x, conv, bn)
            y = stem_conv_bn_relu_pool(x, conv, bn)
        else:
            y = bn_relu_max_pool2d(conv(x), bn)
        y.backward(dy)
        bn.eval()
        with torch.no_grad():
            ye = stem_conv_bn_relu_pool(x, conv, bn) if fused else bn_relu_max_pool2d(conv(x), bn)
        res.append([y, conv.weight.grad, bn.weight.grad, bn.bias.grad, bn.running_mean,
                    bn.running_var, ye])
    wr = w0.float().requires_grad_(True)
    gr, br = gam.clone().to(torch.bfloat16).float().requires_grad_(True), \
        bet.clone().to(torch.bfloat16).float().requires_grad_(True)
    rm, rv = torch.zeros(64, device=cuda), torch.ones(64, device=cuda)
    zr = F.conv2d(x.float(), wr, stride=2, padding=3)
    yr = F.max_pool2d(torch.relu(F.batch_norm(zr, rm, rv, gr, br, True, 0.1, 1e-5)), 3, 2, 1)
    yr.backward(dy.float())
    with torch.no_grad():
        yre = F.max_pool2d(torch.relu(F.batch_norm(F.conv2d(x.float(), w0.float(), stride=2,
                                                            padding=3),
                                                   rm, rv, gr, br, False, 0.1, 1e-5)), 3, 2, 1)
    ref = [yr, wr.grad, gr.grad, br.grad, rm, rv, yre]
    names = ["y", "dW", "dgamma", "dbeta", "running_mean", "running_var", "y_eval"]
    for name, f, u, r in zip(names, res[0], res[1], ref):
        ef, eu = _rel(f, r), _rel(u, r)
        # the floor covers ReLU-mask / argmax flips of near-tie windows (a few per channel at
        # these sizes); the kernels themselves are checked exactly in test_stem_kernels_exact
        assert ef <= max(2 * eu, 0.05), (name, ef, eu)


def test_stem_model_path_matches_unfused(cuda):
    """ResNet-50 forward/backward with the fused stem vs the library stem, both against the same
    model in fp32: the stem weight gradient sits under 50 bf16 layers, so the yardstick is the
    library path's own distance to fp32."""
    import copy

    import consensusml_amd.models.resnet as R
    torch.manual_seed(0)
    m32 = R.resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    m = copy.deepcopy(m32).to(torch.bfloat16)
    x = torch.randn(8, 3, 96, 96, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    loss32 = F.cross_entropy(m32(x.float()), y)
    loss32.backward()
    g32 = m32.conv1.weight.grad.float()
    out = {}
    for fused in (True, False):
        from consensusml_amd import perf
        with perf.use_policy(perf.policy().replace(fuse_stem_conv=fused)):
            m.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            out[fused] = (loss.item(), m.conv1.weight.grad.float().clone())
    assert abs(out[True][0] - loss32.item()) < 0.05 * max(1.0, abs(loss32.item()))
    ef, eu = _rel(out[True][1], g32), _rel(out[False][1], g32)
    assert ef <= max(1.5 * eu, 0.1), (ef, eu)


@pytest.mark.parametrize("N,C,H,W", [(4, 3, 64, 64), (3, 4, 50, 46)])
def test_stem_kernels_exact(cuda, N, C, H, W):
    """Each kernel against a float64 evaluation on ITS OWN inputs (no bf16 re-rounding noise)."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(1)
    x = torch.randn(N, C, H, W, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, C, 7, 7, device=cuda) * 0.1).to(torch.bfloat16)
    gam = torch.empty(64, device=cuda).uniform_(-0.5, 1.5).to(torch.bfloat16)
    bet = torch.empty(64, device=cuda).uniform_(-0.5, 0.5).to(torch.bfloat16)
    z, mean, invstd = lib().stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
    zr = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    assert _rel(z.double(), zr) < 4e-3                       # bf16 output rounding
    mr, vr = zr.mean((0, 2, 3)), zr.var((0, 2, 3), unbiased=False)
    assert (mean.double() - mr).abs().max().item() < 1e-5 * max(1.0, mr.abs().max().item())
    assert ((invstd.double() * (vr + 1e-5).sqrt()) - 1).abs().max().item() < 1e-5
    y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                             False, 3, 2, 1)
    dy = torch.randn_like(y)
    g, gsum = lib().maxpool_bwd_sum(dy, idx, z.shape[2], z.shape[3])
    sc = (invstd.double() * gam.double()).view(1, -1, 1, 1)
    u = (z.double() - mean.double().view(1, -1, 1, 1)) * sc + bet.double().view(1, -1, 1, 1)
    ud = u.requires_grad_(True)
    F.max_pool2d(torch.relu(ud), 3, 2, 1).backward(dy.double())
    assert _rel(g.double(), ud.grad) < 4e-3                  # bf16 output rounding
    # gsum adds the unrounded fp32 gradients: compare on the scale of sum |g|
    gabs = g.double().abs().sum((0, 2, 3)).clamp_min(1e-6)
    assert ((gsum.double() - g.double().sum((0, 2, 3))).abs() / gabs).max().item() < 2e-3
    dw, dg, db = lib().stem_wgrad(g, z, x, mean, invstd, gam, gsum)
    gd = g.double()
    xh = (z.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
    s1, s2 = gd.sum((0, 2, 3)), (gd * xh).sum((0, 2, 3))
    assert ((db.double() - s1).abs() / gabs).max().item() < 2e-3
    assert _rel(dg.double(), s2) < 1e-5
    M = gd.numel() / 64
    dz = (gam.double() * invstd.double()).view(1, -1, 1, 1) * (
        gd - s1.view(1, -1, 1, 1) / M - xh * (s2.view(1, -1, 1, 1) / M))
    wq = w.double().requires_grad_(True)
    F.conv2d(x.double(), wq, stride=2, padding=3).backward(dz)
    assert _rel(dw.double(), wq.grad) < 5e-3                 # g - mean(g) and xhat staged as bf16


def test_stem_pool_link_second_gradient(cuda):
    """layer1.0's downsample data gradient parked on the stem's pool link and summed inside the
    pool backward (kernel dy2) instead of by an autograd add of the two bf16 gradients: both
    paths measured against the same model in fp32 (the stem gradients sit under 50 bf16 layers,
    so the yardstick is the add path's own distance to fp32)."""
    import copy

    import consensusml_amd.models.resnet as R
    from consensusml_amd.ops.bn import TAP_STATS
    torch.manual_seed(0)
    m32 = R.resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    m = copy.deepcopy(m32).to(torch.bfloat16)
    x = torch.randn(8, 3, 96, 96, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    F.cross_entropy(m32(x.float()), y).backward()
    ref = [m32.conv1.weight.grad, m32.bn1.weight.grad, m32.bn1.bias.grad]
    out = {}
    for on in (True, False):
        from consensusml_amd import perf
        TAP_STATS.update(parked=0, fallback=0)
        # c1_dgrad64_gemm off: layer1.0's conv1 data gradient on the library conv, so the
        # downsample's dX takes the pool link (with it on, conv1's GEMM absorbs it instead)
        with perf.use_policy(perf.policy().replace(pool_link=on, c1_dgrad64_gemm=False)):
            m.zero_grad(set_to_none=True)
            F.cross_entropy(m(x).float(), y).backward()
            out[on] = [m.conv1.weight.grad.float().clone(), m.bn1.weight.grad.float().clone(),
                       m.bn1.bias.grad.float().clone()]
            stats = dict(TAP_STATS)
        assert stats["fallback"] == 0
        if on:
            assert stats["parked"] >= 1
    for a, b, r in zip(out[True], out[False], ref):
        e_on, e_off = _rel(a, r), _rel(b, r)
        print(f"rel err vs fp32: link {e_on:.4f}, add {e_off:.4f}, link vs add {_rel(a, b):.4f}")
        assert e_on <= max(1.5 * e_off, 0.1), (e_on, e_off)


@pytest.mark.parametrize("N,C,H,W,two", [(4, 3, 64, 64, False), (3, 4, 50, 46, True),
                                         (2, 3, 224, 224, False), (2, 3, 224, 224, True),
                                         (5, 3, 30, 62, False), (1100, 3, 16, 16, True),
                                         (1030, 4, 18, 14, False)])
def test_stem_wgrad_pool_gather(cuda, N, C, H, W, two):
    """stem_wgrad_pool (the pool's input gradient gathered from the pooled gradient inside the
    weight-gradient kernel, after a routed channel-sum pass) vs the two-pass path (maxpool_bwd_sum
    writes the full-resolution gradient, stem_wgrad reads it) and vs float64. 224 x 224 runs the
    fixed-width (OW = 112) instance of the bench; (5, 3, 30, 62) has partial bands and chunks;
    N > 1024 runs the input column sums (stem_cola) over > 8 chunk partials (the unrolled batch
    plus the remainder)."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(N + H + int(two))
    x = torch.randn(N, C, H, W, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, C, 7, 7, device=cuda) * 0.1).to(torch.bfloat16)
    gam = torch.empty(64, device=cuda).uniform_(-0.5, 1.5).to(torch.bfloat16)
    bet = torch.empty(64, device=cuda).uniform_(-0.5, 0.5).to(torch.bfloat16)
    z, mean, invstd = lib().stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
    y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                             False, 3, 2, 1)
    assert (idx == 255).any()                                 # some ReLU-masked windows
    dy = torch.randn_like(y)
    dy2 = torch.randn_like(y) if two else None
    dw, dg, db = lib().stem_wgrad_pool(dy, idx, dy2, z, x, mean, invstd, gam)
    # bf16 outputs from the final kernel == the fp32 ones cast (the parameters' dtype)
    for a, b in zip(lib().stem_wgrad_pool(dy, idx, dy2, z, x, mean, invstd, gam, True),
                    (dw, dg, db)):
        assert a.dtype == torch.bfloat16 and torch.equal(a, b.to(torch.bfloat16))
    g, gsum = lib().maxpool_bwd_sum(dy, idx, z.shape[2], z.shape[3], dy2)
    dw2, dg2, db2 = lib().stem_wgrad(g, z, x, mean, invstd, gam, gsum)
    gabs = g.double().abs().sum((0, 2, 3)).clamp_min(1e-6)
    assert ((db.double() - db2.double()).abs() / gabs).max().item() < 1e-3
    assert _rel(dg, dg2) < 2e-3
    # float64 on the pool gradient the kernels route (dy + dy2 rounded to bf16 when two)
    dyt = (dy.float() + dy2.float()).to(torch.bfloat16) if two else dy
    sc = (invstd.double() * gam.double()).view(1, -1, 1, 1)
    u = ((z.double() - mean.double().view(1, -1, 1, 1)) * sc +
         bet.double().view(1, -1, 1, 1)).requires_grad_(True)
    F.max_pool2d(torch.relu(u), 3, 2, 1).backward(dyt.double())
    gd = u.grad
    xh = (z.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
    s1, s2 = gd.sum((0, 2, 3)), (gd * xh).sum((0, 2, 3))
    assert ((db.double() - s1).abs() / gabs).max().item() < 2e-3
    assert _rel(dg.double(), s2) < 1e-4
    M = gd.numel() / 64
    dz = sc * (gd - s1.view(1, -1, 1, 1) / M - xh * (s2.view(1, -1, 1, 1) / M))
    wq = w.double().requires_grad_(True)
    F.conv2d(x.double(), wq, stride=2, padding=3).backward(dz)
    # g - mean(g) and xhat are staged as bf16 on both paths (the two-pass path rounds g first):
    # each is ~2-4e-3 from float64 and they differ from each other by as much
    e_gather, e_two = _rel(dw.double(), wq.grad), _rel(dw2.double(), wq.grad)
    assert e_gather < 5e-3, (e_gather, e_two)
    assert e_gather <= 1.25 * e_two + 5e-4, (e_gather, e_two)


@pytest.mark.parametrize("N,two", [(3, False), (40, True)])
def test_stem_wgrad_pc_matches_alternating(cuda, monkeypatch, N, two):
    """stem_wgrad_pc_kernel (fixed producer / consumer waves, the 224 x 224 bench shape) vs the
    alternating kernel (CML_STEM_PC=0) on the same inputs. The products are summed in the same
    order; only the BN sums (s1, s2) take a different per-thread pixel order. N = 40: 280 bands
    over the persistent grid, so workgroups cross band changes (input tile restaged mid-loop)."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(N)
    x = torch.randn(N, 3, 224, 224, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device=cuda) * 0.1).to(torch.bfloat16)
    gam = torch.empty(64, device=cuda).uniform_(-0.5, 1.5).to(torch.bfloat16)
    bet = torch.empty(64, device=cuda).uniform_(-0.5, 0.5).to(torch.bfloat16)
    z, mean, invstd = lib().stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
    y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                             False, 3, 2, 1)
    dy = torch.randn_like(y)
    dy2 = torch.randn_like(y) if two else None
    out = {}
    for pc in ("1", "0"):
        monkeypatch.setenv("CML_STEM_PC", pc)
        out[pc] = lib().stem_wgrad_pool(dy, idx, dy2, z, x, mean, invstd, gam)
    for a, b in zip(out["1"], out["0"]):
        assert torch.isfinite(a).all()
        assert _rel(a, b) < 2e-5, _rel(a, b)


def test_layer1_conv1_dgrad_gemm_absorbs_downsample(cuda):
    """PerfPolicy.c1_dgrad64_gemm: layer1.0's conv1 data gradient as a GEMM whose beta = 1
    epilogue takes the downsample's dX (no pool two-gradient sum) vs the library data gradient +
    the pool link: the stem gradients of both paths against the same model in fp32."""
    import copy

    import consensusml_amd.models.resnet as R
    from consensusml_amd import perf
    torch.manual_seed(1)
    m32 = R.resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    m = copy.deepcopy(m32).to(torch.bfloat16)
    x = torch.randn(8, 3, 96, 96, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=cuda)
    F.cross_entropy(m32(x.float()), y).backward()
    ref = [m32.conv1.weight.grad, m32.layer1[0].conv1.weight.grad]
    out = {}
    for on in (True, False):
        with perf.use_policy(perf.policy().replace(c1_dgrad64_gemm=on)):
            m.zero_grad(set_to_none=True)
            F.cross_entropy(m(x).float(), y).backward()
            out[on] = [m.conv1.weight.grad.float().clone(),
                       m.layer1[0].conv1.weight.grad.float().clone()]
    for a, b, r in zip(out[True], out[False], ref):
        e_on, e_off = _rel(a, r), _rel(b, r)
        assert e_on <= max(1.5 * e_off, 0.1), (e_on, e_off)
