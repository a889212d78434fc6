"""Fused NHWC BatchNorm(+residual)(+ReLU) HIP kernels vs an fp32 PyTorch reference."""
import copy

import pytest
import torch
import torch.nn.functional as F

from consensusml_amd.ops.bn import BatchNormAct2d, bn_act

pytestmark = pytest.mark.gpu


def _ref(x, g, b, res, relu, rm, rv):
    y = F.batch_norm(x.float(), rm, rv, g.float(), b.float(), True, 0.1, 1e-5)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


@pytest.mark.parametrize("C", [8, 64, 256, 2048])
@pytest.mark.parametrize("mode", ["relu", "res_relu", "plain", "res"])
def test_bn_act_fwd_bwd(cuda, C, mode):
    torch.manual_seed(C)
    N, H, W = 4, 9, 7
    relu = "relu" in mode
    use_res = "res" in mode
    x = (torch.randn(N, C, H, W, device=cuda) * 3 + 1.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    res = None
    if use_res:
        res = torch.randn(N, C, H, W, device=cuda).to(torch.bfloat16)
        res = res.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    g = (torch.rand(C, device=cuda) + 0.5).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(C, device=cuda).to(torch.bfloat16).requires_grad_(True)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y = bn_act(x, g, b, rm, rv, res, relu, True)
    dy = torch.randn_like(y)
    y.backward(dy)
    # reference in fp32 on the same bf16 inputs
    xr = x.detach().float().requires_grad_(True)
    gr = g.detach().float().requires_grad_(True)
    br = b.detach().float().requires_grad_(True)
    resr = res.detach().float().requires_grad_(True) if use_res else None
    rm2, rv2 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    yr = _ref(xr, gr, br, resr, relu, rm2, rv2)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(g.grad.float(), gr.grad, rtol=3e-2, atol=0.5)
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=3e-2, atol=0.5)
    if use_res:
        torch.testing.assert_close(res.grad.float(), resr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rv, rv2, rtol=1e-3, atol=1e-3)


def test_bn_large_mean_small_var(cuda):
    """Shifted sums keep the variance accurate when |mean| >> std."""
    C = 64
    x = (torch.randn(2, C, 32, 32, device=cuda) * 0.05 + 40.0).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    m = BatchNormAct2d(C, relu=False).to(cuda).to(torch.bfloat16)
    y = m(x)
    yr = F.batch_norm(x.float(), None, None, None, None, True, 0.1, 1e-5)
    torch.testing.assert_close(y.float(), yr, rtol=5e-2, atol=6e-2)


def test_bn_eval_mode(cuda):
    C = 128
    m = BatchNormAct2d(C).to(cuda).to(torch.bfloat16)
    x = torch.randn(3, C, 5, 5, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    for _ in range(3):
        m(x)
    m.eval()
    y = m(x)
    yr = F.relu(F.batch_norm(x.float(), m.running_mean, m.running_var, m.weight.float(),
                             m.bias.float(), False, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    assert m.running_mean.dtype == torch.float32


def test_resnet_tiny_fused_vs_reference(cuda):
    """Whole tiny ResNet: fused kernels (bf16 NHWC) vs the same weights through PyTorch fp32."""
    from consensusml_amd.models.resnet import resnet_tiny
    torch.manual_seed(0)
    m = resnet_tiny(10).to(cuda)
    for mod in m.modules():
        if isinstance(mod, BatchNormAct2d):
            mod.weight.data.uniform_(0.5, 1.5)
    ref = resnet_tiny(10).to(cuda)
    ref.load_state_dict(m.state_dict())
    mb = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 32, 32, device=cuda)
    out = mb(x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)).float()
    out_ref = ref(x)   # fp32 NCHW -> composition path
    torch.testing.assert_close(out, out_ref, rtol=0.1, atol=0.15)


@pytest.mark.parametrize("shape,ksp", [((2, 64, 112, 112), (3, 2, 1)), ((3, 16, 9, 7), (3, 2, 1)),
                                       ((2, 16, 10, 9), (2, 2, 0)), ((2, 8, 9, 11), (3, 1, 1)),
                                       ((2, 8, 13, 12), (5, 2, 2))])
def test_maxpool_nhwc(cuda, shape, ksp):
    from consensusml_amd.ops.pool import max_pool2d
    k, s, p = ksp
    torch.manual_seed(1)
    x = torch.randn(*shape, device=cuda).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    y = max_pool2d(x, k, s, p)
    xr = x.detach().float().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr)
    dy = torch.randn_like(yr)
    y.backward(dy.to(torch.bfloat16))
    yr.backward(dy.to(torch.bfloat16).float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("mode", ["auto", "gemm", "miopen"])
@pytest.mark.parametrize("cin,cout", [(64, 256), (256, 64), (24, 40), (1024, 256)])
def test_conv1x1_gemm_matches_conv(cuda, cin, cout, mode):
    from consensusml_amd.models import resnet as R
    torch.manual_seed(0)
    m = R.Conv1x1(cin, cout).to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, 9, 7, device=cuda, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_(True)
    from consensusml_amd import perf
    with perf.use_policy(perf.policy().replace(conv1x1_gemm=mode)):
        y = m(x)
    assert y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    wr = m.weight.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr)
    yr.backward(g.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, rtol=2e-2, atol=1e-1)


@pytest.mark.parametrize("gemm", [False, True, "auto"])
def test_residual_link_matches_autograd_add(cuda, gemm):
    """Downsample block + 3 identity blocks: with the residual gradient parked on the producer's
    link (consumed as dy2 by the producer's BN backward, or by conv1's GEMM epilogue) and the
    ReLU bit mask, grads equal the plain autograd path (separate add, no links)."""
    from consensusml_amd.models import resnet as R
    torch.manual_seed(0)
    net = torch.nn.Sequential(R.Bottleneck(32, 16, downsample=True), R.Bottleneck(64, 16),
                              R.Bottleneck(64, 16), R.Bottleneck(64, 16))
    net = net.to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    for m in net:
        torch.nn.init.normal_(m.bn3.weight, 1.0, 0.1)
    x0 = torch.randn(4, 32, 10, 10, device=cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    res = []
    from consensusml_amd import perf
    from consensusml_amd.ops.bn import TAP_STATS
    TAP_STATS.update(parked=0, fallback=0)
    mode = {False: "miopen", True: "gemm"}.get(gemm, gemm)
    for link in (True, False):
        with perf.use_policy(perf.policy().replace(conv1x1_gemm=mode, residual_link=link)):
            net.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            y = net(x)
            y.float().square().sum().backward()
            res.append((x.grad.clone(), [p.grad.clone() for p in net.parameters()]))
    # the downsample branch's backward runs before conv1's: the tap always parks
    assert TAP_STATS["fallback"] == 0
    assert TAP_STATS["parked"] == (0 if gemm is False else 1)
    # fp32 reference: same weights, composition path (no fused kernels, no links)
    ref = copy.deepcopy(net).float().to(memory_format=torch.contiguous_format)
    xr = x0.float().contiguous().requires_grad_(True)
    ref(xr).square().sum().backward()
    refs = [xr.grad] + [p.grad for p in ref.parameters()]

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()
    for i, (a, b, r) in enumerate(zip([res[0][0]] + res[0][1], [res[1][0]] + res[1][1], refs)):
        # the linked path must be as close to fp32 as the plain bf16 path (both bf16 noise)
        e_link, e_plain = rel(a, r), rel(b, r)
        assert e_link <= max(2 * e_plain, 0.03), (i, e_link, e_plain)
        assert rel(a, b) <= max(2 * e_plain, 0.03), (i, rel(a, b), e_plain)


@pytest.mark.parametrize("mode", ["relu", "res_relu"])
def test_bn_act_two_part_output_grad(cuda, mode):
    """out_link: a gradient parked on the link is summed with dy inside the BN backward."""
    from consensusml_amd.ops.bn import ResidualLink
    torch.manual_seed(3)
    C = 64
    x = (torch.randn(4, C, 6, 5, device=cuda) * 2).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    res = None
    if mode == "res_relu":
        res = torch.randn(4, C, 6, 5, device=cuda).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
    g = (torch.rand(C, device=cuda) + 0.5).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(C, device=cuda).to(torch.bfloat16).requires_grad_(True)
    link = ResidualLink()
    y = bn_act(x, g, b, torch.zeros(C, device=cuda), torch.ones(C, device=cuda), res, True, True,
               out_link=link)
    dy = torch.randn_like(y)
    extra = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
    link.grad = extra
    y.backward(dy)
    assert link.grad is None
    x2 = x.detach().clone().requires_grad_(True)
    r2 = res.detach().clone().requires_grad_(True) if res is not None else None
    y2 = bn_act(x2, g.detach(), b.detach(), torch.zeros(C, device=cuda), torch.ones(C, device=cuda),
                r2, True, True)
    y2.backward((dy.float() + extra.float()).to(torch.bfloat16))
    torch.testing.assert_close(x.grad.float(), x2.grad.float(), rtol=2e-2, atol=3e-2)
    if res is not None:
        torch.testing.assert_close(res.grad.float(), r2.grad.float(), rtol=2e-2, atol=3e-2)


def test_stem_pad4_matches_conv(cuda):
    """3 -> 4 channel zero-padded stem (HIP pad kernel + padded weight view) == the plain conv."""
    from consensusml_amd.models import resnet as R
    torch.manual_seed(5)
    m = R.resnet_tiny().to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(3, 3, 33, 31, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    from consensusml_amd import perf
    for pad in (True, False):
        with perf.use_policy(perf.policy().replace(stem_pad4=pad)):
            m.zero_grad(set_to_none=True)
            y = m.stem(x)
            y.float().square().sum().backward()
            outs.append((y.float(), m.conv1.weight.grad.float().clone()))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=2e-2, atol=0.5)
    assert m.conv1.weight.grad.shape == (8, 3, 7, 7)


@pytest.mark.parametrize("C", [64, 256, 2048])
@pytest.mark.parametrize("with_dy2", [False, True])
def test_bn_add_bn_relu_matches_composition(cuda, C, with_dy2):
    """Fused relu(bn3(x1) + bn_d(x2)) (one apply, one dual reduce, one dual apply) vs the two
    separate fused BN ops + residual add, both against an fp32 reference of the same math on the
    same bf16 inputs: the fused path must be at least as accurate (it adds the shortcut BN output
    in fp32 instead of rounding it to bf16 first). Running stats and eval mode included."""
    from consensusml_amd.ops.bn import BatchNormAct2d, ResidualLink, bn_add_bn_relu
    torch.manual_seed(C)
    shp = (4, C, 6, 5)
    mk = lambda s, o: ((torch.randn(*shp, device=cuda) * s + o).to(torch.bfloat16)
                       .contiguous(memory_format=torch.channels_last))
    x1, x2 = mk(2.0, 0.5), mk(1.5, -0.3)
    dy = torch.randn(*shp, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy2 = torch.randn(*shp, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.empty(4, C, device=cuda).uniform_(0.5, 1.5)
    bb = torch.empty(4, C, device=cuda).uniform_(-0.5, 0.5)
    res = []
    for fused in (True, False):
        bn1 = BatchNormAct2d(C, relu=True).to(cuda, torch.bfloat16)
        bn2 = BatchNormAct2d(C, relu=False).to(cuda, torch.bfloat16)
        with torch.no_grad():
            bn1.weight.copy_(g[0]); bn1.bias.copy_(bb[0]); bn2.weight.copy_(g[1]); bn2.bias.copy_(bb[1])
        a, c = x1.clone().requires_grad_(True), x2.clone().requires_grad_(True)
        link = ResidualLink() if with_dy2 else None
        y = bn_add_bn_relu(a, bn1, c, bn2, link) if fused else bn1(a, residual=bn2(c), out_link=link)
        if with_dy2:
            link.grad = dy2.clone()
        y.backward(dy)
        bn1.eval()
        bn2.eval()
        ye = bn_add_bn_relu(x1, bn1, x2, bn2) if fused else bn1(x1, residual=bn2(x2))
        res.append([y, a.grad, c.grad, bn1.weight.grad, bn1.bias.grad, bn2.weight.grad,
                    bn2.bias.grad, bn1.running_mean, bn1.running_var, bn2.running_mean,
                    bn2.running_var, ye])
    # fp32 reference
    a, c = x1.float().requires_grad_(True), x2.float().requires_grad_(True)
    ps = [t.clone().requires_grad_(True) for t in (g[0], bb[0], g[1], bb[1])]
    rms = [torch.zeros(C, device=cuda), torch.ones(C, device=cuda), torch.zeros(C, device=cuda),
           torch.ones(C, device=cuda)]
    yr = torch.relu(F.batch_norm(a, rms[0], rms[1], ps[0], ps[1], True, 0.1, 1e-5)
                    + F.batch_norm(c, rms[2], rms[3], ps[2], ps[3], True, 0.1, 1e-5))
    yr.backward(dy.float() + (dy2.float() if with_dy2 else 0))
    yre = torch.relu(F.batch_norm(x1.float(), rms[0], rms[1], ps[0], ps[1], False, 0.1, 1e-5)
                     + F.batch_norm(x2.float(), rms[2], rms[3], ps[2], ps[3], False, 0.1, 1e-5))
    ref = [yr, a.grad, c.grad, ps[0].grad, ps[1].grad, ps[2].grad, ps[3].grad] + rms + [yre]

    def rel(p, q):
        p, q = p.float(), q.float()
        return ((p - q).norm() / q.norm().clamp_min(1e-6)).item()
    for i, (f, u, r) in enumerate(zip(res[0], res[1], ref)):
        ef, eu = rel(f, r), rel(u, r)
        assert ef <= max(2 * eu, 0.05), (i, ef, eu)   # bf16 noise: ~2-4 % on both paths


def test_stem_bn_relu_maxpool_fused(cuda):
    """maxpool(relu(bn(x))) fused (BN output never stored) vs BN then pool, against fp32."""
    from consensusml_amd.ops.bn import BatchNormAct2d
    from consensusml_amd.ops.pool import bn_relu_max_pool2d, max_pool2d
    torch.manual_seed(9)
    C = 64
    x0 = (torch.randn(4, C, 17, 15, device=cuda) * 2 + 0.3).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dyp = torch.randn(4, C, 9, 8, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.empty(C, device=cuda).uniform_(-1.0, 1.5)     # some negative gammas: affine flips
    b = torch.empty(C, device=cuda).uniform_(-0.5, 0.5)
    res = []
    for fused in (True, False):
        bn = BatchNormAct2d(C, relu=True).to(cuda, torch.bfloat16)
        with torch.no_grad():
            bn.weight.copy_(g)
            bn.bias.copy_(b)
        x = x0.clone().requires_grad_(True)
        y = bn_relu_max_pool2d(x, bn) if fused else max_pool2d(bn(x))
        y.backward(dyp)
        bn.eval()
        ye = bn_relu_max_pool2d(x0, bn) if fused else max_pool2d(bn(x0))
        res.append([y, x.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var, ye])
    xr = x0.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    yr = F.max_pool2d(torch.relu(F.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)), 3, 2, 1)
    yr.backward(dyp.float())
    yre = F.max_pool2d(torch.relu(F.batch_norm(x0.float(), rm, rv, gr, br, False, 0.1, 1e-5)), 3, 2, 1)
    ref = [yr, xr.grad, gr.grad, br.grad, rm, rv, yre]

    def rel(p, q):
        return ((p.float() - q.float()).norm() / q.float().norm().clamp_min(1e-6)).item()
    for i, (f, u, r) in enumerate(zip(res[0], res[1], ref)):
        ef, eu = rel(f, r), rel(u, r)
        assert ef <= max(2 * eu, 0.03), (i, ef, eu)


@pytest.mark.parametrize("N,H,W", [(3, 23, 30), (5, 112, 112), (1, 9, 9), (9, 56, 40)])
def test_stem_maxpool_band_mapping(cuda, N, H, W):
    """The stem's fused BN + ReLU + 3x3 / s2 max-pool forward (2 x 2 outputs per thread, a band of
    two output rows per workgroup; odd output heights / widths, band counts that do not divide by
    8) vs fp32 PyTorch on the same affine: every output row written."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(N + H)
    C = 64
    z = (torch.randn(N, C, H, W, device=cuda) + 0.2).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    gam = torch.empty(C, device=cuda).uniform_(-1.0, 1.5).to(torch.bfloat16)
    bet = torch.empty(C, device=cuda).uniform_(-0.5, 0.5).to(torch.bfloat16)
    mean = torch.randn(C, device=cuda) * 0.1
    invstd = torch.rand(C, device=cuda) + 0.5
    y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1,
                                             False, 3, 2, 1)
    sc = invstd * gam.float()
    bi = bet.float() - mean * sc
    u = z.float() * sc.view(1, -1, 1, 1) + bi.view(1, -1, 1, 1)
    ref = F.max_pool2d(torch.relu(u), 3, 2, 1)
    assert y.shape == ref.shape
    err = (y.float() - ref).abs()
    assert float(err.max()) <= 1e-2 * float(ref.abs().max()) + 1e-3
    # ReLU-masked windows (argmax 255) where the reference max is <= 0 (layout-free count; an
    # affine output within rounding of 0 may land either side)
    assert abs(int((idx == 255).sum()) - int((ref <= 0).sum())) <= max(2, ref.numel() // 10000)
