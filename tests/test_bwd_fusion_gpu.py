"""Backward fusion of the identity-block tail (ops.conv.bnrelu_conv1x1_bn_res): the BN-backward
prologue of the 1x1 data-gradient kernel, the masked-link epilogue (+ BN-backward sums), the
coefficient kernel and the weight-gradient dz prologue, each against an fp32 PyTorch oracle; and
whole blocks with the fusion on vs off."""
import copy

import pytest
import torch

from consensusml_amd import perf

pytestmark = pytest.mark.gpu


def _lib():
    from consensusml_amd.ops.native import lib
    return lib()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _bits(mask, C):
    sh = torch.arange(8, device=mask.device, dtype=torch.uint8)
    return ((mask.view(-1, C // 8, 1) >> sh) & 1).view(-1, C).float()


def _rows(t):
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).float()


def _rand_mask(M, C, dev, gen):
    return torch.randint(0, 256, (M, C // 8), generator=gen, device=dev, dtype=torch.uint8)


def _close(a, b, tol):
    err = (a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)
    assert err < tol, f"relative error {err:.3e} >= {tol}"


@pytest.mark.parametrize("N,K,No,H", [(2, 256, 64, 28), (3, 512, 128, 14), (2, 1024, 256, 7),
                                      (1, 2048, 512, 7)])
def test_conv1x1_bnbwd(cuda, N, K, No, H):
    g0 = torch.Generator(device=cuda).manual_seed(0)
    g = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    z = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    mask = _rand_mask(M, K, cuda, g0)
    ca, cb, cc = (torch.randn(K, device=cuda, generator=g0) for _ in range(3))
    w = (torch.randn(No, K, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    y = _lib().conv1x1_bnbwd(g, z, mask, ca, cb, cc, w)
    dz = (ca * (_bits(mask, K) * _rows(g)) + cb * _rows(z) + cc).bfloat16().float()
    ref = dz @ w.float().t()
    _close(_rows(y), ref, 1e-2)


@pytest.mark.parametrize("sums", [False, True])
@pytest.mark.parametrize("N,K,No,H", [(2, 64, 256, 28), (2, 128, 512, 14), (3, 256, 1024, 7),
                                      (2, 512, 2048, 7), (1, 128, 512, 2)])
def test_conv1x1_link(cuda, sums, N, K, No, H):
    g0 = torch.Generator(device=cuda).manual_seed(1)
    x = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(No, K, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    link = _nhwc(torch.randn(N, No, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    lm = _rand_mask(M, No, cuda, g0)
    ref = (_rows(x) @ w.float().t()).bfloat16().float() + _bits(lm, No) * _rows(link)
    if not sums:
        y, _, _ = _lib().conv1x1_link(x, w, link, lm)
        _close(_rows(y), ref, 1e-2)
        return
    sz = _nhwc(torch.randn(N, No, H, H, device=cuda, generator=g0).bfloat16())
    sm = _rand_mask(M, No, cuda, g0)
    mean = torch.randn(No, device=cuda, generator=g0) * 0.1
    invstd = torch.rand(No, device=cuda, generator=g0) + 0.5
    y, sdz, sdzx = _lib().conv1x1_link(x, w, link, lm, sz, sm, mean, invstd)
    _close(_rows(y), ref, 1e-2)
    yv = _rows(y) * _bits(sm, No)
    torch.testing.assert_close(sdz, yv.sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    q = (yv * (_rows(sz) - mean) * invstd).sum(0)
    torch.testing.assert_close(sdzx, q, rtol=1e-3, atol=1e-2 * M ** 0.5)


def test_coeffs_reproduce_bn_backward(cuda):
    """a (m ? g : 0) + b z + c from bn_bwd_sums / bn_bwd_coeffs == the BN backward's dx."""
    g0 = torch.Generator(device=cuda).manual_seed(2)
    N, C, H = 4, 256, 14
    z = _nhwc((torch.randn(N, C, H, H, device=cuda, generator=g0) * 2 + 0.5).bfloat16())
    res = _nhwc(torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16())
    gamma = (torch.rand(C, device=cuda, generator=g0) + 0.5).bfloat16()
    beta = (torch.randn(C, device=cuda, generator=g0) * 0.1).bfloat16()
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, mean, invstd, mask = _lib().bn_fwd(z, res, gamma, beta, rm, rv, None, None, 1e-5, 0.1,
                                          True, True, True)
    gy = _nhwc(torch.randn(N, C, H, H, device=cuda, generator=g0).bfloat16())
    dx, dg, db, dres = _lib().bn_bwd(gy, None, z, mask, gamma, beta, mean, invstd, True, True)
    sdz, sdzx = _lib().bn_bwd_sums(gy, None, z, mask, gamma, beta, mean, invstd, True)
    M = N * H * H
    ca, cb, cc, dg2, db2 = _lib().bn_bwd_coeffs(sdz, sdzx, gamma, mean, invstd, M)
    dz = ca * (_bits(mask, C) * _rows(gy)) + cb * _rows(z) + cc
    _close(dz, _rows(dx), 2e-2)
    torch.testing.assert_close(dg2.float(), dg.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(db2.float(), db.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(_bits(mask, C) * _rows(gy), _rows(dres))


@pytest.mark.parametrize("Co,Ci,H", [(256, 64, 28), (512, 128, 14), (1024, 256, 14),
                                     (2048, 512, 7)])
def test_wgrad_dz_prologue(cuda, Co, Ci, H):
    g0 = torch.Generator(device=cuda).manual_seed(3)
    N = 4
    gy = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    z3 = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    z2 = _nhwc(torch.randn(N, Ci, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    mask = _rand_mask(M, Co, cuda, g0)
    ca, cb, cc = (torch.randn(Co, device=cuda, generator=g0) for _ in range(3))
    sc = torch.rand(Ci, device=cuda, generator=g0) + 0.5
    bi = torch.randn(Ci, device=cuda, generator=g0) * 0.1
    dw = _lib().wgrad1x1(gy, z2, torch.float32, sc, bi, z3, mask, ca, cb, cc)
    dz = (ca * (_bits(mask, Co) * _rows(gy)) + cb * _rows(z3) + cc).bfloat16().float()
    x = torch.relu(_rows(z2) * sc + bi).bfloat16().float()
    ref = dz.t() @ x
    _close(dw.view(Co, Ci), ref, 1e-2)


def _chain(cuda, planes, blocks, seed=0):
    from consensusml_amd.models.resnet import Bottleneck
    torch.manual_seed(seed)
    m = torch.nn.Sequential(*[Bottleneck(planes * 4, planes) for _ in range(blocks)])
    for mod in m.modules():
        if hasattr(mod, "bias") and isinstance(mod.bias, torch.nn.Parameter) \
                and mod.__class__.__name__ == "BatchNormAct2d":
            with torch.no_grad():
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.1, 0.1)
    return m.to(device=cuda, dtype=torch.bfloat16, memory_format=torch.channels_last).train()


def _err(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("planes,H", [(64, 28), (256, 14), (512, 7)])
def test_identity_chain_fused_vs_unfused(cuda, planes, H):
    """Three identity blocks (links between them: phase-2 sums in the conv1 epilogue). Both bf16
    backwards -- fusion on and off -- are compared with an fp32 run of the same weights: the fused
    one must be as accurate as the unfused one (BN backward amplifies bf16 rounding, so the
    absolute error level depends on the shape)."""
    m_on = _chain(cuda, planes, 3)
    m_off = copy.deepcopy(m_on)
    m32 = copy.deepcopy(m_on).float()
    g0 = torch.Generator(device=cuda).manual_seed(5)
    x = _nhwc(torch.randn(8, planes * 4, H, H, device=cuda, generator=g0).bfloat16())
    gy = _nhwc(torch.randn(8, planes * 4, H, H, device=cuda, generator=g0).bfloat16())
    outs = {}
    for key, m, dt in (("on", m_on, torch.bfloat16), ("off", m_off, torch.bfloat16),
                       ("fp32", m32, torch.float32)):
        with perf.use_policy(perf.policy().replace(fused_bn3_bwd=key == "on",
                                                   fused_bn3_bwd_max_planes=4096)):
            xi = x.to(dt).clone().requires_grad_(True)
            y = m(xi)
            y.backward(gy.to(dt))
        outs[key] = (y.detach().float(), xi.grad.float(), [p.grad.float() for p in m.parameters()])
    ref = outs["fp32"]
    for k in (0, 1):
        e_on, e_off = _err(outs["on"][k], ref[k]), _err(outs["off"][k], ref[k])
        assert e_on <= 1.5 * e_off + 1e-2, (k, e_on, e_off)
    for a, b, r in zip(outs["on"][2], outs["off"][2], ref[2]):
        e_on, e_off = _err(a, r), _err(b, r)
        assert e_on <= 1.5 * e_off + 2e-2, (e_on, e_off)


# ---- recompute tail (ops.conv._RecomputeTailFn): kernels and the whole chain ----

# (1, 128, 3): M = 9 pixels, so whole wave blocks of the tile start past M (their epilogue operand
# loads must stay inside the tensors)
@pytest.mark.parametrize("N,K,H", [(2, 64, 28), (3, 128, 14), (2, 128, 9), (1, 128, 3)])
def test_stats_only_and_bnres_match_stored_path(cuda, N, K, H):
    """The statistics-only pass gives conv1x1_bn_fwd's statistics bit for bit, and the recompute
    apply gives bn_fwd(z3, res)'s output and mask (same bf16 z3, same plan)."""
    g0 = torch.Generator(device=cuda).manual_seed(21)
    Co = 4 * K
    z = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, K, 1, 1, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    sc = torch.rand(K, device=cuda, generator=g0) + 0.5
    bi = torch.randn(K, device=cuda, generator=g0) * 0.1
    res = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    rm = torch.randn(Co, device=cuda, generator=g0) * 0.1
    z3, m_ref, i_ref = _lib().conv1x1_bn_fwd(z, w, sc, bi, rm.clone(), None, None, 1, True, 1e-5,
                                             0.1)
    m, i = _lib().conv1x1_bn_stats_only(z, w, sc, bi, rm.clone(), None, None, 1e-5, 0.1)
    assert torch.equal(m, m_ref) and torch.equal(i, i_ref)
    g3 = (torch.rand(Co, device=cuda, generator=g0) + 0.5).bfloat16()
    b3 = (torch.randn(Co, device=cuda, generator=g0) * 0.1).bfloat16()
    sc3 = g3.float() * i
    bi3 = b3.float() - m * sc3
    y, mask = _lib().conv1x1_bnres(z, w, sc, bi, sc3, bi3, res)
    t = _rows(z3) * sc3 + bi3 + _rows(res)
    _close(_rows(y), torch.relu(t), 1e-2)
    agree = (_bits(mask, Co) == (t > 0).float()).float().mean().item()
    assert agree > 0.999, agree


@pytest.mark.parametrize("id2", [False, True])
@pytest.mark.parametrize("N,K1,K2,No,H", [(2, 256, 64, 64, 28), (3, 512, 128, 128, 14),
                                          (2, 512, 128, 128, 9)])
def test_conv1x1_cat(cuda, id2, N, K1, K2, No, H):
    """[a (mask ? g : 0) + c | f2(x2)] w^T with a, c folded into the weights and a bias
    (ops.conv.fold_cat); f2 = relu(x2 sc + bi), or x2 as is (id2, x2 a ReLU output)."""
    from consensusml_amd.ops.conv import fold_cat
    g0 = torch.Generator(device=cuda).manual_seed(22)
    g = _nhwc(torch.randn(N, K1, H, H, device=cuda, generator=g0).bfloat16())
    x2 = _nhwc(torch.randn(N, K2, H, H, device=cuda, generator=g0).bfloat16())
    if id2:
        x2 = torch.relu(x2)
    M = N * H * H
    mask = _rand_mask(M, K1, cuda, g0)
    a = torch.randn(K1, device=cuda, generator=g0)
    c = torch.randn(K1, device=cuda, generator=g0) * 0.1
    sc = torch.rand(K2, device=cuda, generator=g0) + 0.5
    bi = torch.randn(K2, device=cuda, generator=g0) * 0.1
    w = torch.randn(No, K1 + K2, device=cuda, generator=g0) * (K1 + K2) ** -0.5
    w_cat, bias = fold_cat(w[:, :K1], a, c, w[:, K1:])
    if id2:
        y = _lib().conv1x1_cat(g, mask, x2, None, None, w_cat, bias)
        v = _rows(x2)
    else:
        y = _lib().conv1x1_cat(g, mask, x2, sc, bi, w_cat, bias)
        v = torch.relu(_rows(x2) * sc + bi).bfloat16().float()
    u = a * (_bits(mask, K1) * _rows(g)) + c
    ref = torch.cat([u, v], 1) @ w.t()
    _close(_rows(y), ref, 1e-2)


@pytest.mark.parametrize("N,K1,K2,H", [(2, 256, 64, 28), (3, 512, 128, 14), (2, 1024, 256, 9),
                                       (1, 256, 64, 3)])
def test_conv1x1_cat_bnsums(cuda, N, K1, K2, H):
    """conv1x1_cat whose output feeds relu(bn(x2))'s backward: the epilogue's sums (ReLU mask
    recomputed from x2) against fp64 sums of the kernel's own output, and bn_bwd_apply from those
    sums against the two-pass bn_bwd."""
    g0 = torch.Generator(device=cuda).manual_seed(24)
    g = _nhwc(torch.randn(N, K1, H, H, device=cuda, generator=g0).bfloat16())
    x2 = _nhwc(torch.randn(N, K2, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    mask = _rand_mask(M, K1, cuda, g0)
    a = torch.randn(K1, device=cuda, generator=g0)
    c = torch.randn(K1, device=cuda, generator=g0) * 0.1
    gam = (torch.rand(K2, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = (torch.randn(K2, device=cuda, generator=g0) * 0.1).bfloat16()
    X = _rows(x2).double()
    mean = X.mean(0).float()
    invstd = (X.var(0, unbiased=False) + 1e-5).rsqrt().float()
    sc = gam.float() * invstd
    bi = bet.float() - mean * sc
    w = torch.randn(K2, K1 + K2, device=cuda, generator=g0) * (K1 + K2) ** -0.5
    from consensusml_amd.ops.conv import fold_cat
    w_cat, bias = fold_cat(w[:, :K1], a, c, w[:, K1:])
    y, s, q = _lib().conv1x1_cat_bnsums(g, mask, x2, sc, bi, w_cat, bias, mean, invstd)
    _close(_rows(y), _rows(_lib().conv1x1_cat(g, mask, x2, sc, bi, w_cat, bias)), 1e-2)
    m = (torch.addcmul(bi, _rows(x2), sc) > 0).double()
    dyv = _rows(y).double() * m
    s_ref = dyv.sum(0)
    q_ref = (dyv * (X - mean.double()) * invstd.double()).sum(0)
    _close(s, s_ref, 1e-5)
    _close(q, q_ref, 1e-5)
    dz = _lib().bn_bwd_apply(y, x2, gam, bet, mean, invstd, s, q)
    dz_ref, _, _, _ = _lib().bn_bwd(y, None, x2, None, gam, bet, mean, invstd, True, False)
    _close(_rows(dz), _rows(dz_ref), 1e-2)
    # the BN's parameter gradients from the sums' finalize launch == bn_bwd_coeffs' values
    dg, db = torch.empty_like(gam), torch.empty_like(bet)
    y2, s2, q2 = _lib().conv1x1_cat_bnsums(g, mask, x2, sc, bi, w_cat, bias, mean, invstd, dg, db)
    assert torch.equal(y2, y) and torch.equal(s2, s) and torch.equal(q2, q)
    _, _, _, dg_ref, db_ref = _lib().bn_bwd_coeffs(s, q, gam, mean, invstd, M)
    assert torch.equal(dg, dg_ref) and torch.equal(db, db_ref)


@pytest.mark.parametrize("N,Cin,Co,H", [(2, 64, 64, 20), (2, 128, 128, 14), (3, 256, 256, 7),
                                        (2, 512, 512, 5), (1, 64, 128, 3)])
def test_conv_gemm_bnsums(cuda, N, Cin, Co, H):
    """3x3 implicit GEMM whose output feeds relu(bn(z))'s backward: dy equal to conv_gemm's, the
    epilogue sums against fp64 sums of that output, bn_bwd_apply against the two-pass bn_bwd."""
    g0 = torch.Generator(device=cuda).manual_seed(25)
    x = _nhwc(torch.randn(N, Cin, H, H, device=cuda, generator=g0).bfloat16())
    z = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, 9 * Cin, device=cuda, generator=g0) * (9 * Cin) ** -0.5).bfloat16()
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
    _close(s, dyv.sum(0), 1e-5)
    _close(q, (dyv * (Z - mean.double()) * invstd.double()).sum(0), 1e-5)
    dz = _lib().bn_bwd_apply(y, z, gam, bet, mean, invstd, s, q)
    dz_ref, _, _, _ = _lib().bn_bwd(y, None, z, None, gam, bet, mean, invstd, True, False)
    _close(_rows(dz), _rows(dz_ref), 1e-2)


@pytest.mark.parametrize("H", [14, 28])
def test_bottleneck_bn1_dgrad_sums_matches_unfused(cuda, H):
    """A bottleneck block's gradients with bn1's backward sums from the 3x3 data gradient's
    epilogue equal those of bn_act + its own reduction pass. H = 14: conv1 on the library (its
    output under 784 pixels), bn1's statistics from a separate pass (bn1_sums_lib_conv1); H = 28:
    the statistics from the fused conv1's epilogue."""
    import consensusml_amd.models.resnet as R
    torch.manual_seed(5)
    blk = R.Bottleneck(256, 64).to(cuda, torch.bfloat16).to(memory_format=torch.channels_last)
    blk.train()
    x0 = _nhwc(torch.randn(4, 256, H, H, device=cuda).relu().bfloat16())
    gy = _nhwc(torch.randn(4, 256, H, H, device=cuda).bfloat16())
    grads = {}
    for on in (True, False):
        with perf.use_policy(perf.policy().replace(bn1_dgrad_sums=on, bn1_sums_lib_conv1=on)):
            b = copy.deepcopy(blk)
            x = x0.clone().requires_grad_(True)
            b(x).backward(gy)
        grads[on] = [x.grad] + [p.grad for p in b.parameters()]
    for a, r in zip(grads[True], grads[False]):
        _close(a, r, 2e-2)


@pytest.mark.parametrize("Co,Ci,H", [(256, 64, 28), (512, 128, 14), (64, 64, 20), (128, 128, 9),
                                    (1024, 256, 7), (256, 256, 7), (512, 512, 5)])
def test_wgrad1x1_ex_modes(cuda, Co, Ci, H):
    """Mode 2 (masked affine dy) and mode 3 (BN-ReLU dy), each with the column sums."""
    g0 = torch.Generator(device=cuda).manual_seed(23)
    N = 3
    dy = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    x = _nhwc(torch.randn(N, Ci, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    sc = torch.rand(Ci, device=cuda, generator=g0) + 0.5
    bi = torch.randn(Ci, device=cuda, generator=g0) * 0.1
    X = torch.relu(_rows(x) * sc + bi).bfloat16().float()
    mask = _rand_mask(M, Co, cuda, g0)
    a = torch.randn(Co, device=cuda, generator=g0)
    c = torch.randn(Co, device=cuda, generator=g0) * 0.1
    dw, cs = _lib().wgrad1x1_ex(dy, x, sc, bi, 2, mask, a, None, c, True)
    D = (a * (_bits(mask, Co) * _rows(dy)) + c).bfloat16().float()
    _close(dw, D.t() @ X, 1e-3)
    torch.testing.assert_close(cs, D.sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    da = torch.rand(Co, device=cuda, generator=g0) + 0.5
    db = torch.randn(Co, device=cuda, generator=g0) * 0.1
    dw3, cs3 = _lib().wgrad1x1_ex(dy, x, sc, bi, 3, None, da, db, None, True)
    D3 = torch.relu(_rows(dy) * da + db).bfloat16().float()
    _close(dw3, D3.t() @ X, 1e-3)
    torch.testing.assert_close(cs3, D3.sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)


@pytest.mark.parametrize("planes,H", [(64, 28), (128, 14), (256, 14), (512, 7)])
def test_identity_chain_recompute_tail(cuda, planes, H):
    """Three identity blocks with the recompute tail vs the stored-z3 fused tail, both against an
    fp32 run of the same weights (output, input gradient and every parameter gradient)."""
    m_on = _chain(cuda, planes, 3, seed=1)
    m_off = copy.deepcopy(m_on)
    m32 = copy.deepcopy(m_on).float()
    g0 = torch.Generator(device=cuda).manual_seed(6)
    x = _nhwc(torch.randn(8, planes * 4, H, H, device=cuda, generator=g0).bfloat16())
    gy = _nhwc(torch.randn(8, planes * 4, H, H, device=cuda, generator=g0).bfloat16())
    outs = {}
    for key, m, dt in (("on", m_on, torch.bfloat16), ("off", m_off, torch.bfloat16),
                       ("fp32", m32, torch.float32)):
        with perf.use_policy(perf.policy().replace(recompute_tail=key == "on",
                                                   recompute_tail_max_planes=4096)):
            xi = x.to(dt).clone().requires_grad_(True)
            y = m(xi)
            y.backward(gy.to(dt))
        outs[key] = (y.detach().float(), xi.grad.float(), [p.grad.float() for p in m.parameters()],
                     [b.float().clone() for b in m.buffers()])
    ref = outs["fp32"]
    for k in (0, 1):
        e_on, e_off = _err(outs["on"][k], ref[k]), _err(outs["off"][k], ref[k])
        assert e_on <= 1.5 * e_off + 1e-2, (k, e_on, e_off)
    for a, b, r in zip(outs["on"][2], outs["off"][2], ref[2]):
        e_on, e_off = _err(a, r), _err(b, r)
        assert e_on <= 1.5 * e_off + 2e-2, (e_on, e_off)
    for a, b in zip(outs["on"][3], outs["off"][3]):   # running statistics
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("cin,planes,H,stride", [(64, 64, 28, 1), (128, 128, 14, 1),
                                                 (256, 128, 28, 2), (128, 64, 14, 2),
                                                 (512, 256, 14, 2), (1024, 512, 8, 2)])
def test_downsample_recompute_tail(cuda, cin, planes, H, stride):
    """Downsample block (stride 1, or stride 2 through ops.conv.subsample2) with the recompute
    tail (no z3 / zd) vs the stored path, both against an fp32 copy: output, input gradient,
    parameter gradients, running statistics."""
    from consensusml_amd.models.resnet import Bottleneck
    torch.manual_seed(3)
    m_on = Bottleneck(cin, planes, stride, downsample=True)
    for mod in m_on.modules():
        if mod.__class__.__name__ == "BatchNormAct2d":
            with torch.no_grad():
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.1, 0.1)
    m_on = m_on.to(device=cuda, dtype=torch.bfloat16, memory_format=torch.channels_last).train()
    m_off = copy.deepcopy(m_on)
    m32 = copy.deepcopy(m_on).float()
    g0 = torch.Generator(device=cuda).manual_seed(7)
    x = _nhwc(torch.relu(torch.randn(8, cin, H, H, device=cuda, generator=g0)).bfloat16())
    Ho = (H - 1) // stride + 1
    gy = _nhwc(torch.randn(8, planes * 4, Ho, Ho, device=cuda, generator=g0).bfloat16())
    outs = {}
    for key, m, dt in (("on", m_on, torch.bfloat16), ("off", m_off, torch.bfloat16),
                       ("fp32", m32, torch.float32)):
        with perf.use_policy(perf.policy().replace(recompute_down_tail=key == "on",
                                                   down_tail_s2_max_cin=1024)):
            xi = x.to(dt).clone().requires_grad_(True)
            y = m(xi)
            y.backward(gy.to(dt))
        outs[key] = (y.detach().float(), xi.grad.float(), [p.grad.float() for p in m.parameters()],
                     [b.float().clone() for b in m.buffers()])
    ref = outs["fp32"]
    for k in (0, 1):
        e_on, e_off = _err(outs["on"][k], ref[k]), _err(outs["off"][k], ref[k])
        assert e_on <= 1.5 * e_off + 1e-2, (k, e_on, e_off)
    for a, b, r in zip(outs["on"][2], outs["off"][2], ref[2]):
        e_on, e_off = _err(a, r), _err(b, r)
        assert e_on <= 1.5 * e_off + 2e-2, (e_on, e_off)
    for a, b in zip(outs["on"][3], outs["off"][3]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("N,K,H", [(2, 64, 28), (3, 128, 14), (2, 256, 9), (1, 128, 3), (1, 512, 5)])
def test_bn_stats_gram_vs_fp64(cuda, N, K, H):
    """bn3's statistics from y2's Gram matrix (wgrad1x1_ex mode 3 + bn_stats_gram) equal the fp64
    statistics of z3 = y2 W^T (y2 = relu(z sc + bi) in bf16), running stats included."""
    g0 = torch.Generator(device=cuda).manual_seed(24)
    Co = 4 * K
    z = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, K, 1, 1, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    sc = torch.rand(K, device=cuda, generator=g0) + 0.5
    bi = torch.randn(K, device=cuda, generator=g0) * 0.1 + 0.2
    gram, cy = _lib().wgrad1x1_ex(z, z, sc, bi, 3, None, sc, bi, None, True)
    y2 = torch.relu(_rows(z) * sc + bi).bfloat16().double()
    M = y2.shape[0]
    torch.testing.assert_close(gram.double(), y2.t() @ y2, rtol=1e-5, atol=1e-3)
    rm = torch.randn(Co, device=cuda, generator=g0) * 0.1
    rv = torch.rand(Co, device=cuda, generator=g0) + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    mean, invstd = _lib().bn_stats_gram(gram, cy, w, M, rm, rv, 1e-5, 0.1)
    z3 = y2 @ w.view(Co, K).double().t()
    m_ref = z3.mean(0)
    v_ref = z3.var(0, unbiased=False)
    torch.testing.assert_close(mean.double(), m_ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(invstd.double(), torch.rsqrt(v_ref + 1e-5), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rm.double(), 0.9 * rm0.double() + 0.1 * m_ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv.double(), 0.9 * rv0.double() + 0.1 * z3.var(0, unbiased=True),
                               rtol=1e-4, atol=1e-5)
    # with gamma / beta the same launch also returns the BN affine, bit-identical to bn_affine
    gam = (torch.rand(Co, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = (torch.randn(Co, device=cuda, generator=g0) * 0.1).bfloat16()
    m2, i2, sc3, bi3 = _lib().bn_stats_gram(gram, cy, w, M, None, None, 1e-5, 0.1, gam, bet)
    assert torch.equal(m2, mean) and torch.equal(i2, invstd)
    ab = _lib().bn_affine(gam, bet, mean, invstd)
    assert torch.equal(sc3, ab[0]) and torch.equal(bi3, ab[1])


@pytest.mark.parametrize("N,C,H,W", [(2, 256, 56, 56), (3, 64, 7, 9), (1, 512, 14, 14)])
def test_subsample2_and_scatter(cuda, N, C, H, W):
    """subsample2 = x[:, :, ::2, ::2] (dense NHWC) and its backward scatter (zeros at odd pixels),
    exactly; through ops.conv.subsample2's autograd too."""
    from consensusml_amd.ops import conv as fconv
    g0 = torch.Generator(device=cuda).manual_seed(25)
    x = _nhwc(torch.randn(N, C, H, W, device=cuda, generator=g0).bfloat16())
    y = _lib().subsample2(x)
    assert torch.equal(y, x[:, :, ::2, ::2])
    assert y.is_contiguous(memory_format=torch.channels_last)
    g = _nhwc(torch.randn(y.shape, device=cuda, generator=g0).bfloat16())
    dx = _lib().upsample2_scatter(g, H, W)
    ref = torch.zeros_like(x)
    ref[:, :, ::2, ::2] = g
    assert torch.equal(dx, ref)
    xi = x.clone().requires_grad_(True)
    fconv.subsample2(xi).backward(g)
    assert torch.equal(xi.grad, ref)


@pytest.mark.parametrize("N,K,No,H,W", [(2, 128, 256, 56, 56), (3, 64, 128, 7, 9),
                                        (1, 512, 1024, 14, 14)])
def test_conv1x1_link_s2(cuda, N, K, No, H, W):
    """dX = dY W^T plus a stride-2 conv's compact gradient at the even pixels, vs fp32."""
    g0 = torch.Generator(device=cuda).manual_seed(26)
    dy = _nhwc(torch.randn(N, K, H, W, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(No, K, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    g = _nhwc(torch.randn(N, No, (H + 1) // 2, (W + 1) // 2, device=cuda, generator=g0).bfloat16())
    y = _lib().conv1x1_link_s2(dy, w.contiguous(), g)
    full = torch.zeros(N, No, H, W, device=cuda)
    full[:, :, ::2, ::2] = g.float()
    ref = _rows(dy) @ w.float().t() + _rows(full)
    _close(_rows(y), ref, 1e-2)


@pytest.mark.parametrize("C", [64, 256, 2048, 100])
def test_bn_affine_bit_identical(cuda, C):
    """bn_affine (one launch) equals gamma.float() * invstd and beta.float() - mean * sc bit for
    bit."""
    g0 = torch.Generator(device=cuda).manual_seed(C)
    gam = (torch.rand(C, device=cuda, generator=g0) + 0.5).bfloat16()
    bet = torch.randn(C, device=cuda, generator=g0).bfloat16()
    mean = torch.randn(C, device=cuda, generator=g0)
    invstd = torch.rand(C, device=cuda, generator=g0) * 3 + 0.1
    ab = _lib().bn_affine(gam, bet, mean, invstd)
    sc = gam.float() * invstd
    assert torch.equal(ab[0], sc)
    assert torch.equal(ab[1], bet.float() - mean * sc)


@pytest.mark.parametrize("Co,p,need_dw", [(256, 64, True), (1024, 256, True), (512, 128, False),
                                          (2048, 512, True)])
def test_tail_bwd_prep_vs_torch(cuda, Co, p, need_dw):
    """tail_bwd_prep's two launches against the fp64 PyTorch algebra they replace: bn3's backward
    coefficients / dgamma / dbeta, dW3 = diag(a) P + diag(b) W Gram + c cy^T, and the folded
    w_cat = [W^T diag(a) | W^T diag(b) W], bias = W^T c."""
    g0 = torch.Generator(device=cuda).manual_seed(41)
    M = 4096
    w = (torch.randn(Co, p, 1, 1, device=cuda, generator=g0) * p ** -0.5).bfloat16()
    y = torch.relu(torch.randn(M, p, device=cuda, generator=g0)).bfloat16().float()
    u = torch.randn(M, Co, device=cuda, generator=g0).bfloat16().float()
    P, s = (u.t() @ y).contiguous(), u.sum(0)
    gram, cy = (y.t() @ y).contiguous(), y.sum(0)
    g3 = (torch.rand(Co, device=cuda, generator=g0) + 0.5).bfloat16()
    m3 = torch.randn(Co, device=cuda, generator=g0) * 0.1
    i3 = torch.rand(Co, device=cuda, generator=g0) + 0.5
    w_cat, bias, dw, dg, db = _lib().tail_bwd_prep(w, P, s, gram, cy, g3, m3, i3, M, need_dw)
    W = w.view(Co, p).double()
    Pd, sd, Gd, cyd = P.double(), s.double(), gram.double(), cy.double()
    q = ((W * Pd).sum(1) - m3.double() * sd) * i3.double()
    a = i3.double() * g3.double()
    b = -a * i3.double() * q / M
    c = -a * sd / M - b * m3.double()
    _close(dg, q, 1e-2)
    _close(db, sd, 1e-2)
    if need_dw:
        dw_ref = a[:, None] * Pd + b[:, None] * (W @ Gd) + c[:, None] * cyd[None, :]
        _close(dw, dw_ref, 1e-2)
    else:
        assert dw is None
    wc_ref = torch.cat([W.t() * a[None, :], W.t() @ (b[:, None] * W)], 1)
    assert w_cat.shape == (p, Co + p)
    _close(w_cat[:, :Co], wc_ref[:, :Co], 1e-2)
    _close(w_cat[:, Co:], wc_ref[:, Co:], 1e-2)
    _close(bias, W.t() @ c, 1e-4)
