"""The global_load_lds fused 1x1 kernels (csrc/kernels/conv1x1g.hip) against the register-staged
kernels of conv1x1.hip (same launchers, ``set_conv1x1g_mode`` 1 = the 2-buffer kernel, 3 = the
quad-phase ping-pong kernel where eligible (N % 256 == 0, K >= 128), vs 0) and against fp32
oracles.

The two families compute the same bf16 operands (same prologue arithmetic) and the same MFMA
products in the same k order, so every stored output is compared bit for bit; BN statistics and
BN-backward sums are folded from differently shaped partial slabs (fp64), so they agree to float
rounding. Shapes include partial m-tiles (M not a multiple of 256, whole wave blocks past M) and
both tile widths (N % 256 == 0: 256 x 256 tiles; N = 128: 256 x 128)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from consensusml_amd.ops.native import lib
    return lib()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rows(t):
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1]).float()


def _bits(mask, C):
    sh = torch.arange(8, device=mask.device, dtype=torch.uint8)
    return ((mask.view(-1, C // 8, 1) >> sh) & 1).view(-1, C).float()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


_MODE = [3]


def _both(fn):
    """fn() under conv1x1.hip (mode 0) and the quad-phase DMA kernel (mode 3, where eligible)."""
    L = _lib()
    prev = L.conv1x1g_mode()
    try:
        L.set_conv1x1g_mode(0)
        a = fn()
        L.set_conv1x1g_mode(_MODE[0])
        b = fn()
    finally:
        L.set_conv1x1g_mode(prev)
    return a, b


SHAPES = [(2, 256, 256, 14), (3, 512, 128, 9), (1, 1024, 512, 7), (2, 128, 256, 3)]


@pytest.mark.parametrize("pro", [False, True])
@pytest.mark.parametrize("N,K,Co,H", SHAPES)
def test_bn_fwd_and_stats_only(cuda, pro, N, K, Co, H):
    g0 = torch.Generator(device=cuda).manual_seed(31)
    x = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, K, 1, 1, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    sc = (torch.rand(K, device=cuda, generator=g0) + 0.5) if pro else None
    bi = (torch.randn(K, device=cuda, generator=g0) * 0.1) if pro else None
    rm = torch.randn(Co, device=cuda, generator=g0) * 0.1
    rv = torch.rand(Co, device=cuda, generator=g0) + 0.5
    L = _lib()

    def run():
        r1, r2 = rm.clone(), rv.clone()
        y, m, i = L.conv1x1_bn_fwd(x, w, sc, bi, r1, r1, r2, 1, True, 1e-5, 0.1)
        m2, i2 = L.conv1x1_bn_stats_only(x, w, sc, bi, rm.clone(), None, None, 1e-5, 0.1)
        y0, m0, _ = L.conv1x1_bn_fwd(x, w, sc, bi, None, None, None, 1, False, 1e-5, 0.1)
        assert m0 is None
        return y, m, i, r1, r2, m2, i2, y0

    a, b = _both(run)
    assert torch.equal(a[0], b[0]) and torch.equal(a[7], b[7]) and torch.equal(b[0], b[7])
    a, b = a[:7], b[:7]
    for u, v in zip(a[1:], b[1:]):
        torch.testing.assert_close(u, v, rtol=2e-5, atol=1e-6)
    xin = _rows(x)
    if pro:
        xin = torch.relu(xin * sc + bi).bfloat16().float()
    ref = xin @ w.view(Co, K).float().t()
    assert _rel(_rows(b[0]), ref) < 1e-2
    yb = _rows(b[0]).double()
    torch.testing.assert_close(b[1].double(), yb.mean(0), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("sums", [False, True])
@pytest.mark.parametrize("N,K,No,H", [(2, 256, 1024, 7), (3, 512, 2048, 5), (2, 256, 512, 14),
                                      (1, 512, 128, 9)])
def test_link(cuda, sums, N, K, No, H):
    g0 = torch.Generator(device=cuda).manual_seed(32)
    x = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(No, K, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    link = _nhwc(torch.randn(N, No, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    lm = torch.randint(0, 256, (M, No // 8), generator=g0, device=cuda, dtype=torch.uint8)
    extra = ()
    if sums:
        sz = _nhwc(torch.randn(N, No, H, H, device=cuda, generator=g0).bfloat16())
        sm = torch.randint(0, 256, (M, No // 8), generator=g0, device=cuda, dtype=torch.uint8)
        mean = torch.randn(No, device=cuda, generator=g0) * 0.1
        invstd = torch.rand(No, device=cuda, generator=g0) + 0.5
        extra = (sz, sm, mean, invstd)
    a, b = _both(lambda: _lib().conv1x1_link(x, w, link, lm, *extra))
    assert torch.equal(a[0], b[0])
    ref = (_rows(x) @ w.float().t()).bfloat16().float() + _bits(lm, No) * _rows(link)
    assert _rel(_rows(b[0]), ref) < 1e-2
    if sums:
        torch.testing.assert_close(a[1], b[1], rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(a[2], b[2], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("N,K,No,H,W", [(2, 256, 1024, 14, 14), (3, 512, 256, 7, 9)])
def test_link_s2(cuda, N, K, No, H, W):
    g0 = torch.Generator(device=cuda).manual_seed(33)
    dy = _nhwc(torch.randn(N, K, H, W, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(No, K, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    g = _nhwc(torch.randn(N, No, (H + 1) // 2, (W + 1) // 2, device=cuda, generator=g0).bfloat16())
    a, b = _both(lambda: _lib().conv1x1_link_s2(dy, w.contiguous(), g))
    assert torch.equal(a, b)


@pytest.mark.parametrize("N,K,H", [(2, 256, 14), (3, 128, 9), (1, 512, 7)])
def test_bnres(cuda, N, K, H):
    g0 = torch.Generator(device=cuda).manual_seed(34)
    Co = 4 * K
    z = _nhwc(torch.randn(N, K, H, H, device=cuda, generator=g0).bfloat16())
    w = (torch.randn(Co, K, 1, 1, device=cuda, generator=g0) * K ** -0.5).bfloat16()
    sc = torch.rand(K, device=cuda, generator=g0) + 0.5
    bi = torch.randn(K, device=cuda, generator=g0) * 0.1
    sc3 = torch.rand(Co, device=cuda, generator=g0) + 0.5
    bi3 = torch.randn(Co, device=cuda, generator=g0) * 0.1
    res = _nhwc(torch.randn(N, Co, H, H, device=cuda, generator=g0).bfloat16())
    a, b = _both(lambda: _lib().conv1x1_bnres(z, w, sc, bi, sc3, bi3, res))
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("bnsums", [False, True])
@pytest.mark.parametrize("N,K1,K2,H", [(2, 512, 128, 14), (2, 1024, 256, 9), (1, 1024, 256, 3),
                                       (2, 2048, 512, 7)])
def test_cat(cuda, bnsums, N, K1, K2, H):
    g0 = torch.Generator(device=cuda).manual_seed(35)
    g = _nhwc(torch.randn(N, K1, H, H, device=cuda, generator=g0).bfloat16())
    x2 = _nhwc(torch.randn(N, K2, H, H, device=cuda, generator=g0).bfloat16())
    M = N * H * H
    mask = torch.randint(0, 256, (M, K1 // 8), generator=g0, device=cuda, dtype=torch.uint8)
    a1 = torch.randn(K1, device=cuda, generator=g0)
    c1 = torch.randn(K1, device=cuda, generator=g0) * 0.1
    sc = torch.rand(K2, device=cuda, generator=g0) + 0.5
    bi = torch.randn(K2, device=cuda, generator=g0) * 0.1
    w = torch.randn(K2, K1 + K2, device=cuda, generator=g0) * (K1 + K2) ** -0.5
    from consensusml_amd.ops.conv import fold_cat
    w_cat, bias = fold_cat(w[:, :K1], a1, c1, w[:, K1:])
    L = _lib()
    if not bnsums:
        a, b = _both(lambda: L.conv1x1_cat(g, mask, x2, sc, bi, w_cat, bias))
        assert torch.equal(a, b)
        u = a1 * (_bits(mask, K1) * _rows(g)) + c1
        v = torch.relu(_rows(x2) * sc + bi).bfloat16().float()
        assert _rel(_rows(b), torch.cat([u, v], 1) @ w.t()) < 1e-2
        xr = torch.relu(x2)   # identity second source (a ReLU output staged as is)
        a, b = _both(lambda: L.conv1x1_cat(g, mask, xr, None, None, w_cat, bias))
        assert torch.equal(a, b)
        assert _rel(_rows(b), torch.cat([u, _rows(xr)], 1) @ w.t()) < 1e-2
        return
    X = _rows(x2).double()
    mean = X.mean(0).float()
    invstd = (X.var(0, unbiased=False) + 1e-5).rsqrt().float()
    a, b = _both(lambda: L.conv1x1_cat_bnsums(g, mask, x2, sc, bi, w_cat, bias, mean, invstd))
    assert torch.equal(a[0], b[0])
    torch.testing.assert_close(a[1], b[1], rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(a[2], b[2], rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,K1,K2,Co,H", [(2, 128, 256, 512, 14), (1, 256, 512, 1024, 7),
                                          (3, 64, 64, 256, 9)])
def test_cat_bnres(cuda, N, K1, K2, Co, H):
    """The downsample tail's K-concatenated apply GEMM (both sources through max(x sc + bi, 0))."""
    g0 = torch.Generator(device=cuda).manual_seed(36)
    x1 = _nhwc(torch.randn(N, K1, H, H, device=cuda, generator=g0).bfloat16())
    x2 = _nhwc(torch.randn(N, K2, H, H, device=cuda, generator=g0).bfloat16())
    sc = torch.rand(K1 + K2, device=cuda, generator=g0) + 0.5
    bi = torch.randn(K1 + K2, device=cuda, generator=g0) * 0.1
    w = (torch.randn(Co, K1 + K2, device=cuda, generator=g0) * (K1 + K2) ** -0.5).bfloat16()
    esc = torch.rand(Co, device=cuda, generator=g0) + 0.5
    ebi = torch.randn(Co, device=cuda, generator=g0) * 0.1
    a, b = _both(lambda: _lib().conv1x1_cat_bnres(x1, x2, sc[:K1], bi[:K1], sc[K1:], bi[K1:],
                                                  w.contiguous(), esc, ebi))
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    xr = torch.relu(x2)   # identity second source == max(x * 1 + 0, 0) of a ReLU output
    a, b = _both(lambda: _lib().conv1x1_cat_bnres(x1, xr, sc[:K1], bi[:K1], None, None,
                                                  w.contiguous(), esc, ebi))
    one, zero = torch.ones(K2, device=cuda), torch.zeros(K2, device=cuda)
    c = _lib().conv1x1_cat_bnres(x1, xr, sc[:K1], bi[:K1], one, zero, w.contiguous(), esc, ebi)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert torch.equal(a[0], c[0]) and torch.equal(a[1], c[1])
