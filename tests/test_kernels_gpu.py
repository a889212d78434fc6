"""HIP kernel numerics vs the pure-PyTorch fp32/fp64 oracles."""
import math

import pytest
import torch

from consensusml_amd.ops import kernels as K
from consensusml_amd.ops import reference as R

pytestmark = pytest.mark.gpu

NS = [1, 2, 3, 5, 8, 9, 16, 17, 33, 64]


def _x(n, D, dtype, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.randn(n, D, generator=g, device=dev).to(dtype)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("D", [4096, 1001])
def test_median_trimmed(cuda, dtype, n, D):
    X = _x(n, D, dtype, cuda, n)
    got = K.aggregate(X, "median")
    ref = R.coord_median(X.float())
    assert torch.equal(got, ref) or torch.allclose(got, ref, atol=1e-6, rtol=1e-6)
    if n >= 3:
        b = (n - 1) // 2 if n < 5 else 2
        got = K.aggregate(X, "trimmed_mean", trim=b)
        ref = R.trimmed_mean(X.float(), b)
        torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_median_nan_and_ties(cuda, dtype):
    X = torch.zeros(5, 256, device=cuda)
    X[0] = float("nan")
    X[1] = 1.0
    X[2] = 1.0
    X[3] = -1.0
    X = X.to(dtype)
    if dtype == torch.bfloat16:    # negative-sign NaN and -0.0 bit patterns for the u16 keys
        bits = X.view(torch.int16)
        bits[0, ::2] = -64          # 0xFFC0: -NaN
        bits[4, 1::2] = -32768      # 0x8000: -0.0
    got = K.aggregate(X, "median")
    torch.testing.assert_close(got, R.coord_median(X.float()))
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("n", [4, 8, 16])
def test_sorted_bf16_extremes(cuda, n):
    """+-inf, +-NaN, +-0 and subnormal bf16 values through the packed-key sort."""
    g = torch.Generator(device=cuda).manual_seed(n)
    X = torch.randn(n, 4096, generator=g, device=cuda).to(torch.bfloat16)
    bits = X.view(torch.int16)
    special = torch.tensor([0x7F80, -128, 0x7FC0, -64, 0, -32768, 1, -32767],  # +inf -inf +nan -nan +0 -0 sub -sub
                           dtype=torch.int16, device=cuda)
    idx = torch.randint(0, n * 4096, (n * 512,), generator=g, device=cuda)
    bits.view(-1)[idx] = special[torch.arange(idx.numel(), device=cuda) % 8]
    Xf = X.float()
    for lo, cnt in [(n // 2 - 1, 2), (1, n - 2), (0, n)]:
        got = torch.empty(4096, device=cuda)
        K.agg_update(X, combine="sorted", lo=lo, cnt=cnt, gout=got)
        ref = torch.where(torch.isnan(Xf), torch.inf, Xf).sort(0).values[lo:lo + cnt].mean(0)
        torch.testing.assert_close(got, ref, atol=1e-6, rtol=1e-6, equal_nan=True)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", NS)
@pytest.mark.parametrize("D", [8192, 1000, 37, 65544])
def test_gram(cuda, dtype, n, D):
    X = _x(n, D, dtype, cuda, 7 * n)
    G = K.gram(X)
    ref = R.gram(X.float())
    scale = (X.float().abs() ** 2).sum(1).max().item()
    assert (G - ref).abs().max().item() <= 1e-5 * scale + 1e-6


@pytest.mark.parametrize("n", [3, 7, 20])
def test_gram_asymmetric_rows(cuda, n):
    # rows with very different scales catch a transposed / row-swapped C write (and, for n <= 8,
    # a mis-folded column-group block)
    D = 20488
    X = torch.randn(n, D, device=cuda) * torch.arange(1, n + 1, device=cuda)[:, None]
    G = K.gram(X)
    ref = R.gram(X)
    # fp32 products accumulated in fp32 per lane: error scales with the largest squared norm
    torch.testing.assert_close(G, ref, rtol=0, atol=1e-7 * ref.diagonal().max().item())


def test_gram_accumulate_and_rows(cuda):
    X = _x(8, 4096, torch.bfloat16, cuda)
    G = K.gram(X[:, :2048])
    K.gram(X[:, 2048:], out=G, accumulate=True)
    torch.testing.assert_close(G, R.gram(X.float()), rtol=1e-5, atol=1e-2)
    rows = torch.tensor([5, 1, 3], dtype=torch.int32, device=cuda)
    G2 = K.gram(X, rows=rows)
    torch.testing.assert_close(G2, R.gram(X[rows.long()].float()), rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("rule", ["krum", "multi_krum", "geomed", "bulyan", "centered_clip", "mean"])
@pytest.mark.parametrize("n", [3, 7, 8, 16])
def test_gram_rules(cuda, rule, n):
    f = 1 if rule != "bulyan" else (n - 3) // 4
    if rule == "bulyan" and f < 1:
        f = 0
    X = _x(n, 4096, torch.float32, cuda, 3)
    X[0] *= 50          # an outlier
    got = K.aggregate(X, rule, f=f)
    ref = R.aggregate(X.cpu(), rule, f=f)
    torch.testing.assert_close(got.cpu(), ref, rtol=2e-4, atol=2e-4)


def test_weights_kernel_matches_oracle(cuda):
    n = 12
    X = _x(n, 2048, torch.float32, cuda, 11)
    G = R.gram(X).to(cuda)
    for rule in ["krum", "multi_krum", "geomed"]:
        w = K.robust_weights(G, rule, n, f=2, m=6)
        wr = K.robust_weights(G.cpu(), rule, n, f=2, m=6)
        torch.testing.assert_close(w.cpu(), wr, rtol=1e-5, atol=1e-6)
    sc = torch.zeros(n, dtype=torch.float64, device=cuda)
    K.robust_weights(G, "krum", n, f=2, scores=sc)
    torch.testing.assert_close(sc.cpu(), R.krum_scores(G.cpu(), 2), rtol=1e-9, atol=1e-6)


def test_weights_nonfinite_worker(cuda):
    X = _x(6, 1024, torch.float32, cuda)
    X[2, 5] = float("nan")
    for rule in ["krum", "multi_krum", "geomed", "median", "trimmed_mean"]:
        out = K.aggregate(X, rule, f=1)
        assert torch.isfinite(out).all(), rule
    # the robust "mean" weights (RULE_MEAN) drop the non-finite worker too
    w = K.robust_weights(K.gram(X), "mean", 6)
    assert w[2].item() == 0.0 and abs(w.sum().item() - 1.0) < 1e-6


@pytest.mark.parametrize("bad", ["nan", "inf"])
def test_weights_nonfinite_cclip_bulyan(cuda, bad):
    """Centered clipping and Bulyan with a NaN / overflowed worker match the CPU oracle
    (which zeroes the bad rows and columns) and stay finite: clipping must stay ON for the
    honest workers."""
    n, D = 7, 2048
    X = _x(n, D, torch.float32, cuda, 3)
    X[4, 17] = float(bad)
    v0 = torch.randn(D, device=cuda) * 0.1
    Xa = torch.cat([X, v0[None]], 0)
    G = K.gram(Xa)
    w = K.robust_weights(G, "centered_clip", n, tau=0.5, iters=3)
    ref = R.centered_clip_weights(G.cpu().double(), tau=0.5, iters=3).float()
    assert torch.isfinite(w).all()
    assert w[4].item() == 0.0
    torch.testing.assert_close(w.cpu(), ref, rtol=1e-5, atol=1e-6)
    # clipping is active: weights are not the unclipped 1/n mean
    assert (w[:n].sum() - 1.0).abs().item() > 1e-3 or w[n].abs().item() > 1e-3
    out = K.aggregate(X, "bulyan", f=1)
    assert torch.isfinite(out).all()
    Xh = torch.cat([X[:4], X[5:]], 0)
    assert (out.cpu() - Xh.cpu().median(0).values).abs().max() < (Xh.cpu().abs().max() + 1)


def test_geomed_gram_vs_direct(cuda):
    X = _x(9, 4096, torch.float32, cuda, 5)
    X[:2] += 20.0
    got = K.aggregate(X, "geomed", iters=50)
    ref = R.geomed_direct(X.cpu(), iters=50)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
@pytest.mark.parametrize("combine", ["sorted", "weighted"])
def test_fused_update(cuda, kind, combine):
    n, D = 5, 10007
    X = _x(n, D, torch.bfloat16, cuda, 1)
    master = torch.randn(D, device=cuda)
    s1 = torch.randn(D, device=cuda).abs() if kind == "sgd" else torch.zeros(D, device=cuda)
    s2 = torch.zeros(D, device=cuda) if kind != "sgd" else None
    p = torch.empty(D, dtype=torch.bfloat16, device=cuda)
    opt = K.OptArgs(kind=kind, lr=0.05, momentum=0.9 if kind == "sgd" else 0.0,
                    weight_decay=0.01, nesterov=kind == "sgd", step=3)
    w = torch.rand(n, device=cuda)
    w[1] = 0
    m0, s10 = master.clone(), s1.clone()
    s20 = s2.clone() if s2 is not None else None
    if combine == "sorted":
        lo, cnt = K.sorted_range("median", n)
        K.agg_update(X, combine="sorted", lo=lo, cnt=cnt, opt=opt, master=master, s1=s1, s2=s2,
                     param_out=p)
        g = R.coord_median(X.float())
    else:
        K.agg_update(X, combine="weighted", w=w, opt=opt, master=master, s1=s1, s2=s2,
                     param_out=p)
        g = (w[:, None] * X.float()).sum(0)
    if kind == "sgd":
        pr, br = R.sgd_update(m0, g, s10, 0.05, 0.9, 0.01, True, False)
        torch.testing.assert_close(s1, br, rtol=1e-5, atol=1e-5)
    else:
        # adam: L2 term in the gradient (torch.optim.Adam); adamw: decoupled decay
        pr, mr, vr = R.adam_update(m0, g, s10, s20, 3, 0.05, 0.9, 0.999, 1e-8, 0.01,
                                   decoupled=kind == "adamw")
        # fp32 fma-order differences: relative error ~1e-5 on g^2 terms
        torch.testing.assert_close(s1, mr, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(s2, vr, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(master, pr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(p, pr.to(torch.bfloat16))


def test_gossip_mix(cuda):
    D = 100003
    x = torch.randn(D, device=cuda)
    l = torch.randn(D, device=cuda).to(torch.bfloat16)
    r = (torch.randn(D, device=cuda) * 5).to(torch.bfloat16)
    for clip in [0.0, 10.0]:
        xx = x.clone()
        p = torch.empty(D, dtype=torch.bfloat16, device=cuda)
        K.gossip_mix(xx, l, r, 0.5, 0.25, 0.25, clip, param_out=p)
        ref = R.gossip_mix(x, l, r, 0.5, 0.25, 0.25, clip)
        torch.testing.assert_close(xx, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("k", [1, 2, 3, 5, 7, 8])
def test_gossip_mix_k(cuda, k):
    """k-neighbour mixing vs the fp64 reference; k = 2 bit-identical to the ring kernel."""
    D = 100003
    g = torch.Generator(device=cuda).manual_seed(k)
    x = torch.randn(D, device=cuda, generator=g)
    nbs = [(torch.randn(D, device=cuda, generator=g) * (1 + i)).to(torch.bfloat16)
           for i in range(k)]
    w = [0.1 * (i + 1) for i in range(k)]
    for clip in [0.0, 20.0]:
        xx = x.clone()
        p = torch.empty(D, dtype=torch.bfloat16, device=cuda)
        K.gossip_mix_k(xx, nbs, w, 0.3, clip, param_out=p)
        ref = R.gossip_mix_k(x, nbs, w, 0.3, clip)
        torch.testing.assert_close(xx, ref, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(p, xx.to(torch.bfloat16))
        if k == 2:
            yy = x.clone()
            K.gossip_mix(yy, nbs[0], nbs[1], 0.3, w[0], w[1], clip)
            assert torch.equal(xx, yy)


def test_fault_kernel(cuda):
    g = torch.randn(4096, device=cuda).to(torch.bfloat16)
    h = g.clone()
    K.inject_fault(h, "sign_flip", scale=2.0)
    torch.testing.assert_close(h.float(), -2.0 * g.float())
    K.inject_fault(h, "gaussian", sigma=3.0, seed=1)
    assert 2.5 < h.float().std().item() < 3.5
    K.inject_fault(h, "nan")
    assert torch.isnan(h.float()).all()


def test_deterministic_bitwise(cuda):
    X = _x(8, 1 << 20, torch.bfloat16, cuda, 2)
    a = K.gram(X).clone()
    b = K.gram(X).clone()
    assert torch.equal(a, b)
    m1 = K.aggregate(X, "trimmed_mean", trim=2)
    m2 = K.aggregate(X, "trimmed_mean", trim=2)
    assert torch.equal(m1, m2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_multi_copy(cuda, dtype):
    """Gradient capture copy: many tensors (odd sizes, > 32 entries -> several launches), with
    non-qualifying (misaligned / non-contiguous) entries reported back to the caller."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(0)
    sizes = [1, 7, 8, 9, 64, 1000, 4099, 123457] * 5
    buf = torch.zeros(sum(s + 128 for s in sizes), device=cuda, dtype=dtype)
    dst, src, off = [], [], 0
    for s in sizes:
        dst.append(buf[off:off + s])
        src.append(torch.randn(s, device=cuda).to(dtype))
        off += (s + 63) // 64 * 64 + 64
    bad_src = torch.randn(10, device=cuda).to(dtype)[1:]          # misaligned view
    bad_dst = torch.zeros(9, device=cuda, dtype=dtype)
    rest = lib().multi_copy(dst + [bad_dst], src + [bad_src])
    assert rest == [len(dst)]
    torch.cuda.synchronize()
    for d, s in zip(dst, src):
        assert torch.equal(d, s)


def test_multi_copy_channels_last(cuda):
    """Same-strided dense 4-D tensors (channels_last conv weights and their gradients) go through
    the byte copy; a contiguous destination for a channels_last source stays with the caller."""
    from consensusml_amd.ops.native import lib
    torch.manual_seed(1)
    cl = torch.channels_last
    src = [torch.randn(64, 32, 3, 3, device=cuda).bfloat16().contiguous(memory_format=cl),
           torch.randn(128, 64, 3, 3, device=cuda).bfloat16().contiguous(memory_format=cl)]
    dst = [torch.zeros_like(t, memory_format=cl) for t in src]
    mixed = torch.zeros(64, 32, 3, 3, device=cuda, dtype=torch.bfloat16)   # contiguous
    rest = lib().multi_copy(dst + [mixed], src + [src[0]])
    assert rest == [2]
    torch.cuda.synchronize()
    for d, s in zip(dst, src):
        assert torch.equal(d, s)
