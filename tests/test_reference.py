"""Property tests of the aggregation oracles — CPU."""
import pytest
import torch

from consensusml_amd.ops import kernels as K
from consensusml_amd.ops import reference as R

RULES = ["mean", "median", "trimmed_mean", "krum", "multi_krum", "geomed", "bulyan",
         "centered_clip"]


def _rule_f(rule, n):
    if rule == "bulyan":
        return max(0, (n - 3) // 4)
    if rule in ("krum", "multi_krum"):
        return max(0, (n - 3) // 2)
    if rule == "trimmed_mean":
        return max(0, (n - 1) // 2 - 1)
    return 0


@pytest.mark.parametrize("rule", RULES)
def test_identical_inputs(rule):
    x = torch.randn(257)
    X = x[None].repeat(7, 1)
    out = R.aggregate(X, rule, f=_rule_f(rule, 7), tau=1e9, v0=x)
    torch.testing.assert_close(out, x, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("rule", ["mean", "median", "trimmed_mean", "geomed", "multi_krum"])
def test_permutation_invariance(rule):
    torch.manual_seed(0)
    X = torch.randn(9, 300)
    perm = torch.randperm(9)
    a = R.aggregate(X, rule, f=2, m=9)
    b = R.aggregate(X[perm], rule, f=2, m=9)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("rule", ["median", "trimmed_mean", "bulyan"])
def test_coordinate_bounds(rule):
    X = torch.randn(11, 500)
    out = R.aggregate(X, rule, f=2)
    assert (out <= X.max(0).values + 1e-6).all() and (out >= X.min(0).values - 1e-6).all()


@pytest.mark.parametrize("n,f", [(7, 2), (10, 3), (16, 5)])
def test_krum_picks_honest(n, f):
    torch.manual_seed(n)
    honest = torch.randn(n - f, 1000) * 0.1 + 1.0
    byz = torch.randn(f, 1000) * 0.1 - 50.0
    X = torch.cat([byz, honest])
    w = R.krum_weights(R.gram(X), f, 1)
    assert w[:f].sum() == 0
    w = R.krum_weights(R.gram(X), f, n - f)
    assert w[:f].sum() == 0


def test_median_even_and_nan():
    X = torch.tensor([[1.0, float("nan")], [3.0, 2.0], [2.0, 5.0], [10.0, 1.0]])
    out = R.coord_median(X)
    torch.testing.assert_close(out, torch.tensor([2.5, 3.5]))


def test_geomed_gram_equals_direct():
    torch.manual_seed(1)
    X = torch.randn(9, 400)
    X[:3] += 10
    a = R.aggregate(X, "geomed", iters=60)
    b = R.geomed_direct(X, iters=60)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_geomed_robust_to_outliers():
    torch.manual_seed(2)
    X = torch.randn(9, 100) * 0.1
    X[:4] = 1000.0
    out = R.aggregate(X, "geomed", iters=100)
    assert out.abs().max() < 5.0


def test_centered_clip_bounds_outlier():
    torch.manual_seed(3)
    X = torch.randn(8, 100)
    X[0] = 1e6
    out = R.aggregate(X, "centered_clip", tau=1.0, clip_iters=5)
    assert out.norm() < 10


def test_nonfinite_worker_excluded():
    X = torch.randn(6, 50)
    X[1, 3] = float("inf")
    for rule in ["krum", "multi_krum", "geomed", "centered_clip"]:
        out = R.aggregate(X, rule, f=1)
        assert torch.isfinite(out).all(), rule


def test_bulyan_select_count():
    X = torch.randn(11, 64)
    sel = R.bulyan_select(R.gram(X), 2)
    assert sel.numel() == 7 and len(set(sel.tolist())) == 7


def test_vote_is_intersection():
    X = torch.tensor([[1.0, 0.0, 2.0], [3.0, 0.0, 0.0], [1.0, 1.0, 1.0]])
    v = R.vote(X)
    assert v.tolist() == [3.0, 1.0, 2.0]


def test_sorted_range():
    assert K.sorted_range("median", 5) == (2, 1)
    assert K.sorted_range("median", 4) == (1, 2)
    assert K.sorted_range("trimmed_mean", 7, 2) == (2, 3)
    with pytest.raises(ValueError):
        K.sorted_range("trimmed_mean", 4, 2)


@pytest.mark.parametrize("rule", RULES)
def test_cpu_dispatch_matches_oracle(rule):
    torch.manual_seed(4)
    X = torch.randn(7, 333)
    f = _rule_f(rule, 7)
    a = K.aggregate(X, rule, f=f)
    b = R.aggregate(X, rule, f=f)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_sgd_adam_oracles_match_torch():
    torch.manual_seed(5)
    p0 = torch.randn(100)
    grads = [torch.randn(100) for _ in range(3)]
    # SGD
    t = torch.nn.Parameter(p0.clone())
    o = torch.optim.SGD([t], lr=0.1, momentum=0.9, weight_decay=0.01, nesterov=True)
    p, b = p0.clone(), torch.zeros(100)
    for i, g in enumerate(grads):
        t.grad = g.clone()
        o.step()
        p, b = R.sgd_update(p, g, b, 0.1, 0.9, 0.01, True, first=i == 0)
    torch.testing.assert_close(p, t.detach(), rtol=1e-6, atol=1e-6)
    # AdamW
    t = torch.nn.Parameter(p0.clone())
    o = torch.optim.AdamW([t], lr=0.01, weight_decay=0.1)
    p, m, v = p0.clone(), torch.zeros(100), torch.zeros(100)
    for i, g in enumerate(grads):
        t.grad = g.clone()
        o.step()
        p, m, v = R.adam_update(p, g, m, v, i + 1, 0.01, 0.9, 0.999, 1e-8, 0.1, decoupled=True)
    torch.testing.assert_close(p, t.detach(), rtol=1e-6, atol=1e-6)


def test_bf16_key_roundtrip():
    """numpy model of common.h bf16_key / bf16_unkey over all 65536 bf16 bit patterns: the u16
    key order is the value order, NaN -> +inf, and decoding returns the (NaN -> +inf) value."""
    import numpy as np
    w = np.arange(65536, dtype=np.uint32)
    sgn = np.where(w & 0x8000, 0xFFFF, 0)
    key = np.minimum(((w ^ (sgn | 0x8000)) - 127) & 0xFFFF, 0xFF01)
    f = (w << 16).astype(np.uint32).view(np.float32)
    vals = np.where(np.isnan(f), np.inf, f)
    srt = vals[np.argsort(key, kind="stable")]
    assert np.all(srt[1:] >= srt[:-1])
    uk = (key + 127) & 0xFFFF
    s2 = np.where(uk & 0x8000, 0xFFFF, 0)
    back = (((uk ^ ((~s2) | 0x8000)) & 0xFFFF).astype(np.uint32) << 16).view(np.float32)
    assert np.array_equal(back, vals)
