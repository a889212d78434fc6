"""agg_update_multi (one launch over the sharded engine's buckets) == one agg_update per bucket,
bit for bit, for the weighted (Krum / mean) and sorted (median / trimmed mean / Bulyan rows)
combines with SGD-momentum and AdamW, including a ragged segment (per-segment fallback)."""
import pytest
import torch

from consensusml_amd.ops import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("combine,opt_kind", [("weighted", "sgd"), ("weighted", "adamw"),
                                              ("sorted", "sgd"), ("sorted", "adamw")])
@pytest.mark.parametrize("ragged", [False, True])
def test_multi_equals_per_bucket(cuda, combine, opt_kind, ragged):
    torch.manual_seed(0)
    n = 8
    lens = [4096, 12288, 808 if ragged else 800, 20000]
    offs = [0]
    for L in lens[:-1]:
        offs.append(offs[-1] + L)
    total = sum(lens)
    Xs = [torch.randn(n, L, device=cuda).bfloat16() for L in lens]
    w = torch.rand(n, device=cuda)
    w[3] = 0.0
    opt = K.OptArgs(kind=opt_kind, lr=0.05, momentum=0.9 if opt_kind == "sgd" else 0.0,
                    weight_decay=1e-3, step=3)
    kw = dict(combine=combine, n=n) if combine == "weighted" else \
        dict(combine=combine, n=n, lo=2, cnt=4)
    if combine == "weighted":
        kw["w"] = w

    def state():
        g = torch.Generator(device=cuda).manual_seed(1)
        m, a, b = (torch.randn(total, device=cuda, generator=g) for _ in range(3))
        return m, a, b.abs()          # Adam's second moment is non-negative

    m1, a1, b1 = state()
    p1 = [torch.zeros(L, device=cuda, dtype=torch.bfloat16) for L in lens]
    for X, L, o, p in zip(Xs, lens, offs, p1):
        K.agg_update(X, D=L, opt=opt, master=m1[o:o + L], s1=a1[o:o + L],
                     s2=b1[o:o + L] if opt_kind == "adamw" else None, param_out=p, **kw)
    m2, a2, b2 = state()
    p2 = [torch.zeros(L, device=cuda, dtype=torch.bfloat16) for L in lens]
    K.agg_update_multi(list(zip(Xs, lens, offs, p2)), opt=opt, master=m2, s1=a2,
                       s2=b2 if opt_kind == "adamw" else None, **kw)
    assert torch.equal(m1, m2) and torch.equal(a1, a2)
    if opt_kind == "adamw":
        assert torch.equal(b1, b2)
    for x, y in zip(p1, p2):
        assert torch.equal(x, y)
