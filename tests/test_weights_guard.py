"""The weights launch's centered-pass guard and fused tail (weights.hip), CPU reference path:
selection counts, next Gram center, and the captured-center refusal."""
import torch

from consensusml_amd.ops import kernels as K
from consensusml_amd.ops import reference as ref


def _gram(X):
    X = X.double()
    return X @ X.T


def test_fused_tail_counts_and_center():
    torch.manual_seed(0)
    X = torch.randn(8, 64)
    X[5] += 40.0                                   # an outlier
    G = _gram(X)
    cnt = torch.zeros(8, dtype=torch.float64)
    c = torch.zeros(1, dtype=torch.int32)
    w = K.robust_weights(G, "multi_krum", 8, f=2, m=4, sel_counts=cnt, center_out=c)
    assert int((w > 0).sum()) == 4 and float(w[5]) == 0.0
    assert torch.equal(cnt, (w > 0).double())
    assert int(c) == ref.gram_center(G)


def test_guard_refuses_majority_nonfinite():
    torch.manual_seed(1)
    G = _gram(torch.randn(8, 32))
    # a centered G whose honest rows overflowed: every diagonal but the center's is inf
    Gc = torch.full((8, 8), float("inf"), dtype=torch.float64)
    Gc[3, 3] = 0.0
    c = torch.zeros(1, dtype=torch.int32)
    cnt = torch.zeros(8, dtype=torch.float64)
    w = K.robust_weights(Gc, "krum", 8, f=2, guard=True, center_out=c, sel_counts=cnt)
    assert float(w.abs().sum()) == 0.0 and int(c) == -1 and float(cnt.sum()) == 0.0
    # without the guard (a two-pass G) the same matrix is not refused
    w2 = K.robust_weights(Gc, "krum", 8, f=2, guard=False)
    assert float(w2.sum()) > 0
    # a minority of non-finite rows (ordinary Byzantine NaN workers) passes the guard
    G[1, :] = float("nan")
    G[:, 1] = float("nan")
    w3 = K.robust_weights(G, "krum", 8, f=2, guard=True, center_out=c)
    assert float(w3.sum()) > 0 and float(w3[1]) == 0.0 and int(c) != -1


def test_centered_clip_guard_keeps_previous_aggregate():
    Gc = torch.full((9, 9), float("inf"), dtype=torch.float64)
    Gc[8, 8] = 1.0
    Gc[2, 2] = 0.0
    w = K.robust_weights(Gc, "centered_clip", 8, guard=True)
    assert float(w[8]) == 1.0 and float(w[:8].abs().sum()) == 0.0


def test_negative_center_is_uncentered():
    torch.manual_seed(2)
    X = torch.randn(4, 40)
    G0 = K.gram(X, n=4)
    G1 = K.gram(X, n=4, center=torch.tensor([-1], dtype=torch.int32))
    torch.testing.assert_close(G0, G1)


def test_gram_sum_bucket_order():
    Gb = torch.randn(5, 3, 3, dtype=torch.float64)
    out = torch.empty(3, 3, dtype=torch.float64)
    K.gram_sum(Gb, out)
    want = Gb[0].clone()
    for k in range(1, 5):
        want += Gb[k]
    assert torch.equal(out, want)


import pytest  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize("rule", ["krum", "multi_krum", "geomed", "centered_clip"])
def test_fused_tail_gpu_matches_reference(rule):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.manual_seed(3)
    n = 8
    dim = n + 1 if rule == "centered_clip" else n
    X = torch.randn(dim, 96)
    X[6] *= 30
    G = _gram(X)
    for Gi, guard in ((G, True), (G, False)):
        outs = []
        for dev in ("cpu", "cuda"):
            Gd = Gi.to(dev)
            c = torch.zeros(1, dtype=torch.int32, device=dev)
            cnt = torch.ones(n, dtype=torch.float64, device=dev)
            w = K.robust_weights(Gd, rule, n, f=2, m=5, guard=guard, center_out=c, sel_counts=cnt)
            outs.append((w.cpu(), int(c), cnt.cpu()))
        (wc, cc, nc), (wg, cg, ng) = outs
        torch.testing.assert_close(wg, wc, rtol=1e-5, atol=1e-6)
        assert cc == cg and torch.equal(nc, ng)
    Gc = torch.full((dim, dim), float("inf"), dtype=torch.float64)
    Gc[0, 0] = 0.0
    c = torch.zeros(1, dtype=torch.int32, device="cuda")
    w = K.robust_weights(Gc.cuda(), rule, n, f=2, guard=True, center_out=c)
    assert int(c) == -1 and float(w[:n].abs().sum()) == 0.0


@pytest.mark.gpu
def test_gram_sum_and_negative_center_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    Gb = torch.randn(8, 9, 9, dtype=torch.float64, device="cuda")
    out = torch.empty(9, 9, dtype=torch.float64, device="cuda")
    K.gram_sum(Gb, out)
    want = Gb[0].clone()
    for k in range(1, 8):
        want += Gb[k]
    assert torch.equal(out, want)
    X = torch.randn(6, 4000, device="cuda").bfloat16()
    G0 = K.gram(X, n=6)
    G1 = K.gram(X, n=6, center=torch.tensor([-1], dtype=torch.int32, device="cuda"))
    assert torch.equal(G0, G1)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3, 8, 20])
def test_gram_deferred_multi_reduce_bitwise(n):
    """Per-bucket stage-1 partials + ONE multi-bucket reduce == one gram() per bucket into slots
    summed in bucket order (the engine's early-Gram path), bit for bit; centered and not."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from consensusml_amd.ops.native import lib
    torch.manual_seed(n)
    lens = [4096, 70000, 1024, 333333 // 8 * 8]
    Xs = [torch.randn(n, L, device="cuda").bfloat16() for L in lens]
    for center in (None, torch.tensor([n // 2], dtype=torch.int32, device="cuda")):
        slots = torch.zeros(len(lens), n, n, dtype=torch.float64, device="cuda")
        for i, X in enumerate(Xs):
            K.gram(X, n=n, out=slots[i], center=center)
        want = torch.empty(n, n, dtype=torch.float64, device="cuda")
        K.gram_sum(slots, want)
        works, nblks = [], []
        for X in Xs:
            ws = torch.empty(int(lib().gram_workspace_bytes(n, X.shape[1])) // 4 + 1,
                             dtype=torch.float32, device="cuda")
            nblks.append(lib().gram_partial(X, n, X.shape[1], ws, center))
            works.append(ws)
        got = torch.empty(n, n, dtype=torch.float64, device="cuda")
        lib().gram_reduce_multi(works, nblks, n, got)
        assert torch.equal(got, want)


def test_guard_disarmed_after_trip_half_nan():
    """n = 2 with one genuinely NaN worker (geomed): half the rows non-finite on EVERY pass. With
    the engine's 2-element center state the guard trips only when rows TURN non-finite, so the
    finite worker keeps getting the weight step after step instead of training freezing
    (ADVICE r05); a 1-element center still disarms the guard on the uncentered pass after a trip."""
    torch.manual_seed(3)
    X = torch.randn(2, 16).double()
    X[1] = float("nan")
    G = X @ X.T
    c = torch.tensor([0, 1], dtype=torch.int32)     # centered on worker 0, 1 bad row last pass
    for _ in range(3):
        w = K.robust_weights(G, "geomed", 2, guard=True, center_out=c)
        assert float(w[0]) > 0.0 and float(w[1]) == 0.0
        assert int(c[0]) == 0 and int(c[1]) == 1
    # rows turning non-finite on a centered pass (a captured center) still trip
    c = torch.tensor([0, 0], dtype=torch.int32)
    w = K.robust_weights(G, "geomed", 2, guard=True, center_out=c)
    assert float(w.abs().sum()) == 0.0 and int(c[0]) == -1
    w = K.robust_weights(G, "geomed", 2, guard=True, center_out=c)   # uncentered pass: disarmed
    assert float(w[0]) > 0.0
    c1 = torch.zeros(1, dtype=torch.int32)
    K.robust_weights(G, "geomed", 2, guard=True, center_out=c1)
    assert int(c1) == -1
    w = K.robust_weights(G, "geomed", 2, guard=True, center_out=c1)
    assert float(w[0]) > 0.0
