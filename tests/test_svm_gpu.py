"""Batched SMO kernel (csrc/kernels/svm_smo.hip) against the host oracle ``svm.smo`` and libsvm
(sklearn.svm.SVC, which wraps it)."""
import numpy as np
import pytest
import torch

from consensusml_amd.select.svm import SVC, fit_svcs, kernel_matrix, smo, smo_batched

pytestmark = pytest.mark.gpu


def _problem(n, p, seed, sep=1.0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, p, generator=g, dtype=torch.float64)
    y = (X[:, 0] + 0.5 * X[:, 1] + sep * torch.randn(n, generator=g, dtype=torch.float64) > 0).long()
    return X, y


@pytest.mark.parametrize("kind", ["linear", "radial"])
def test_smo_kernel_matches_host_oracle(cuda, kind):
    Ks, ys, Cs, ref = [], [], [], []
    for b, (n, p) in enumerate([(40, 10), (97, 300), (145, 1984), (64, 5), (300, 50)]):
        X, y = _problem(n, p, b)
        X = (X - X.mean(0)) / X.std(0)
        K = kernel_matrix(X, X, kind, 1.0 / p)
        yy = torch.where(y > 0, 1.0, -1.0).double()
        C = [1.0, 0.5, 2.0, 10.0, 1.0][b]
        Ks.append(K.to(cuda))
        ys.append(yy.to(cuda))
        Cs.append(C)
        a, G = smo(K.numpy(), yy.numpy(), C, 1e-8, return_grad=True)
        ref.append(a)
    out = smo_batched(Ks, ys, Cs, 1e-8)
    for (a, b_, it), a_ref, K, yy, C in zip(out, ref, Ks, ys, Cs):
        # the dual optimum can be non-unique (rank-deficient K): compare the objective and the
        # decision values on the training points, which are unique
        assert it > 0
        Kc, y_ = K.cpu().numpy(), yy.cpu().numpy()
        Q = Kc * np.outer(y_, y_)
        obj = lambda v: 0.5 * v @ Q @ v - v.sum()
        a = a.cpu().numpy()
        assert abs(obj(a) - obj(a_ref)) <= 1e-7 * max(1.0, abs(obj(a_ref)))
        np.testing.assert_allclose(Kc @ (a * y_), Kc @ (a_ref * y_), atol=1e-5, rtol=1e-6)
        assert abs(float((a * y_).sum())) < 1e-8 and a.min() >= 0 and a.max() <= C


def test_svc_gpu_matches_libsvm(cuda):
    from sklearn.svm import SVC as SK
    X, y = _problem(120, 60, 7, sep=0.7)
    for kern in ("linear", "radial"):
        m = SVC(kern, tol=1e-6).fit(X.to(cuda), y.to(cuda))
        Xs = ((X - X.mean(0)) / X.std(0)).numpy()
        sk = SK(kernel="linear" if kern == "linear" else "rbf", C=1.0, gamma=1.0 / X.shape[1],
                tol=1e-6).fit(Xs, y.numpy())
        d_ours = m.decision_function(X.to(cuda)).cpu().numpy()
        d_sk = sk.decision_function(Xs)
        np.testing.assert_allclose(d_ours, d_sk, atol=1e-4, rtol=1e-4)
        if kern == "linear":
            np.testing.assert_allclose(m.weights.cpu().numpy(), sk.coef_[0], atol=1e-4, rtol=1e-4)


def test_fit_svcs_batched_equals_single(cuda):
    Xs, ys = [], []
    for s in range(6):
        X, y = _problem(80 + 7 * s, 40, 20 + s)
        Xs.append(X.to(cuda))
        ys.append(y.to(cuda))
    many = fit_svcs(Xs, ys, "radial", C=[0.25, 0.5, 1, 2, 4, 8])
    for m, X, y, C in zip(many, Xs, ys, [0.25, 0.5, 1, 2, 4, 8]):
        one = SVC("radial", C=C).fit(X, y)
        torch.testing.assert_close(m.decision_function(X), one.decision_function(X))
