"""4-wave 256 x 256-tile GEMM (csrc/kernels/gemm_w4.hip) in all four operand layouts against fp32
PyTorch oracles: y = A B^T with A [M, K] or [K, M] and B [N, K] or [K, N] -- the forward (mode 0),
data-gradient (mode 2) and weight-gradient (mode 3) products of a linear layer read in place --
at whole-tile and ragged M / N, with bias and the in-place residual add (cin), plus exact
integer checks with asymmetric operands that pin every element's placement."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).mul_(scale).bfloat16()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _ops(mode, A, B):
    """A [M, K], B [N, K] -> the stored operands of `mode`."""
    a = A.t().contiguous() if mode & 1 else A
    b = B.t().contiguous() if mode & 2 else B
    return a, b


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 128), (1024, 512, 768),
                                   (296, 520, 192), (8, 264, 64), (1000, 1016, 320),
                                   (2048, 256, 4096)])
def test_gemm_w4_vs_fp32(cuda, mode, M, N, K):
    from consensusml_amd.ops.native import lib
    A, B = _rand(M, K, dev=cuda, seed=1), _rand(N, K, dev=cuda, seed=2)
    a, b = _ops(mode, A, B)
    ref = A.float() @ B.float().t()
    y = lib().gemm_w4(a, b, mode)
    assert y.shape == (M, N)
    assert _rel(y, ref) < 4e-3
    bias = _rand(N, dev=cuda, seed=3)
    yb = lib().gemm_w4(a, b, mode, bias=bias)
    assert _rel(yb, ref + bias.float()) < 4e-3
    # in-place residual add: bf16(bf16(acc + bias) + cin)
    cin = _rand(M, N, dev=cuda, seed=4, scale=4.0)
    yc = cin.clone()
    lib().gemm_w4(a, b, mode, out=yc, bias=bias, cin=yc)
    want = (yb.float() + cin.float()).bfloat16()
    assert (yc.float() - want.float()).abs().max().item() <= 2 ** -6 * want.float().abs().max().item()


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N", [(256, 256), (520, 776), (1024, 264)])
def test_gemm_w4_exact_layout(cuda, mode, M, N):
    """Integer operands (|sum| < 2^8: exact fp32 sums, exact bf16 outputs), asymmetric in both
    row and column index, so a swapped or shifted element anywhere fails."""
    from consensusml_amd.ops.native import lib
    K = 128
    A = ((torch.arange(M * K, device=cuda).view(M, K) * 7 + torch.arange(M, device=cuda)[:, None])
         % 5 - 2).bfloat16()
    B = ((torch.arange(N * K, device=cuda).view(N, K) * 3 + 2 * torch.arange(N, device=cuda)[:, None])
         % 3 - 1).bfloat16()
    a, b = _ops(mode, A, B)
    y = lib().gemm_w4(a, b, mode)
    assert torch.equal(y.float(), A.float() @ B.float().t())


def test_gemm_w4_strided_out_and_rows(cuda):
    """Row-strided operands / output (views into wider buffers): lda, ldb, ldy > the logical width."""
    from consensusml_amd.ops.native import lib
    M, N, K = 512, 384, 256
    Abig, Bbig = _rand(M, K + 64, dev=cuda, seed=5), _rand(N, K + 128, dev=cuda, seed=6)
    A, B = Abig[:, :K], Bbig[:, :K]
    out = torch.zeros(M, N + 64, dtype=torch.bfloat16, device=cuda)
    lib().gemm_w4(A, B, 0, out=out[:, :N])
    assert _rel(out[:, :N], A.float() @ B.float().t()) < 4e-3
    assert torch.count_nonzero(out[:, N:]) == 0
    # weight-gradient layout with row-strided k-major operands
    dyb, xb = _rand(K, M + 32, dev=cuda, seed=7), _rand(K, N + 16, dev=cuda, seed=8)
    dy, x = dyb[:, :M], xb[:, :N]
    dw = lib().gemm_w4(dy, x, 3)
    assert _rel(dw, dy.float().t() @ x.float()) < 4e-3


def test_gemm_w4_llama_shapes(cuda):
    """The three products of a Llama-3-8B projection at a reduced token count (M = 1024)."""
    from consensusml_amd.ops.native import lib
    M, N, K = 1024, 6144, 4096
    x, w, dy = _rand(M, K, dev=cuda, seed=9), _rand(N, K, dev=cuda, seed=10), _rand(M, N, dev=cuda, seed=11)
    assert _rel(lib().gemm_w4(x, w, 0), x.float() @ w.float().t()) < 4e-3
    assert _rel(lib().gemm_w4(dy, w, 2), dy.float() @ w.float()) < 4e-3
    assert _rel(lib().gemm_w4(dy, x, 3), dy.float().t() @ x.float()) < 4e-3


def test_gemm_w4_rejects_bad_shapes(cuda):
    from consensusml_amd.ops.native import lib
    a = _rand(256, 96, dev=cuda)
    with pytest.raises(RuntimeError):
        lib().gemm_w4(a, _rand(256, 96, dev=cuda), 0)        # K % 64
    with pytest.raises(RuntimeError):
        lib().gemm_w4(_rand(100, 128, dev=cuda), _rand(256, 128, dev=cuda), 0)   # M % 8
