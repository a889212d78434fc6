"""Dense NT GEMM with fused epilogues (csrc/kernels/gemm.hip) against fp32 PyTorch oracles:
y = x W^T (+ bias), the bias + GELU forward (h and gelu(h)), and the GELU backward with the
bias-gradient column sums (per row segment = per virtual worker)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rand(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return (torch.rand(*shape, generator=g, device=dev) * 2 - 1).mul_(scale).bfloat16()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 768), (1024, 3072, 768),
                                   (768, 512, 3072), (2048, 2304, 128)])
@pytest.mark.parametrize("tile", [256, 128])
def test_gemm_store_vs_fp32(cuda, M, N, K, tile):
    from consensusml_amd.ops.native import lib
    a, b = _rand(M, K, dev=cuda, seed=1), _rand(N, K, dev=cuda, seed=2)
    bias = _rand(N, dev=cuda, seed=3)
    ref = a.float() @ b.float().t()
    y = lib().gemm_nt(a, b, 0, tile=tile)
    assert _rel(y, ref) < 4e-3
    yb = lib().gemm_nt(a, b, 0, bias=bias, tile=tile)
    assert _rel(yb, ref + bias.float()) < 4e-3
    # exactness of the layout: integer-valued operands give exact fp32 sums (|sum| < 2^8 keeps
    # the bf16 output exact), so every element must match, not just the norm
    ai = torch.randint(-2, 3, (M, K), device=cuda).bfloat16()
    bi = torch.randint(-2, 3, (N, K), device=cuda).bfloat16()
    if K <= 64:
        yi = lib().gemm_nt(ai, bi, 0, tile=tile)
        assert torch.equal(yi.float(), ai.float() @ bi.float().t())


# 128 x 128 tiles (gemm128.hip): M and N multiples of 128 that are NOT multiples of 256, the
# BERT per-rank shapes, an asymmetric integer check of the C^T layout, bias + residual (cin)
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (384, 640, 192), (8192, 768, 768),
                                   (8192, 768, 3072), (1152, 2304, 704), (640, 128, 4096)])
def test_gemm128_vs_fp32(cuda, M, N, K):
    from consensusml_amd.ops.native import lib
    a, b = _rand(M, K, dev=cuda, seed=11), _rand(N, K, dev=cuda, seed=12)
    bias = _rand(N, dev=cuda, seed=13)
    cin = _rand(M, N, dev=cuda, seed=14, scale=4.0)
    ref = a.float() @ b.float().t()
    y = lib().gemm_nt(a, b, 0, bias=bias, tile=128)
    assert _rel(y, ref + bias.float()) < 4e-3
    # in-place residual add (out = cin): bf16(bf16(acc + bias) + cin), gemm.hip's rounding points
    yc = cin.clone()
    lib().gemm_nt(a, b, 0, bias=bias, out=yc, cin=yc, tile=128)
    want = (y.float() + cin.float()).bfloat16()
    assert (yc.float() - want.float()).abs().max().item() <= 2 ** -6 * want.float().abs().max().item()
    ai = torch.randint(-2, 3, (M, 64), device=cuda).bfloat16()
    bi = (torch.arange(N * 64, device=cuda).view(N, 64) % 5 - 2).bfloat16()   # asymmetric
    yi = lib().gemm_nt(ai, bi, 0, tile=128)
    assert torch.equal(yi.float(), ai.float() @ bi.float().t())


def test_gemm_pick():
    from consensusml_amd.ops.native import lib
    L = lib()
    assert L.gemm_nt_pick(8192, 768, 768) == 128          # 96 tiles of 256^2: under-filled
    assert L.gemm_nt_pick(8192, 28672, 4096) == 256       # Llama w13: 3584 tiles
    assert L.gemm_nt_pick(8192, 4096, 4096) == 256        # 512 tiles
    assert L.gemm_nt_pick(1000, 768, 768) == 0


def test_gemm_strided_rows(cuda):
    """Operands and output as column slices of wider rows (the fused QKV weights / outputs)."""
    from consensusml_amd.ops.native import lib
    M, N, K = 512, 256, 128
    A = _rand(M, 2 * K, dev=cuda, seed=4)
    B = _rand(N, K + 64, dev=cuda, seed=5)
    Y = torch.zeros(M, 3 * N, dtype=torch.bfloat16, device=cuda)
    a, b, y = A[:, K:], B[:, :K], Y[:, N:2 * N]
    lib().gemm_nt(a, b, 0, out=y)
    assert _rel(y, a.float() @ b.float().t()) < 4e-3
    assert float(Y[:, :N].abs().max()) == 0.0 and float(Y[:, 2 * N:].abs().max()) == 0.0


@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (1024, 3072, 768)])
def test_gemm_bias_gelu(cuda, M, N, K):
    from consensusml_amd.ops.native import lib
    a, b = _rand(M, K, dev=cuda, seed=6), _rand(N, K, dev=cuda, seed=7, scale=0.1)
    bias = _rand(N, dev=cuda, seed=8)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    y = lib().gemm_nt(a, b, 1, bias=bias, aux=h)
    href = a.float() @ b.float().t() + bias.float()
    assert _rel(h, href) < 4e-3
    # gelu from the kernel's own bf16 h: only the final rounding may differ
    torch.testing.assert_close(y.float(), F.gelu(h.float()).bfloat16().float(), rtol=8e-3, atol=1e-5)
    assert _rel(y, F.gelu(href)) < 6e-3


@pytest.mark.parametrize("nseg", [1, 4])
def test_gemm_dgelu_colsum(cuda, nseg):
    from consensusml_amd.ops.native import lib
    M, N, K = 1024, 3072, 768
    dy, w = _rand(M, K, dev=cuda, seed=9), _rand(N, K, dev=cuda, seed=10, scale=0.1)
    h = _rand(M, N, dev=cuda, seed=11, scale=3.0)
    cs = torch.empty(nseg, N, dtype=torch.float32, device=cuda)
    dh = lib().gemm_nt(dy, w, 2, aux=h, colsum_out=cs)
    g = (dy.float() @ w.float().t())
    hf = h.float().requires_grad_(True)
    F.gelu(hf).backward(g)
    ref = hf.grad
    assert _rel(dh, ref) < 6e-3
    # gelu' from the kernel's own bf16 g: elementwise agreement
    gb = lib().gemm_nt(dy, w, 0)
    hf2 = h.float().requires_grad_(True)
    F.gelu(hf2).backward(gb.float())
    torch.testing.assert_close(dh.float(), hf2.grad.bfloat16().float(), rtol=1.6e-2, atol=1e-4)
    seg = dh.float().view(nseg, M // nseg, N).sum(1)
    torch.testing.assert_close(cs, seg, rtol=1e-4, atol=1e-3)
    csb = torch.empty(nseg, N, dtype=torch.bfloat16, device=cuda)
    lib().gemm_nt(dy, w, 2, aux=h, colsum_out=csb)
    torch.testing.assert_close(csb.float(), seg, rtol=1e-2, atol=1e-2)


def test_gemm_deterministic(cuda):
    from consensusml_amd.ops.native import lib
    a, b = _rand(2048, 768, dev=cuda, seed=12), _rand(3072, 768, dev=cuda, seed=13)
    y1 = lib().gemm_nt(a, b, 0)
    y2 = lib().gemm_nt(a, b, 0)
    assert torch.equal(y1, y2)


def test_gemm_cin_inplace(cuda):
    """y = a b^T + cin written over cin (the parked residual gradient of a data gradient)."""
    from consensusml_amd.ops.native import lib
    a, b = _rand(512, 768, dev=cuda, seed=14), _rand(256, 768, dev=cuda, seed=15)
    c = _rand(512, 256, dev=cuda, seed=16)
    ref = a.float() @ b.float().t() + c.float()
    y = lib().gemm_nt(a, b, 0, out=c, cin=c)
    assert y.data_ptr() == c.data_ptr()
    assert _rel(c, ref) < 4e-3


@pytest.mark.parametrize("R,C", [(768, 3072), (2304, 768), (64, 64), (256, 1024)])
def test_transpose_bf16(cuda, R, C):
    from consensusml_amd.ops.native import lib
    w = _rand(R, C, dev=cuda, seed=9)
    assert torch.equal(lib().transpose_bf16(w), w.t().contiguous())
    big = _rand(R, C + 64, dev=cuda, seed=10)
    v = big[:, 64:]
    assert torch.equal(lib().transpose_bf16(v), v.t().contiguous())
    odd = _rand(R, 40, dev=cuda, seed=11)   # not a 64-multiple: ATen fallback
    assert torch.equal(lib().transpose_bf16(odd), odd.t().contiguous())
