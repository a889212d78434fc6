"""CPU checks of the small weight-preparation helpers of ops/conv.py that run inside the fused
ResNet blocks' forward (no GPU needed: plain PyTorch ops)."""
import pytest
import torch

from consensusml_amd.ops.conv import scaled_cat


@pytest.mark.parametrize("Co,K1,K2", [(256, 64, 64), (512, 128, 256), (7, 5, 3)])
def test_scaled_cat_bit_identical(Co, K1, K2):
    """The down-sample tail's BN-folded weights [diag(sc3) W3 | diag(scd) Wd] in two launches are
    bit-identical to the six-op form they replace (fp32 products, one bf16 rounding)."""
    g = torch.Generator().manual_seed(Co + K1)
    w1 = torch.randn(Co, K1, generator=g).bfloat16()
    w2 = torch.randn(Co, K2, generator=g).bfloat16()
    s1 = torch.rand(Co, generator=g) * 3
    s2 = torch.randn(Co, generator=g)
    ref = torch.cat([w1.float() * s1[:, None], w2.float() * s2[:, None]], 1).to(torch.bfloat16)
    out = scaled_cat(w1, s1, w2, s2)
    assert out.dtype == torch.bfloat16 and out.is_contiguous()
    assert torch.equal(out, ref)
