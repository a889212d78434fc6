"""CPU-side pieces of the fused stem (ops/stem.py): weight packing and the fallback gate."""
import torch
import torch.nn as nn

from consensusml_amd.ops.bn import BatchNormAct2d
from consensusml_amd.ops.stem import pack_stem_weight, stem_ok


def test_stem_pack_layout():
    """[64, C, 7, 7] -> [64, 224] with k = (ky * 8 + kx) * 4 + c, zero tap kx = 7 and channel 3."""
    w = torch.arange(64 * 3 * 49, dtype=torch.float32).reshape(64, 3, 7, 7)
    p = pack_stem_weight(w.to(torch.bfloat16)).float().view(64, 7, 8, 4)
    assert torch.equal(p[:, :, :7, :3], w.to(torch.bfloat16).float().permute(0, 2, 3, 1))
    assert p[:, :, 7].abs().sum() == 0 and p[..., 3].abs().sum() == 0


def test_stem_gate_cpu_and_shapes():
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(torch.bfloat16)
    bn = BatchNormAct2d(64, relu=True).to(torch.bfloat16)
    x = torch.randn(2, 3, 32, 32).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert not stem_ok(x, conv, bn)                      # CPU tensors take the module path
    narrow = nn.Conv2d(3, 8, 7, 2, 3, bias=False)        # resnet_tiny's stem: not 64 channels
    assert not stem_ok(x, narrow, BatchNormAct2d(8, relu=True))
