"""conv3x3_wlayouts (csrc/kernels/conv_gemm.hip): the implicit-GEMM forward and data-gradient
layouts of a 3x3 weight in one launch, bit-identical to the PyTorch permute / flip copies it
replaces, for contiguous and channels_last weights."""
import pytest
import torch

from consensusml_amd.ops.native import lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Co,Ci", [(64, 64), (128, 64), (256, 512), (3, 5)])
@pytest.mark.parametrize("cl", [False, True])
def test_conv3x3_wlayouts_exact(cuda, Co, Ci, cl):
    w = torch.randn(Co, Ci, 3, 3, device=cuda).to(torch.bfloat16)
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    wf, wr = lib().conv3x3_wlayouts(w, True)
    assert torch.equal(wf, w.permute(0, 2, 3, 1).reshape(Co, 9 * Ci))
    assert torch.equal(wr, w.flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co))
    none, wr2 = lib().conv3x3_wlayouts(w, False)
    assert none is None and torch.equal(wr2, wr)
