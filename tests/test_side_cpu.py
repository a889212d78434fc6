"""ops.side bookkeeping without a GPU: unarmed (or CPU) runs are inline, arm() needs the policy
and a CUDA device, disarm() clears the state."""
import torch

from consensusml_amd import perf
from consensusml_amd.ops import side


def test_side_inline_when_unarmed():
    side.disarm()
    x = torch.randn(4, 4)
    out = side.run(lambda: x * 2, x)
    assert torch.equal(out, x * 2)
    assert side._S.used is False


def test_side_arm_needs_cuda_and_policy():
    with perf.use_policy(perf.policy().replace(side_wgrad=True)):
        side.arm(torch.device("cpu"))
        assert side._S.armed is None
    with perf.use_policy(perf.policy().replace(side_wgrad=False)):
        side.arm(torch.device("cuda", 0))
        assert side._S.armed is None
    side.disarm()
    assert side._S.armed is None and side._S.used is False
