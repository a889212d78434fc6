"""CPU checks of the host-side bookkeeping behind the folded batch-256 launches (ops/conv.py):
the BN affine parked on a statistics tensor by its finalize, and the per-forward weight-layout
prefetch (GPU-only: a no-op for CPU weights)."""
import torch

from consensusml_amd import perf
from consensusml_amd.ops import conv as C


class _BN:
    def __init__(self, dtype):
        self.weight = torch.ones(8, dtype=dtype)
        self.bias = torch.zeros(8, dtype=dtype)


def test_cached_affine_valid_until_parameters_change():
    g = torch.rand(8).bfloat16()
    b = torch.rand(8).bfloat16()
    mean, sc, bi = torch.rand(8), torch.rand(8), torch.rand(8)
    C._stash_affine(mean, sc, bi, (g, b))
    got = C._cached_affine(g, b, mean)
    assert got is not None and got[0] is sc and got[1] is bi
    assert C._affine(g, b, mean, torch.rand(8))[0] is sc   # no recompute
    assert C._cached_affine(g.clone(), b, mean) is None    # another tensor
    with torch.no_grad():
        g.mul_(2)                                           # optimizer-style in-place update
    assert C._cached_affine(g, b, mean) is None
    assert C._cached_affine(g, b, torch.rand(8)) is None    # nothing parked


def test_fin_aff_policy_and_dtypes():
    with perf.use_policy(perf.policy().replace(fin_affine=True)):
        assert C._fin_aff(_BN(torch.bfloat16)) is not None
        assert C._fin_aff(_BN(torch.float32)) is None
    with perf.use_policy(perf.policy().replace(fin_affine=False)):
        assert C._fin_aff(_BN(torch.bfloat16)) is None


def test_own_dgb_policy():
    g, b = torch.ones(4).bfloat16(), torch.zeros(4).bfloat16()
    with perf.use_policy(perf.policy().replace(fin_dgamma=True)):
        assert C._own_dgb(g, b) and not C._own_dgb(g.float(), b)
    with perf.use_policy(perf.policy().replace(fin_dgamma=False)):
        assert not C._own_dgb(g, b)


def test_prefetch_is_gpu_only():
    ws = [torch.randn(8, 8, 3, 3).bfloat16(), torch.randn(8, 8, 1, 1).bfloat16()]
    assert C.prefetch_wlayouts(ws) is False
    assert not C._WL_BATCH and C.cached_wt(ws[1]) is None
    wf, wr = C._w3x3_layouts(ws[0].float(), True)   # the CPU reference layouts
    assert wf.shape == (8, 72) and wr.shape == (8, 72)
