"""ResNet global average pool with an NHWC backward (models/resnet.py:_GlobalAvgPoolFn): the value
and the gradient must equal F.adaptive_avg_pool2d's bit for bit, and the gradient must already be
channels_last (so the following BN backward never re-lays it out)."""
import pytest
import torch
import torch.nn.functional as F

from consensusml_amd.models.resnet import _GlobalAvgPoolFn


def _check(dev):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(6, 40, 7, 7, generator=g, device=dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    dy = torch.randn(6, 40, generator=g, device=dev).to(torch.bfloat16)
    a = x.clone().requires_grad_(True)
    b = x.clone().requires_grad_(True)
    ya = _GlobalAvgPoolFn.apply(a)
    yb = torch.flatten(F.adaptive_avg_pool2d(b, 1), 1)
    assert torch.equal(ya, yb)
    ya.backward(dy)
    yb.backward(dy)
    assert a.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(a.grad, b.grad, rtol=0, atol=0)


def test_global_avg_pool_cpu():
    _check(torch.device("cpu"))


@pytest.mark.gpu
def test_global_avg_pool_gpu(cuda):
    _check(cuda)
