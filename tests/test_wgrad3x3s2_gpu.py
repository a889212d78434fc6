"""Stride-2 3x3 weight gradient (wgrad3x3s2.hip: nine taps per workgroup from the raw input rows
of each output-row chunk) against fp32 autograd: the ResNet-50 downsample shapes at small batch,
non-square and odd output sizes (chunks of several rows, one row), a partial last k-step, and
the model op (_Conv3x3S2BNStatsFn) end to end."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _lib():
    from consensusml_amd.ops.native import lib
    return lib()


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


# (images, Ci, Co, Ho, Wo): input 2 Ho x 2 Wo
SHAPES = [(4, 128, 128, 28, 28), (6, 256, 256, 14, 14), (8, 512, 512, 7, 7),
          (3, 64, 128, 5, 9), (2, 128, 64, 12, 20)]


def _ref(dy, x, Co):
    xr = x.float().requires_grad_(True)
    wr = torch.zeros(Co, x.shape[1], 3, 3, device=x.device, requires_grad=True)
    y = F.conv2d(xr, wr, stride=2, padding=1)
    y.backward(dy.float())
    return wr.grad


@pytest.mark.parametrize("N,Ci,Co,Ho,Wo", SHAPES)
def test_wgrad3x3_s2_vs_fp32(cuda, N, Ci, Co, Ho, Wo):
    g0 = torch.Generator(device=cuda).manual_seed(51)
    x = _nhwc(torch.randn(N, Ci, 2 * Ho, 2 * Wo, device=cuda, generator=g0).bfloat16())
    dy = _nhwc(torch.randn(N, Co, Ho, Wo, device=cuda, generator=g0).bfloat16())
    assert _lib().wgrad3x3_s2_ok(N, Ho, Wo, Co, Ci)
    dw = _lib().wgrad3x3_s2(dy, x, torch.float32)
    ref = _ref(dy, x, Co)
    assert dw.shape == ref.shape
    assert _rel(dw, ref) < 1e-3
    # every tap (the border taps read the zero row / column) as close as the centre one
    err = (dw - ref).abs().amax((0, 1))
    assert float(err.max()) < 4 * float(err[1, 1]) + 1e-3
    dwb = _lib().wgrad3x3_s2(dy, x, torch.bfloat16)
    assert dwb.dtype == torch.bfloat16 and _rel(dwb, ref) < 5e-3


def test_wgrad3x3_s2_deterministic(cuda):
    g0 = torch.Generator(device=cuda).manual_seed(52)
    x = _nhwc(torch.randn(16, 128, 56, 56, device=cuda, generator=g0).bfloat16())
    dy = _nhwc(torch.randn(16, 128, 28, 28, device=cuda, generator=g0).bfloat16())
    a = _lib().wgrad3x3_s2(dy, x, torch.float32)
    b = _lib().wgrad3x3_s2(dy, x, torch.float32)
    assert torch.equal(a, b)


def test_wgrad3x3_s2_through_model_op(cuda):
    """conv3x3_s2 forward + backward (parity-class data gradient, this weight gradient) vs fp32
    autograd."""
    from consensusml_amd.ops import conv as fconv
    g0 = torch.Generator(device=cuda).manual_seed(53)
    x = _nhwc((torch.randn(4, 128, 56, 56, device=cuda, generator=g0) + 0.2).bfloat16())
    w = (torch.randn(128, 128, 3, 3, device=cuda, generator=g0) * 1152 ** -0.5).bfloat16()
    conv = torch.nn.Conv2d(128, 128, 3, stride=2, padding=1, bias=False).to(cuda, torch.bfloat16)
    bn = torch.nn.BatchNorm2d(128).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(w)
    assert fconv.conv3x3_s2_ok(x, conv)
    xi = x.clone().requires_grad_(True)
    z, _ = fconv.conv3x3_s2_bn_stats(xi, conv, bn)
    gy = _nhwc(torch.randn(z.shape, device=cuda, generator=g0).bfloat16())
    z.backward(gy)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    F.conv2d(xr, wr, stride=2, padding=1).backward(gy.float())
    assert _rel(xi.grad, xr.grad) < 5e-3
    assert _rel(conv.weight.grad, wr.grad) < 1e-2
