"""consensusml_amd.optim: fused optimizers over flat buffers against torch.optim (CPU oracle path
here, the HIP kernel under @gpu)."""
import copy

import pytest
import torch

from consensusml_amd.optim import FusedAdam, FusedAdamW, FusedSGD


def _model(dtype=torch.float32, device="cpu"):
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(),
                            torch.nn.AdaptiveAvgPool2d(1), torch.nn.Flatten(),
                            torch.nn.Linear(8, 5))
    return m.to(device=device, dtype=dtype, memory_format=torch.channels_last)


def _mlp(dtype=torch.float32, device="cpu"):
    """GPU tests: Linear layers only (deterministic kernels, unlike conv weight gradients)."""
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Flatten(), torch.nn.Linear(192, 64), torch.nn.GELU(),
                               torch.nn.Linear(64, 5)).to(device=device, dtype=dtype)


def _batches(k, device="cpu", dtype=torch.float32):
    g = torch.Generator().manual_seed(1)
    return [(torch.randn(6, 3, 8, 8, generator=g).to(device, dtype)
             .contiguous(memory_format=torch.channels_last),
             torch.randint(0, 5, (6,), generator=g).to(device)) for _ in range(k)]


CASES = [
    (FusedSGD, torch.optim.SGD, dict(lr=0.1)),
    (FusedSGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-2)),
    (FusedSGD, torch.optim.SGD, dict(lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-3)),
    (FusedAdamW, torch.optim.AdamW, dict(lr=1e-2, weight_decay=0.05)),
    (FusedAdam, torch.optim.Adam, dict(lr=1e-2, weight_decay=0.05)),
    (FusedAdam, torch.optim.Adam, dict(lr=1e-2, betas=(0.8, 0.99), eps=1e-6)),
]


def _train(model, opt, batches, grad_scale=1.0):
    for x, y in batches:
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x).float(), y)
        (loss * grad_scale).backward()
        if grad_scale != 1.0 and not hasattr(opt, "flat_buffers"):
            for p in model.parameters():
                p.grad.div_(grad_scale)
        if hasattr(opt, "flat_buffers"):
            opt.step(grad_scale=1.0 / grad_scale)
        else:
            opt.step()


@pytest.mark.parametrize("fused_cls,torch_cls,kw", CASES)
def test_matches_torch_optim(fused_cls, torch_cls, kw):
    a = _model()
    b = copy.deepcopy(a)
    oa = fused_cls(a.parameters(), **kw)
    ob = torch_cls(b.parameters(), **kw)
    bs = _batches(5)
    _train(a, oa, bs)
    _train(b, ob, bs)
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_flat_views_and_channels_last():
    m = _model()
    opt = FusedSGD(m.parameters(), lr=0.1)
    (fl,) = opt.flat_buffers()
    conv = m[0].weight
    assert conv.is_contiguous(memory_format=torch.channels_last)
    assert conv.grad.is_contiguous(memory_format=torch.channels_last)
    lo = fl.param.data_ptr()
    hi = lo + fl.param.numel() * fl.param.element_size()
    for p in m.parameters():
        assert lo <= p.data_ptr() < hi
    x, y = _batches(1)[0]
    torch.nn.functional.cross_entropy(m(x), y).backward()
    assert fl.grad.abs().sum() > 0          # autograd accumulated into the flat gradient
    opt.zero_grad()
    assert fl.grad.abs().sum() == 0 and m[0].weight.grad is not None


def test_param_groups_and_grad_scale():
    a = _model()
    b = copy.deepcopy(a)
    ga = [{"params": a[0].parameters(), "lr": 0.01}, {"params": a[4].parameters()}]
    gb = [{"params": b[0].parameters(), "lr": 0.01}, {"params": b[4].parameters()}]
    oa = FusedSGD(ga, lr=0.1, momentum=0.9)
    ob = torch.optim.SGD(gb, lr=0.1, momentum=0.9)
    bs = _batches(4)
    _train(a, oa, bs, grad_scale=1024.0)
    _train(b, ob, bs, grad_scale=1024.0)
    assert len(oa.flat_buffers()) == 2
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_foreign_grad_assignment():
    m = _model()
    opt = FusedSGD(m.parameters(), lr=0.5)
    w = m[4].weight
    before = w.detach().clone()
    opt.zero_grad()
    w.grad = torch.ones_like(w)             # replaces the flat view
    opt.step()
    torch.testing.assert_close(w.detach(), before - 0.5)


@pytest.mark.parametrize("fused_cls,torch_cls,kw", [CASES[1], CASES[3]])
def test_state_dict_interop(fused_cls, torch_cls, kw):
    """torch.optim state dict -> fused optimizer and back, then identical continuation."""
    a = _model()
    b = copy.deepcopy(a)
    c = copy.deepcopy(a)
    bs = _batches(6)
    ob = torch_cls(b.parameters(), **kw)
    _train(b, ob, bs[:3])
    # continue the torch run inside a fused optimizer
    with torch.no_grad():
        for p, q in zip(a.parameters(), b.parameters()):
            p.copy_(q)
    oa = fused_cls(a.parameters(), **kw)
    oa.load_state_dict(ob.state_dict())
    _train(a, oa, bs[3:])
    _train(b, ob, bs[3:])
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    # fused state dict -> torch optimizer
    with torch.no_grad():
        for p, q in zip(c.parameters(), a.parameters()):
            p.copy_(q)
    oc = torch_cls(c.parameters(), **kw)
    oc.load_state_dict(copy.deepcopy(oa.state_dict()))   # state() holds views, as torch's
    more = _batches(8)[6:]
    _train(c, oc, more)
    _train(a, oa, more)
    for p, q in zip(a.parameters(), c.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_bf16_master_weights_cpu():
    """bf16 parameters: the fp32 master follows the fp32 torch run; params are its rounding."""
    a = _model(torch.bfloat16)
    b = _model(torch.float32)
    with torch.no_grad():
        for p, q in zip(a.parameters(), b.parameters()):
            q.copy_(p.float())
    oa = FusedAdamW(a.parameters(), lr=1e-2)
    (fl,) = oa.flat_buffers()
    assert fl.lowp and fl.master.dtype == torch.float32
    for p in a.parameters():
        assert oa.state[p]["master"].dtype == torch.float32
    bs = _batches(3, dtype=torch.bfloat16)
    _train(a, oa, bs)
    for p in a.parameters():
        torch.testing.assert_close(p, oa.state[p]["master"].to(p.dtype), rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("fused_cls,torch_cls,kw", CASES)
def test_gpu_fused_optim_matches_torch(cuda, fused_cls, torch_cls, kw):
    a = _mlp(device=cuda)
    b = copy.deepcopy(a)
    oa = fused_cls(a.parameters(), **kw)
    ob = torch_cls(b.parameters(), **kw)
    bs = _batches(5, device=cuda)
    _train(a, oa, bs)
    _train(b, ob, bs)
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(p, q, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_gpu_bf16_master_state_roundtrip(cuda):
    a = _mlp(torch.bfloat16, device=cuda)
    oa = FusedAdamW(a.parameters(), lr=1e-2)
    bs = _batches(3, device=cuda, dtype=torch.bfloat16)
    _train(a, oa, bs[:2])
    sd = copy.deepcopy(oa.state_dict())
    b = copy.deepcopy(a)
    ob = FusedAdamW(b.parameters(), lr=1e-2)
    ob.load_state_dict(sd)
    _train(a, oa, bs[2:])
    _train(b, ob, bs[2:])
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
