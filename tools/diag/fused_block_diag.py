#!/usr/bin/env python3
"""Compare one ResNet bottleneck (and the whole ResNet-50) between the fused conv + BN path and
the unfused path: forward output, every parameter gradient and the input gradient."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import consensusml_amd.models.resnet as R  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def run(block, x, g, fused):
    R.FUSED_CONV1X1 = fused
    try:
        xx = x.detach().clone().requires_grad_(True)
        y = block(xx)
        y.backward(g)
    finally:
        R.FUSED_CONV1X1 = True
    return y.detach(), xx.grad, {k: p.grad.clone() for k, p in block.named_parameters()}


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for cin, planes, hw, down in ((256, 64, 16, False), (64, 64, 16, True), (256, 64, 56, False)):
        b0 = R.Bottleneck(cin, planes, 1, down).to(dev, torch.bfloat16).to(
            memory_format=torch.channels_last)
        with torch.no_grad():
            for m in b0.modules():
                if hasattr(m, "running_mean"):
                    m.weight.copy_(torch.rand_like(m.weight.float()) + 0.5)
                    m.bias.copy_(torch.randn_like(m.bias.float()) * 0.1)
        b1 = copy.deepcopy(b0)
        x = torch.randn(8, cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        g = torch.randn(8, planes * 4, hw, hw, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y0, dx0, p0 = run(b0, x, g, True)
        y1, dx1, p1 = run(b1, x, g, False)
        print(f"block cin={cin} planes={planes} hw={hw} down={down}: y {rel(y0, y1):.2e} "
              f"dx {rel(dx0, dx1):.2e}")
        for k in p1:
            print(f"   {k:24s} {rel(p0[k], p1[k]):.2e}")
        for (k, v0), (_, v1) in zip(b0.named_buffers(), b1.named_buffers()):
            print(f"   buf {k:20s} {rel(v0, v1):.2e}")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def model_vs_fp32():
    """Whole ResNet-50 (64 x 64 images, batch 16): gradient cosine of the fused and the unfused
    bf16 paths against an fp32 copy (PyTorch reference compositions)."""
    dev = torch.device("cuda")
    torch.manual_seed(11)
    m32 = R.resnet50(num_classes=10).to(dev)
    with torch.no_grad():
        for mod in m32.modules():
            if isinstance(mod, R.Bottleneck):
                mod.bn3.weight.fill_(0.2)
    x = torch.randn(16, 3, 64, 64, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    out = {}
    for name in ("fp32", "fused", "unfused"):
        m = copy.deepcopy(m32)
        xx = x
        if name != "fp32":
            m = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
            xx = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        R.FUSED_CONV1X1 = name == "fused"
        loss = F.cross_entropy(m(xx).float(), y)
        loss.backward()
        R.FUSED_CONV1X1 = True
        out[name] = (loss.item(), torch.cat([p.grad.float().flatten() for p in m.parameters()]))
    for name in ("fused", "unfused"):
        c = F.cosine_similarity(out[name][1], out["fp32"][1], dim=0).item()
        print(f"{name}: loss {out[name][0]:.5f} (fp32 {out['fp32'][0]:.5f}) grad cos vs fp32 {c:.4f}")
    print("fused vs unfused cos", F.cosine_similarity(out["fused"][1], out["unfused"][1], dim=0).item())


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "model":
    model_vs_fp32()
