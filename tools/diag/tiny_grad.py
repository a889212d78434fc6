"""One forward/backward of resnet_tiny (bf16, channels_last) with our kernels vs PyTorch-only bf16,
both against an fp32 copy of the same model: relative gradient error (diagnostic)."""
import copy
import sys

import torch
import torch.nn.functional as F

import consensusml_amd.models.resnet as R
import consensusml_amd.ops.bn as B
import consensusml_amd.ops.pool as P

S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 16
torch.manual_seed(0)
dev = torch.device("cuda")
m32 = R.resnet_tiny(10).to(dev).to(memory_format=torch.channels_last)
for mod in m32.modules():
    if mod.__class__.__name__ == "BatchNormAct2d":
        with torch.no_grad():
            mod.weight.uniform_(0.5, 1.5)
            mod.bias.uniform_(-0.2, 0.2)
x = torch.randn(NB, 3, S, S, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (NB,), device=dev)
F.cross_entropy(m32(x), y).backward()
g32 = torch.cat([p.grad.flatten() for p in m32.parameters()])
orig = (B._fused_ok, P._pool_ok, R.CONV1X1_GEMM)
for variant in ("ours", "torch"):
    if variant == "torch":
        B._fused_ok = lambda *a: False
        P._pool_ok = lambda *a: False
        R.CONV1X1_GEMM = "miopen"
        R.FUSE_DOWN_BN = R.FUSE_STEM_POOL = R.FUSE_STEM_CONV = False
    m = copy.deepcopy(m32).to(torch.bfloat16)
    m.zero_grad(set_to_none=True)
    F.cross_entropy(m(x.to(torch.bfloat16)).float(), y).backward()
    g = torch.cat([p.grad.float().flatten() for p in m.parameters()])
    per = []
    for (n, p), p32 in zip(m.named_parameters(), m32.parameters()):
        e = ((p.grad.float() - p32.grad).norm() / p32.grad.norm().clamp_min(1e-12)).item()
        per.append((round(e, 3), n))
    per.sort(reverse=True)
    print(f"S={S} N={NB} {variant}: total rel err {((g - g32).norm() / g32.norm()).item():.4f} worst {per[:3]}")
