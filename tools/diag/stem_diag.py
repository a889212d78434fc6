"""Diagnostics for the stem kernels: every intermediate vs a float64 torch evaluation."""
import torch
import torch.nn.functional as F

from consensusml_amd.ops.native import lib
from consensusml_amd.ops.stem import pack_stem_weight

torch.manual_seed(0)
dev = torch.device("cuda")
N, C, H, W = 4, 3, 64, 64
x = torch.randn(N, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, C, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
gam = torch.empty(64, device=dev).uniform_(-0.5, 1.5).to(torch.bfloat16)
bet = torch.empty(64, device=dev).uniform_(-0.5, 0.5).to(torch.bfloat16)
z, mean, invstd = lib().stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
zr = F.conv2d(x.double(), w.double(), stride=2, padding=3)
print("z rel", ((z.double() - zr).norm() / zr.norm()).item())
mr = zr.mean((0, 2, 3))
vr = zr.var((0, 2, 3), unbiased=False)
print("mean abs err", (mean.double() - mr).abs().max().item(), "invstd rel", ((invstd.double() - (vr + 1e-5).rsqrt()) / (vr + 1e-5).rsqrt()).abs().max().item())
y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1, False, 3, 2, 1)
dy = torch.randn_like(y)
g, gsum = lib().maxpool_bwd_sum(dy, idx, z.shape[2], z.shape[3])
# torch: masked gradient
u = (z.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1) * gam.double().view(1, -1, 1, 1) + bet.double().view(1, -1, 1, 1)
ud = u.detach().requires_grad_(True)
yp = F.max_pool2d(torch.relu(ud), 3, 2, 1)
yp.backward(dy.double())
gr = ud.grad
print("g rel", ((g.double() - gr).norm() / gr.norm()).item(), "frac idx255", (idx == 255).float().mean().item())
dw, dg, db = lib().stem_wgrad(g, z, x, mean, invstd, gam, gsum)
gd = g.double()
xh = (z.double() - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
s1 = gd.sum((0, 2, 3))
s2 = (gd * xh).sum((0, 2, 3))
print("db rel", ((db.double() - s1).norm() / s1.norm()).item())
print("dg rel", ((dg.double() - s2).norm() / s2.norm()).item())
print("dg sample", dg[:6].tolist(), s2[:6].tolist())
# dW through BN
M = gd.numel() / 64
dz = gam.double().view(1, -1, 1, 1) * invstd.double().view(1, -1, 1, 1) * (gd - s1.view(1, -1, 1, 1) / M - xh * (s2.view(1, -1, 1, 1) / M))
wq = w.double().requires_grad_(True)
F.conv2d(x.double(), wq, stride=2, padding=3).backward(dz)
print("dw rel", ((dw.double() - wq.grad).norm() / wq.grad.norm()).item())
# pieces: G = conv wgrad of g
wq2 = w.double().requires_grad_(True)
F.conv2d(x.double(), wq2, stride=2, padding=3).backward(gd)
print("G-only wgrad norm", wq2.grad.norm().item(), "dw norm", wq.grad.norm().item())
