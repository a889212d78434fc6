"""MIOpen weight-gradient time of every stride-1 1x1 conv of ResNet-50 (bf16 NHWC, shipped
find-db) vs its memory floor (dy + x read once)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from consensusml_amd.utils.tuning import configure_miopen  # noqa: E402

configure_miopen()
torch.backends.cudnn.benchmark = True
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dev = torch.device("cuda")
shapes = [(64, 56, 64), (64, 56, 256), (256, 56, 64), (256, 56, 128), (128, 28, 512), (512, 28, 128),
          (512, 28, 256), (256, 14, 1024), (1024, 14, 256), (1024, 14, 512), (512, 7, 2048),
          (2048, 7, 512)]
tot_t = tot_b = 0.0
for cin, hw, cout in shapes:
    x = torch.randn(N, cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, 1, 1, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, cout, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def f():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                   [0, 0], 1, [False, True, False])
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    t = sorted(ts)[5] * 1e-3
    t_own = None
    if cin % 128 == 0 and cout % 128 == 0:
        from consensusml_amd.ops.native import lib
        for _ in range(3):
            lib().wgrad1x1(dy, x, torch.bfloat16)
        torch.cuda.synchronize()
        to = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            lib().wgrad1x1(dy, x, torch.bfloat16)
            b.record()
            torch.cuda.synchronize()
            to.append(a.elapsed_time(b))
        t_own = sorted(to)[5] * 1e-3
    byt = (x.numel() + dy.numel()) * 2
    tot_t += t
    tot_b += byt
    print(f"{cin:5d}->{cout:5d} @{hw:3d}: {t * 1e6:8.1f} us  {byt / t / 1e12:5.2f} TB/s  "
          f"floor@5.5TB/s {byt / 5.5e12 * 1e6:7.1f} us  own "
          f"{'-' if t_own is None else f'{t_own * 1e6:8.1f} us'}", flush=True)
print(f"total {tot_t * 1e3:.2f} ms, floor {tot_b / 5.5e12 * 1e3:.2f} ms")
