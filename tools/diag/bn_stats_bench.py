"""Time the BN forward (statistics + finalize + apply) on the ResNet-50 activation shapes at batch
1024 (cuda events, median of 15); run twice with CML_BN_STATS_ROWS=4 / 8 to compare the stats pass."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from consensusml_amd.ops.native import lib  # noqa: E402

dev = torch.device("cuda")
N = 1024
tot = 0.0
for C, hw in [(64, 56), (256, 56), (128, 28), (512, 28), (256, 14), (1024, 14), (512, 7), (2048, 7)]:
    x = torch.randn(N, C, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.ones(C, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(C, device=dev, dtype=torch.bfloat16)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)

    def f():
        return lib().bn_fwd(x, None, g, b, rm, rv, None, None, 1e-5, 0.1, True, True, False)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    t = sorted(ts)[7]
    tot += t
    print(f"C={C:5d} hw={hw:3d}: {t:8.1f} us  ({3 * x.numel() * 2 / t / 1e6:.2f} TB/s for 2 reads + 1 write)")
print(f"rows={os.environ.get('CML_BN_STATS_ROWS', '4')} total {tot:.1f} us")
