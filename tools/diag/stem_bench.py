"""Time the stem kernels alone at the bench shape (batch 512, 224x224): conv fwd, pool fwd,
pool bwd, wgrad (cuda events, median of 20)."""
import sys

import torch

from consensusml_amd.ops.native import lib
from consensusml_amd.ops.stem import pack_stem_weight

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda")
torch.manual_seed(0)
x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
gam = torch.ones(64, device=dev, dtype=torch.bfloat16)
bet = torch.zeros(64, device=dev, dtype=torch.bfloat16)
wpk = pack_stem_weight(w)


def timeit(fn, reps=20):
    ts = []
    for _ in range(reps + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[3:])
    return ts[len(ts) // 2]


z, mean, invstd = lib().stem_conv_fwd(x, wpk, None, None, 1e-5, 0.1, True)
y, idx, _, _ = lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1, False, 3, 2, 1)
dy = torch.randn_like(y)
g, gsum = lib().maxpool_bwd_sum(dy, idx, 112, 112)
r = {
    "conv_fwd": timeit(lambda: lib().stem_conv_fwd(x, wpk, None, None, 1e-5, 0.1, True)),
    "pool_fwd": timeit(lambda: lib().bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1, False, 3, 2, 1)),
    "pool_bwd": timeit(lambda: lib().maxpool_bwd_sum(dy, idx, 112, 112)),
    "wgrad": timeit(lambda: lib().stem_wgrad(g, z, x, mean, invstd, gam, gsum)),
}
print({k: round(v, 1) for k, v in r.items()}, "us")
