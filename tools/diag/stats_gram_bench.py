"""bn_stats_gram (bn3's statistics from the tail input's Gram matrix: two launches) per ResNet-50
tail shape: time per call (CUDA events, 50 calls)."""
import json

import torch

from consensusml_amd.ops.native import lib


def main():
    dev = torch.device("cuda", 0)
    L = lib()
    # (P, Co): identity tails p -> 4p (layers 1-3) and the downsample tails' x Gram (Cin -> 4p)
    for P, Co in [(64, 256), (128, 512), (256, 1024), (64, 256), (256, 512), (512, 1024)]:
        a = torch.randn(4096, P, device=dev)
        G = (a.t() @ a).contiguous()
        cy = a.sum(0)
        w = (torch.randn(Co, P, 1, 1, device=dev) * P ** -0.5).bfloat16()
        rm, rv = torch.zeros(Co, device=dev), torch.ones(Co, device=dev)
        gm, bt = torch.ones(Co, device=dev).bfloat16(), torch.zeros(Co, device=dev).bfloat16()
        f = lambda: L.bn_stats_gram(G, cy, w, 4096, rm, rv, 1e-5, 0.1, gm, bt)   # noqa: E731
        for _ in range(5):
            f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(50):
            f()
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"P": P, "Co": Co, "us_per_call": round(s.elapsed_time(e) / 50 * 1e3, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
