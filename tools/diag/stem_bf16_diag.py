"""stem_wgrad_pool run-to-run determinism and its bf16-output form vs the fp32 outputs cast."""
import torch

from consensusml_amd.ops.native import lib
from consensusml_amd.ops.stem import pack_stem_weight


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(4)
    N, C, H, W = 4, 3, 64, 64
    x = torch.randn(N, C, H, W, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, C, 7, 7, device=dev) * 0.1).bfloat16()
    gam = torch.empty(64, device=dev).uniform_(-0.5, 1.5).bfloat16()
    bet = torch.empty(64, device=dev).uniform_(-0.5, 0.5).bfloat16()
    L = lib()
    z, mean, invstd = L.stem_conv_fwd(x, pack_stem_weight(w), None, None, 1e-5, 0.1, True)
    y, idx, _, _ = L.bn_relu_maxpool_fwd(z, gam, bet, None, None, mean, invstd, 1e-5, 0.1, False,
                                         3, 2, 1)
    dy = torch.randn_like(y)
    a = L.stem_wgrad_pool(dy, idx, None, z, x, mean, invstd, gam)
    b = L.stem_wgrad_pool(dy, idx, None, z, x, mean, invstd, gam)
    c = L.stem_wgrad_pool(dy, idx, None, z, x, mean, invstd, gam, True)
    for name, p, q, r in zip(("dw", "dg", "db"), a, b, c):
        d = (p - q).abs().max().item()
        m = (r != p.bfloat16()).sum().item()
        print(f"{name}: fp32 run-to-run max diff {d:.3e}; bf16-out vs cast mismatches {m} / "
              f"{r.numel()}, max {(r.float() - p.bfloat16().float()).abs().max().item():.3e}",
              flush=True)


if __name__ == "__main__":
    main()
