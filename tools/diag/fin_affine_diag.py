"""Run-to-run determinism of a ResNet-50 training step with the folded finalize launches on / off:
losses and the first differing gradients for the sequence off, on, off, on."""
import copy

import torch
import torch.nn.functional as F

import consensusml_amd.models.resnet as R
from consensusml_amd import perf


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    base = R.resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last).bfloat16()
    for m in base.modules():
        if hasattr(m, "running_mean") and getattr(m, "weight", None) is not None:
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.normal_(0, 0.1)
    x = torch.randn(8, 3, 96, 96, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev)
    runs = []
    for on in (False, True, False, True, True):
        m = copy.deepcopy(base)
        with perf.use_policy(perf.policy().replace(fin_affine=on, fin_dgamma=on)):
            out = m(x)
            loss = F.cross_entropy(out.float(), y)
            loss.backward()
        torch.cuda.synchronize()
        runs.append((on, loss.item(), out.detach().clone(),
                     {n: p.grad.clone() for n, p in m.named_parameters()}))
        print(f"fin={on} loss={loss.item():.6f}", flush=True)
    for i in range(1, len(runs)):
        a, b = runs[0], runs[i]
        diff = [n for n in a[3] if not torch.equal(a[3][n], b[3][n])]
        print(f"run0 vs run{i} (fin {a[0]} / {b[0]}): out equal {torch.equal(a[2], b[2])}, "
              f"{len(diff)} grads differ, first: {diff[:4]}", flush=True)
    diff = [n for n in runs[1][3] if not torch.equal(runs[1][3][n], runs[3][3][n])]
    print(f"run1 vs run3 (on / on): {len(diff)} grads differ, first {diff[:4]}")


if __name__ == "__main__":
    main()
