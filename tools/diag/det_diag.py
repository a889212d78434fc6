"""Find the first module whose forward output differs between two identical ResNet-50 training
forwards (fresh deep copies of one model, same input)."""
import copy
import sys

import torch

import consensusml_amd.models.resnet as R


def record(m, x):
    outs = []

    def hook(mod, inp, out, name=None):
        o = out[0] if isinstance(out, (tuple, list)) else out
        if torch.is_tensor(o):
            outs.append((name, o.detach().clone()))
    hs = [mod.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n))
          for n, mod in m.named_modules() if n.count(".") <= int(sys.argv[3]) and n]
    y = m(x)
    y.float().sum().backward()
    for h in hs:
        h.remove()
    torch.cuda.synchronize()
    return outs


def main():
    dev = torch.device("cuda", 0)
    n, hw = int(sys.argv[1]), int(sys.argv[2])
    torch.manual_seed(3)
    base = R.resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last).bfloat16()
    for m in base.modules():   # non-trivial BN parameters (bn3 is zero-initialised)
        if hasattr(m, "running_mean") and getattr(m, "weight", None) is not None:
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.normal_(0, 0.1)
    x = torch.randn(n, 3, hw, hw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    a = record(copy.deepcopy(base), x)
    b = record(copy.deepcopy(base), x)
    c = record(copy.deepcopy(base), x)
    for (na, ta), (nb, tb), (nc, tc) in zip(a, b, c):
        if not (torch.equal(ta, tb) and torch.equal(ta, tc)):
            print(f"batch {n} x {hw}: first differing module output: {na} "
                  f"max|a-b| {(ta.float() - tb.float()).abs().max().item():.3e} "
                  f"max|a-c| {(ta.float() - tc.float()).abs().max().item():.3e}", flush=True)
            return
    print(f"batch {n} x {hw}: all {len(a)} module outputs identical over 3 runs", flush=True)


if __name__ == "__main__":
    main()
