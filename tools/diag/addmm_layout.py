"""hipBLASLt acc.addmm_(a, B) for the layer-1.0 conv1 data gradient at batch 2560 (M = 8.03 M rows,
K = N = 64) with B given as W (contiguous) or as (W^T contiguous).t(): time per call."""
import torch


def main():
    dev = torch.device("cuda", 0)
    M = 2560 * 56 * 56
    a = torch.randn(M, 64, device=dev).bfloat16()
    acc = torch.randn(M, 64, device=dev).bfloat16()
    w2 = torch.randn(64, 64, device=dev).bfloat16()
    wt = w2.t().contiguous()
    for name, b in (("W contiguous", w2), ("W^T.t()", wt.t())):
        for _ in range(3):
            acc.addmm_(a, b)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            acc.addmm_(a, b)
        e.record()
        torch.cuda.synchronize()
        print(f"{name}: {s.elapsed_time(e) / 10 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
