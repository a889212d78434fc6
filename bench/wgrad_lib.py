"""Weight gradients still on MIOpen in the ResNet-50 step (the shapes
``tools/list_lib_convs.py`` lists, profiles/r05_11/lib_convs_b2048.jsonl): MIOpen time vs the own
kernel (wgrad1x1.hip for stride-1 1x1, wgrad3x3s2 for stride-2 3x3) per shape, with the HBM
floor (x + dy read once). Emits one JSON line per shape.

    python bench/wgrad_lib.py [batch] [--reps R]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusml_amd.ops.native import lib  # noqa: E402
from consensusml_amd.utils.tuning import configure_miopen  # noqa: E402

# (cin, cout, k, stride, hw_in, calls per step) -- the b2048 list of r05_11
SHAPES = [
    (64, 64, 1, 1, 56, 1), (256, 64, 1, 1, 56, 2), (256, 128, 1, 1, 56, 1),
    (512, 256, 1, 1, 28, 1), (1024, 256, 1, 1, 14, 5), (1024, 512, 1, 1, 14, 1),
    (1024, 2048, 1, 1, 7, 1),
    (128, 128, 3, 2, 56, 1), (256, 256, 3, 2, 28, 1), (512, 512, 3, 2, 14, 1),
    # stride-2 1x1 downsamples (layer 4's stays a stride-2 conv in the step; layers 2-3 recompute
    # from the subsampled input)
    (1024, 2048, 1, 2, 14, 1), (512, 1024, 1, 2, 28, 0), (256, 512, 1, 2, 56, 0),
]
# the own-kernel (core) set, for the own-vs-own A/B (CML_WGRAD_DMA=0 / 1); calls = 0: not on the
# library in the step
CORE = [(128, 512, 1, 1, 28, 0), (512, 128, 1, 1, 28, 0), (256, 1024, 1, 1, 14, 0),
        (512, 2048, 1, 1, 7, 0), (2048, 512, 1, 1, 7, 0)]


def _time(f, reps):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("batch", nargs="?", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--core", action="store_true", help="also the own-kernel set")
    args = ap.parse_args()
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    N, dev, cl = args.batch, torch.device("cuda"), torch.channels_last
    tot_lib = tot_best = 0.0
    for cin, cout, k, s, hw, calls in SHAPES + (CORE if args.core else []):
        ho = (hw + 2 * (k // 2) - k) // s + 1
        x = torch.randn(N, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(N, cout, ho, ho, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        w = torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        pad = k // 2

        def f_lib():
            return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [pad, pad], [1, 1],
                                                       False, [0, 0], 1, [False, True, False])[1]
        t_lib = _time(f_lib, args.reps)
        ref = f_lib().float()
        t_own, err = None, None
        if k == 1 and s == 1 and (cin == 64 and cout % 256 == 0 or cin % 128 == 0 and cout % 128 == 0):
            def f_own():
                return lib().wgrad1x1(dy, x, torch.bfloat16)
        elif k == 1 and s == 2 and lib().wgrad3x3s2_ok(N, hw, hw, cout, cin, 1):
            def f_own():
                return lib().wgrad3x3s2(dy, x, torch.bfloat16, taps=1)
        elif k == 3 and s == 2 and hasattr(lib(), "wgrad3x3s2") and lib().wgrad3x3s2_ok(
                N, hw, hw, cout, cin):
            def f_own():
                return lib().wgrad3x3s2(dy, x, torch.bfloat16)
        else:
            f_own = None
        if f_own is not None:
            t_own = _time(f_own, args.reps)
            out = f_own().float()
            out = (out.permute(0, 2, 3, 1) if k == 3 else out).reshape(cout, -1)
            r = ref.permute(0, 2, 3, 1).reshape(cout, -1) if k == 3 else ref.reshape(cout, -1)
            err = ((out - r).norm() / r.norm()).item()
        byt = (x.numel() + dy.numel()) * 2
        flop = 2.0 * N * ho * ho * cout * cin * k * k
        best = min(t_lib, t_own) if t_own is not None else t_lib
        tot_lib += calls * t_lib
        tot_best += calls * best
        print(json.dumps({"cin": cin, "cout": cout, "k": k, "stride": s, "hw": hw, "calls": calls,
                          "lib_us": round(t_lib * 1e3, 1),
                          "own_us": None if t_own is None else round(t_own * 1e3, 1),
                          "rel_err": err, "floor_us": round(byt / 5.5e12 * 1e6, 1),
                          "lib_tflops": round(flop / t_lib * 1e-9, 1),
                          "own_tflops": None if t_own is None else round(flop / t_own * 1e-9, 1)}),
              flush=True)
        del x, dy, w, ref
    print(json.dumps({"batch": N, "lib_ms_per_step": round(tot_lib, 3),
                      "best_ms_per_step": round(tot_best, 3)}), flush=True)


if __name__ == "__main__":
    main()
