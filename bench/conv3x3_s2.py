"""Stride-2 3x3 conv data gradient per ResNet-50 shape: conv_gemm.hip's parity-class implicit
GEMMs (``conv_gemm_s2dgrad``, plain and with the BN + ReLU backward sums) vs MIOpen's backward-data
(``aten.convolution_backward``), and the forward with BN statistics (conv_gemm stride 2) vs MIOpen.
One JSON line per shape."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from consensusml_amd.ops.native import lib  # noqa: E402


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    L = lib()
    zero = torch.zeros(64, device=dev, dtype=torch.bfloat16)
    for C, H in ((128, 56), (256, 28), (512, 14)):
        N, Ho = args.batch, H // 2
        cl = torch.channels_last
        x = torch.randn(N, C, H, H, device=dev).bfloat16().contiguous(memory_format=cl)
        dy = torch.randn(N, C, Ho, Ho, device=dev).bfloat16().contiguous(memory_format=cl)
        w = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).bfloat16()
        wf, wr = L.conv3x3_wlayouts(w, True)
        z = torch.randn_like(x)
        sc = torch.rand(C, device=dev) + 0.5
        bi = torch.randn(C, device=dev) * 0.1
        mean = torch.zeros(C, device=dev)
        inv = torch.ones(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        own = _time(lambda: L.conv_gemm_s2dgrad(dy, wr, zero), args.iters)
        own_s = _time(lambda: L.conv_gemm_s2dgrad(dy, wr, zero, z, sc, bi, mean, inv), args.iters)
        lib_ms = _time(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]),
            args.iters)
        wg = _time(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]),
            args.iters)
        fwd_own = _time(lambda: L.conv_gemm_bn(x, wf, 9, zero, rm, rm, rv, 1e-5, 0.0, 2),
                        args.iters)
        fwd_lib = _time(lambda: torch.nn.functional.conv2d(x, w, stride=2, padding=1),
                        args.iters)
        ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), stride=2, padding=1) \
            if N <= 256 else None
        err = None
        if ref is not None:
            d = L.conv_gemm_s2dgrad(dy, wr, zero)[0].float()
            err = float((d - ref).norm() / ref.norm())
        flop = 2.0 * N * Ho * Ho * C * C * 9
        print(json.dumps({"C": C, "H": H, "batch": N, "dgrad_own_ms": round(own, 4),
                          "dgrad_own_sums_ms": round(own_s, 4), "dgrad_miopen_ms": round(lib_ms, 4),
                          "wgrad_miopen_ms": round(wg, 4), "fwd_own_bnstats_ms": round(fwd_own, 4),
                          "fwd_miopen_ms": round(fwd_lib, 4),
                          "dgrad_own_pflops": round(flop / own / 1e12, 3),
                          "dgrad_miopen_pflops": round(flop / lib_ms / 1e12, 3), "rel_err": err}),
              flush=True)
        del x, dy, z


if __name__ == "__main__":
    main()
