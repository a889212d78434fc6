#!/usr/bin/env python3
"""3x3 stride-1 convolutions of ResNet-50 at batch 2048: MIOpen (F.conv2d, channels_last bf16)
vs the implicit-GEMM TAP mode of csrc/kernels/conv1x1.hip (with and without the BN + ReLU
prologue and BN statistics epilogue). Prints max error vs an fp32 reference on a slice too.

  python bench/conv3x3.py
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn, it=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    from consensusml_amd.ops.native import lib
    from consensusml_amd.utils.tuning import configure_miopen
    configure_miopen()
    torch.backends.cudnn.benchmark = True
    L = lib()
    dev = torch.device("cuda:0")
    batch = int(os.environ.get("BATCH", "2048"))
    for C, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
        x = torch.randn(batch, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        sc = torch.rand(C, device=dev) + 0.5
        bi = torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        flops = 2 * batch * H * H * 9 * C * C
        t_lib = _t(lambda: F.conv2d(x, w, padding=1))
        gy = torch.randn_like(x)
        t_dg = _t(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        t_wg = _t(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        # data gradient = the forward TAP conv of gy with the rotated, transposed weights
        wr = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        t_own_dg = _t(lambda: L.conv3x3_bn_fwd(gy, wr, None, None, None, None, None, False, 1e-5, 0.1))
        dref = torch.ops.aten.convolution_backward(gy[:4].float(), x[:4].float(), w.float(), None,
                                                   [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0]
        down, _, _ = L.conv3x3_bn_fwd(gy[:4].contiguous(memory_format=torch.channels_last), wr,
                                      None, None, None, None, None, False, 1e-5, 0.1)
        dg_err = float((down.float() - dref).norm() / dref.norm())
        w2 = w.permute(0, 2, 3, 1).reshape(C, 9 * C).contiguous()
        wr2 = wr.permute(0, 2, 3, 1).reshape(C, 9 * C).contiguous()
        t_g = _t(lambda: L.conv_gemm(x, w2, 9))
        zr = torch.zeros(64, dtype=torch.bfloat16, device=dev)
        t_gst = _t(lambda: L.conv_gemm_bn(x, w2, 9, zr, rm, rm, rv, 1e-5, 0.1))
        y_lib = F.conv2d(x, w, padding=1)
        t_st = _t(lambda: L.bn_stats(y_lib, rm, rv, 1e-5, 0.1))
        del y_lib
        t_gdg = _t(lambda: L.conv_gemm(gy, wr2, 9))
        yg = L.conv_gemm(x[:4].contiguous(memory_format=torch.channels_last), w2, 9)
        g_ref = F.conv2d(x[:4].float(), w.float(), padding=1)
        g_err = float((yg.float() - g_ref).norm() / g_ref.norm())
        t_owg = _t(lambda: L.wgrad3x3(gy, x, torch.float32))
        t_owg_pro = _t(lambda: L.wgrad3x3(gy, x, torch.float32, sc, bi))
        wref = torch.ops.aten.convolution_backward(gy[:8].float(), x[:8].float(), w.float(), None,
                                                   [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                   [False, True, False])[1]
        wo = L.wgrad3x3(gy[:8].contiguous(memory_format=torch.channels_last),
                        x[:8].contiguous(memory_format=torch.channels_last), torch.float32)
        wg_err = float((wo.float() - wref).norm() / wref.norm())
        dgg = L.conv_gemm(gy[:4].contiguous(memory_format=torch.channels_last), wr2, 9)
        gdg_err = float((dgg.float() - dref).norm() / dref.norm())
        t_own = _t(lambda: L.conv3x3_bn_fwd(x, w, None, None, None, None, None, False, 1e-5, 0.1))
        t_own_st = _t(lambda: L.conv3x3_bn_fwd(x, w, sc, bi, rm, rm, rv, True, 1e-5, 0.1))
        # numerics on the first 4 images
        xs = x[:4]
        y, _, _ = L.conv3x3_bn_fwd(xs.contiguous(memory_format=torch.channels_last), w, None, None,
                                   None, None, None, False, 1e-5, 0.1)
        ref = F.conv2d(xs.float(), w.float(), padding=1)
        err = float((y.float() - ref).norm() / ref.norm())
        print(json.dumps({"C": C, "H": H, "batch": batch, "miopen_ms": round(t_lib, 4),
                          "own_ms": round(t_own, 4), "own_bnrelu_stats_ms": round(t_own_st, 4),
                          "miopen_tflops": round(flops / t_lib / 1e9, 1),
                          "own_tflops": round(flops / t_own / 1e9, 1), "rel_err": err,
                          "miopen_dgrad_ms": round(t_dg, 4), "own_dgrad_ms": round(t_own_dg, 4),
                          "miopen_wgrad_ms": round(t_wg, 4), "dgrad_rel_err": dg_err,
                          "glds_fwd_ms": round(t_g, 4), "glds_dgrad_ms": round(t_gdg, 4),
                          "glds_fwd_stats_ms": round(t_gst, 4), "bn_stats_ms": round(t_st, 4),
                          "glds_tflops": round(flops / t_g / 1e9, 1),
                          "glds_fwd_err": g_err, "glds_dgrad_err": gdg_err,
                          "own_wgrad_ms": round(t_owg, 4), "own_wgrad_pro_ms": round(t_owg_pro, 4),
                          "own_wgrad_err": wg_err}), flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
