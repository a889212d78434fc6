"""CPU check of the index arithmetic of conv_gemm.hip's stride-2 data gradient (PAR mode): the
four output-parity classes with the kernel's own tap / offset / weight-column formulas, in fp64,
against PyTorch's transposed convolution."""
import pytest
import torch


def _par_dgrad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    N, Co, Ho, Wo = dy.shape
    Ci = w.shape[1]
    # the data-gradient layout: wr[ci][(3 ky + kx) Co + co] = w[co][ci][2 - ky][2 - kx]
    wr = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Ci, 9 * Co)
    dyp = torch.nn.functional.pad(dy, (0, 1, 0, 1))        # rows / cols Ho, Wo read as zero
    dx = torch.zeros(N, Ci, 2 * Ho, 2 * Wo, dtype=dy.dtype)
    for py in (0, 1):
        for px in (0, 1):
            for tap in range((py + 1) * (px + 1)):
                tyi, txi = (tap >> 1, tap & 1) if px else (tap, 0)
                ky = (2 if tyi else 0) if py else 1
                kx = (2 if txi else 0) if px else 1
                oy = 1 if (py and tyi == 0) else 0
                ox = 1 if (px and txi == 0) else 0
                col = 3 * (2 - ky) + (2 - kx)
                wsub = wr[:, col * Co:(col + 1) * Co]                  # [Ci, Co]
                src = dyp[:, :, oy:oy + Ho, ox:ox + Wo]
                dx[:, :, py::2, px::2] += torch.einsum("nchw,ic->nihw", src, wsub)
    return dx


@pytest.mark.parametrize("N,Co,Ci,Ho,Wo", [(2, 3, 5, 4, 4), (1, 4, 2, 3, 5), (2, 2, 3, 1, 2)])
def test_parity_class_dgrad_matches_transposed_conv(N, Co, Ci, Ho, Wo):
    g = torch.Generator().manual_seed(0)
    dy = torch.randn(N, Co, Ho, Wo, generator=g, dtype=torch.float64)
    w = torch.randn(Co, Ci, 3, 3, generator=g, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_input((N, Ci, 2 * Ho, 2 * Wo), w, dy, stride=2, padding=1)
    torch.testing.assert_close(_par_dgrad(dy, w), ref, rtol=1e-12, atol=1e-12)
    # the classes use 4 + 2 + 2 + 1 = 9 taps: every weight tap exactly once
