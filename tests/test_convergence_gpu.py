"""The fused ResNet-50 step trains like the library path (bench/convergence.py at a reduced
length): same random-init weights, same learnable synthetic batches (class templates + noise),
default PerfPolicy (own kernels and fusions) vs PerfPolicy.library() (MIOpen / hipBLASLt +
PyTorch BatchNorm). Both must learn the task, and their loss curves, accuracies and BN running
statistics must agree; the committed 100-step curve at batch 128 is in profiles/r03_convergence/."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "bench"))


def test_fused_step_trains_like_library(cuda):
    import convergence as C
    from consensusml_amd import perf
    torch.backends.cudnn.benchmark = False
    steps, batch = 40, 32
    fused = C.run("fused", perf.policy(), C.make_cfg(batch, 224, 10, 0.05), steps, 4, batch)
    lib = C.run("library", perf.PerfPolicy.library(), C.make_cfg(batch, 224, 10, 0.05), steps, 4,
                batch)
    # noise floor: the library path again from weights perturbed at bf16-rounding level
    libp = C.run("library_perturbed", perf.PerfPolicy.library(), C.make_cfg(batch, 224, 10, 0.05),
                 steps, 4, batch, perturb=2.0 ** -8)
    cmp = C.compare(fused, lib)
    noise = C.compare(libp, lib)
    print("fused vs library:", cmp, "\nperturbed library vs library:", noise, flush=True)
    # both learn the 10-class template task (chance: 2.3 nats, 10 %)
    for r in (fused, lib):
        assert sum(r["losses"][-5:]) / 5 < 0.5 * r["losses"][0], r["losses"]
        assert r["acc_train_mode"] > 0.8, r["acc_train_mode"]
    # SGD at this batch amplifies any rounding difference, so after the first steps the fused path
    # is judged against that noise floor: early losses agree closely, later losses, accuracies and
    # BN running statistics within a small multiple of the floor
    assert cmp["loss_rel_diff"][0] < 0.05, (cmp, noise)
    assert cmp["mean_loss_abs_diff"] <= 3 * noise["mean_loss_abs_diff"] + 0.02, (cmp, noise)
    assert abs(cmp["acc_train_mode_diff_points"]) <= 5.0, (cmp, noise)
    assert cmp["bn_stats_median_rel_diff"] <= 3 * noise["bn_stats_median_rel_diff"] + 0.01, \
        (cmp, noise)
