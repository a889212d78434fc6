"""Fused optimizers over flat buffers (one HIP launch per parameter group and dtype)."""
from .fused import FusedAdam, FusedAdamW, FusedSGD, build_optimizer

__all__ = ["FusedSGD", "FusedAdam", "FusedAdamW", "build_optimizer"]
