"""Per-worker parameter gradients for batched virtual workers.

The engine's virtual workers (``TrainConfig.virtual_workers`` = V micro-batches on one GPU, each
with its own gradient row for the robust rule) normally run V sequential forward / backward
passes. For models whose forward has no cross-sample coupling -- BERT: LayerNorm is per token,
attention per sequence, no BatchNorm -- the V micro-batches can run as ONE batch: every
activation and activation gradient is exactly the per-worker one, and only the parameter
gradients must stay separated. Inside ``ConsensusEngine.worker_batch()`` the ops that own a
parameter (``ops.transformer`` Linear / norms / the BERT embedding) write the gradient of worker
v straight into row v of the engine's flat gradient buffer:

  Linear     dW[v] = dY_v^T X_v (one strided-batched GEMM into the V rows), db[v] = colsum(dY_v)
  norms      dgamma / dbeta folded per worker segment (``norm_bwd_seg``)
  embedding  per-worker dense embedding backward, position / type sums

and return no gradient to autograd, so the engine's copy of autograd gradients into the buffer
(``multi_copy``) disappears as well. GEMMs run at M = V x tokens instead of tokens (the BERT
config: 32 768 rows instead of 4 096) and every per-layer elementwise / norm / attention kernel
launches once instead of V times.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

_CURRENT: Optional["WorkerGrads"] = None


class WorkerGrads:
    """Destination of the per-worker gradients of one batched backward: ``views[id(p)]`` is a
    [V, *p.shape] view of the engine's flat gradient rows. The first op to produce a parameter's
    gradient overwrites the rows; later ones (a tied weight: BERT's token embedding is also the
    MLM output projection) add."""

    def __init__(self, V: int, views: Dict[int, torch.Tensor]):
        self.V = V
        self.views = views
        self.touched: set = set()

    def has(self, p: Optional[torch.Tensor]) -> bool:
        return p is not None and id(p) in self.views

    def out(self, p: torch.Tensor) -> Tuple[torch.Tensor, bool]:
        """(the [V, *shape] destination, True when this is its first write this step)."""
        k = id(p)
        first = k not in self.touched
        self.touched.add(k)
        return self.views[k], first

    def put(self, p: torch.Tensor, g: torch.Tensor) -> None:
        """Write (first producer) or add a [V, *shape] gradient."""
        dst, first = self.out(p)
        if first:
            dst.copy_(g)
        else:
            dst.add_(g)

    def untouched(self):
        return [k for k in self.views if k not in self.touched]


def current() -> Optional[WorkerGrads]:
    return _CURRENT


def activate(wg: Optional[WorkerGrads]) -> Optional[WorkerGrads]:
    global _CURRENT
    prev = _CURRENT
    _CURRENT = wg
    return prev
