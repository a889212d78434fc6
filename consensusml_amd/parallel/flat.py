"""Flat, bucketed parameter and gradient storage (N02).

Every parameter of the model becomes a view into ONE flat bf16 parameter buffer, and its
``.grad`` a view (same strides, so channels_last conv weights stay channels_last) into ONE
flat gradient buffer. autograd then accumulates straight into the flat buffer, the collectives
move whole buckets without packing, and the fused HIP optimizer updates the flat buffer in one
pass.

Layout. Parameters are taken in reverse registration order (≈ the order backward produces their
gradients) and packed into buckets of about ``bucket_elems`` elements. Each bucket is padded to
a multiple of ``world * ALIGN`` so that its per-rank shard (``shard = len / world``) starts on a
128-byte boundary — the unit of the sharded topology's all-to-all / all-gather.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

ALIGN = 64   # elements; 128 B of bf16 -> every shard / bucket start is cache-line aligned


def _native_plan(numels: List[int], world: int, bucket_elems: int):
    try:
        from consensusml_amd import _runtime
    except ImportError:
        return None
    return _runtime.plan_buckets(numels, world, ALIGN, bucket_elems)


@dataclass
class Bucket:
    index: int
    offset: int          # element offset in the flat buffers
    length: int          # padded length (multiple of world * ALIGN)
    shard: int           # length // world
    shard_offset: int    # offset of this bucket's shard inside a rank's shard vector
    params: List[int]    # indices into FlatModel.params


class FlatModel:
    def __init__(self, model: torch.nn.Module, world: int, bucket_mb: float = 64.0,
                 grad_rows: int = 1, param_dtype: torch.dtype = torch.bfloat16):
        self.model = model
        self.world = world
        self.params: List[torch.nn.Parameter] = [p for p in model.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("model has no trainable parameters")
        dev = self.params[0].device
        self.device = dev
        self.dtype = param_dtype
        esize = torch.finfo(param_dtype).bits // 8
        bucket_elems = max(int(bucket_mb * 1024 * 1024 / esize), ALIGN)
        unit = world * ALIGN

        order = list(range(len(self.params)))[::-1]
        self.buckets: List[Bucket] = []
        self.param_offset: Dict[int, int] = {}
        cur: List[int] = []
        cur_len = 0
        off = 0
        shard_off = 0

        def close():
            nonlocal cur, cur_len, off, shard_off
            if not cur:
                return
            L = -(-cur_len // unit) * unit
            b = Bucket(len(self.buckets), off, L, L // world, shard_off, cur)
            self.buckets.append(b)
            off += L
            shard_off += L // world
            cur, cur_len = [], 0

        plan = _native_plan([self.params[i].numel() for i in order], world, bucket_elems)
        if plan is not None:   # C++ planner (csrc/runtime) — same rule as the loop below
            for k, i in enumerate(order):
                self.param_offset[i] = plan.param_offsets[k]
            members: Dict[int, List[int]] = {}
            for k, i in enumerate(order):
                members.setdefault(plan.param_bucket[k], []).append(i)
            so = 0
            for bi, (o, L, S) in enumerate(zip(plan.offsets, plan.lengths, plan.shards)):
                self.buckets.append(Bucket(bi, o, L, S, so, members[bi]))
                so += S
            off, shard_off = plan.total, plan.shard_total
        else:
            for i in order:
                n = self.params[i].numel()
                if cur and cur_len + n > bucket_elems:
                    close()
                self.param_offset[i] = off + cur_len
                cur.append(i)
                # keep each parameter 16-byte aligned inside the bucket
                cur_len += -(-n // 8) * 8
            close()
        self.total = off
        self.shard_total = shard_off
        self.bucket_of = {i: b.index for b in self.buckets for i in b.params}
        self.real_numel = sum(p.numel() for p in self.params)

        # flat storage
        self.flat_param = torch.zeros(self.total, dtype=param_dtype, device=dev)
        self.grad_rows = grad_rows
        self.flat_grad = torch.zeros(grad_rows, self.total, dtype=param_dtype, device=dev)
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self._view(self.flat_param, i)
                v.copy_(p.detach().to(param_dtype))
                p.data = v
        self.bind_grads(0)

    # ------------------------------------------------------------------ views
    def _view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        # as_strided offsets are absolute in the storage: add the view's own offset (grad rows)
        return torch.as_strided(flat, p.shape, p.stride(),
                                flat.storage_offset() + self.param_offset[i])

    def bind_grads(self, row: int) -> None:
        """Point every param.grad at row ``row`` of the gradient buffer (virtual workers)."""
        g = self.flat_grad[row]
        for i, p in enumerate(self.params):
            p.grad = self._view(g, i)
        self.grad_row = row

    def grad_views(self, row: int) -> List[torch.Tensor]:
        """Per-parameter views of gradient row ``row`` (cached) for the copy-on-ready mode."""
        cache = getattr(self, "_gv", None)
        if cache is None:
            cache = self._gv = {}
        if row not in cache:
            g = self.flat_grad[row]
            cache[row] = [self._view(g, i) for i in range(len(self.params))]
        return cache[row]

    def worker_views(self) -> List[torch.Tensor]:
        """Per-parameter [grad_rows, *shape] views spanning every gradient row (cached): the
        destinations of batched virtual workers (ops.worker_grads)."""
        cache = getattr(self, "_wv", None)
        if cache is None:
            g = self.flat_grad
            cache = self._wv = [
                torch.as_strided(g, (self.grad_rows,) + tuple(p.shape),
                                 (g.stride(0),) + tuple(p.stride()),
                                 g.storage_offset() + self.param_offset[i])
                for i, p in enumerate(self.params)]
        return cache

    def release_grads(self, row: int) -> None:
        """Switch to copy-on-ready mode: autograd owns fresh .grad tensors, hooks copy them."""
        for p in self.params:
            p.grad = None
        self.grad_row = row

    def zero_grad(self) -> None:
        self.flat_grad.zero_()

    def bucket_slice(self, flat: torch.Tensor, b: Bucket) -> torch.Tensor:
        return flat[..., b.offset:b.offset + b.length]

    def my_shard(self, flat: torch.Tensor, b: Bucket, rank: int) -> torch.Tensor:
        s = b.offset + rank * b.shard
        return flat[..., s:s + b.shard]

    def gather_shard_vector(self, flat: torch.Tensor, rank: int) -> torch.Tensor:
        """Concatenate this rank's shard of every bucket (layout of the sharded optimizer state)."""
        return torch.cat([self.my_shard(flat, b, rank) for b in self.buckets])

    def param_names(self) -> List[str]:
        names = {id(p): n for n, p in self.model.named_parameters()}
        return [names.get(id(p), f"param{i}") for i, p in enumerate(self.params)]

    def segments(self) -> List[Tuple[str, int, int]]:
        """(name, flat offset, numel) per parameter — used by the consensus table export."""
        return [(n, self.param_offset[i], self.params[i].numel())
                for i, n in enumerate(self.param_names())]
