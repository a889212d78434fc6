"""Python face of the native host runtime (``consensusml_amd/_runtime*.so``, csrc/runtime).

* ``RecordDataset`` / ``DeviceLoader`` — records on disk -> C++ worker threads (mmap, seeded
  per-epoch shuffle, disjoint per-rank shares) -> ring of pinned host slots -> async H2D copy.
* ``Watchdog`` — hang / failure detector for the training loop.
* ``plan_buckets``, ``crc32_file``, ``write_file_atomic``, ``write_csv``.
"""
from __future__ import annotations

import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch


def native():
    from consensusml_amd import _runtime   # noqa: WPS433
    return _runtime


def available() -> bool:
    try:
        native()
        return True
    except ImportError:
        return False


def write_records(path: str, features: np.ndarray, labels: np.ndarray) -> int:
    """Write fixed-size records [features (float32 / uint8 ...) | label int64]; returns record bytes."""
    n = features.shape[0]
    f = np.ascontiguousarray(features).reshape(n, -1)
    lab = np.ascontiguousarray(labels.astype(np.int64)).reshape(n, 1)
    rec = np.concatenate([f.view(np.uint8), lab.view(np.uint8)], axis=1)
    with open(path, "wb") as fh:
        fh.write(rec.tobytes())
    return rec.shape[1]


class DeviceLoader:
    """Iterate device batches (x, y) from a record file with C++ prefetching.

    ``feature_shape`` / ``feature_dtype`` describe the feature part of each record; the label is
    a trailing int64. ``slots`` pinned buffers are filled ahead by ``threads`` C++ workers.
    """

    def __init__(self, path: str, feature_shape: Sequence[int], feature_dtype: torch.dtype,
                 batch: int, device: torch.device, rank: int = 0, world: int = 1, seed: int = 0,
                 threads: int = 4, slots: int = 4, out_dtype: Optional[torch.dtype] = None):
        rt = native()
        self.fshape = tuple(feature_shape)
        self.fdtype = feature_dtype
        fbytes = int(np.prod(self.fshape)) * torch.tensor([], dtype=feature_dtype).element_size()
        self.rec = fbytes + 8
        self.fbytes = fbytes
        self.batch = batch
        self.device = device
        self.out_dtype = out_dtype
        self.loader = rt.RecordLoader(path, self.rec, batch, rank, world, seed, threads, True)
        pin = device.type == "cuda"
        self.bufs = [torch.empty(batch * self.rec, dtype=torch.uint8, pin_memory=pin)
                     for _ in range(slots)]
        self.loader.start([b.data_ptr() for b in self.bufs], batch * self.rec, 0)
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None

    def __len__(self) -> int:
        return self.loader.batches_per_epoch()

    def next(self) -> Tuple[torch.Tensor, torch.Tensor, int]:
        slot, rows, epoch, _ = self.loader.next()
        raw = self.bufs[slot][: rows * self.rec].view(rows, self.rec)
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                d = raw.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            torch.cuda.current_stream(self.device).wait_event(ev)
            # the H2D copy must finish before the slot is refilled
            ev.synchronize()
        else:
            d = raw.clone()
        self.loader.release(slot)
        x = d[:, : self.fbytes].contiguous().view(self.fdtype).view(rows, *self.fshape)
        y = d[:, self.fbytes:].contiguous().view(torch.int64).view(rows)
        if self.out_dtype is not None:
            x = x.to(self.out_dtype)
        return x, y, epoch

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        while True:
            x, y, _ = self.next()
            yield x, y

    def close(self) -> None:
        self.loader.stop()


class Watchdog:
    """``with Watchdog(600, report) as wd: ... wd.beat(step)`` — fires if beats stop."""

    def __init__(self, timeout_s: float, report_path: str = "", hard_abort: bool = False):
        self._w = native().Watchdog(timeout_s, report_path, hard_abort)

    def beat(self, step: int) -> None:
        self._w.beat(step)

    def phase(self, name: str) -> None:
        self._w.set_phase(name)

    @property
    def fired(self) -> bool:
        return self._w.fired()

    def stop(self) -> None:
        self._w.stop()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def plan_buckets(numels: List[int], world: int, align: int, bucket_elems: int):
    return native().plan_buckets(list(numels), world, align, bucket_elems)


def crc32_file(path: str) -> int:
    return native().crc32_file(path)


def write_file_atomic(path: str, data: bytes) -> None:
    native().write_file_atomic(path, data)


def write_csv(path: str, row_names: List[str], cols: List[Tuple[str, list]]) -> None:
    native().write_csv(path, list(row_names), [(n, list(v)) for n, v in cols])
