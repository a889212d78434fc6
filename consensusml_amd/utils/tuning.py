"""Shipped MIOpen tuning (find-db) for the benchmark convolutions.

MIOpen find mode (``torch.backends.cudnn.benchmark = True``) times every applicable conv
solver on first use of each shape; for ResNet-50 at batch 512 that is ~4 minutes of warmup on a
fresh MI355X. The user find-db written by such a run (``tuning/miopen/*.ufdb.txt``: shape key ->
ranked solvers with measured ms; ``*.udb.txt``: tuned performance configs) is plain text keyed by
``gfx950`` + CU count (``100`` hex = 256 CUs), so it is valid on any MI355X with this MIOpen.

Measured on MI355X (profiles/r01_bench7_resnet50_krum_b512_finddb_kernels.md): even with the
find-db present, ~115 s of the warmup was MIOpen timing its *naive reference* convolution solvers
(``naive_conv_ab_nonpacked_{fwd,bwd,wrw}``, 0.1-0.5 s per call at batch 512) — solvers that are never
selected. ``configure_miopen()`` therefore also disables those three solvers
(``MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_{FWD,BWD,WRW}=0``) unless the caller set the variables.

``use_shipped_miopen_db()`` copies it into a scratch dir and points ``MIOPEN_USER_DB_PATH`` at it
(MIOpen reads the variable when it creates its first handle, i.e. at the first conv), unless the
caller already set the variable. Copying keeps the checked-in files untouched when MIOpen appends
new shapes. Returns the directory used, or None.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from typing import Optional

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHIPPED_DIR = os.path.join(_ROOT, "tuning", "miopen")


def use_shipped_miopen_db(src: str = SHIPPED_DIR) -> Optional[str]:
    if os.environ.get("MIOPEN_USER_DB_PATH"):
        return os.environ["MIOPEN_USER_DB_PATH"]
    if not os.path.isdir(src):
        return None
    files = [f for f in os.listdir(src) if f.endswith((".udb.txt", ".ufdb.txt"))]
    if not files:
        return None
    dst = os.path.join(tempfile.gettempdir(), f"cml_miopen_db_{os.getuid()}")
    os.makedirs(dst, exist_ok=True)
    for f in files:   # every rank of a node may get here at once: copy + atomic rename
        target = os.path.join(dst, f)
        if not os.path.exists(target):
            tmp = f"{target}.{os.getpid()}.tmp"
            shutil.copyfile(os.path.join(src, f), tmp)
            os.replace(tmp, target)
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst


NAIVE_SOLVER_VARS = ("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD",
                     "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD",
                     "MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW")


def configure_miopen(find_db: bool = True, skip_naive: bool = True) -> Optional[str]:
    """Call before the first convolution: shipped find-db + no naive reference solvers in find."""
    if skip_naive:
        for v in NAIVE_SOLVER_VARS:
            os.environ.setdefault(v, "0")
    return use_shipped_miopen_db() if find_db else None
