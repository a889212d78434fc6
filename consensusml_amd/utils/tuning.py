"""Shipped MIOpen tuning (find-db) for the benchmark convolutions.

MIOpen find mode (``torch.backends.cudnn.benchmark = True``) times every applicable conv
solver on first use of each shape; for ResNet-50 at batch 512 that is ~4 minutes of warmup on a
fresh MI355X. The user find-db written by such a run (``tuning/miopen/*.ufdb.txt``: shape key ->
ranked solvers with measured ms; ``*.udb.txt``: tuned performance configs) is plain text keyed by
``gfx950`` + CU count (``100`` hex = 256 CUs), so it is valid on any MI355X with this MIOpen.

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
