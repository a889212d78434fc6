"""Loader for the in-tree HIP extension (``consensusml_amd/_C*.so``).

GPU tensors always go through the native kernels; if the extension is missing on a GPU box the
ops raise instead of silently falling back to PyTorch (the CPU path exists only for CPU tensors,
i.e. the gloo plumbing config and tests).
"""
from __future__ import annotations

import os
import threading

_lock = threading.Lock()
_C = None
_err = None


def lib():
    """Return the loaded ``_C`` module or raise with build instructions."""
    global _C, _err
    if _C is not None:
        return _C
    with _lock:
        if _C is None:
            import torch  # noqa: F401  — loads libamdhip64 / libc10_hip first (same SONAME)
            try:
                from consensusml_amd import _C as mod
            except ImportError as e:  # pragma: no cover - depends on build state
                if os.environ.get("CML_AUTOBUILD", "1") == "1":
                    from consensusml_amd import _build
                    _build.build_kernels()
                    from consensusml_amd import _C as mod
                else:
                    _err = e
                    raise RuntimeError(
                        "consensusml_amd native HIP extension is not built; run "
                        "`python -m consensusml_amd._build`") from e
            _C = mod
            from .. import perf     # the policy's native-side switches
            perf.ensure_native_synced()
    return _C


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def so_path() -> str:
    return lib().__file__
