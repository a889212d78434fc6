"""Persistence of named result lists (the reference's ``save(<family>.resultslist, file=...rda)``).

The reference keeps each model family's results as an R named list saved after its stage
(`composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:673` svm4reps_resultslist, `:778`
lasso_resultslist, `:1069` rf_noboost_2k5k10ktrees_allresultslist, `:1239` xgb_resultslist) and
resumes later stages by ``load()``-ing them. Here a result list is a nested dict written as two
files next to each other, neither of which can execute anything on load:

  <prefix>.json          the tree: scalars, strings, small lists, and {"__array__": key} stubs
  <prefix>.safetensors   every array with more than ``SMALL`` elements, keyed by its tree path

``load_results`` rebuilds the dict with numpy arrays in place of the stubs.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict

import numpy as np
import torch

SMALL = 64


def _to_np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return x


def _encode(obj: Any, path: str, arrays: Dict[str, torch.Tensor]) -> Any:
    obj = _to_np(obj)
    if isinstance(obj, dict):
        return {str(k): _encode(v, f"{path}/{k}", arrays) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_encode(v, f"{path}/{i}", arrays) for i, v in enumerate(obj)]
    if isinstance(obj, np.ndarray):
        if obj.dtype == object:
            return [_encode(v, f"{path}/{i}", arrays) for i, v in enumerate(obj.tolist())]
        if obj.size > SMALL:
            key = path.lstrip("/")
            arrays[key] = torch.from_numpy(np.ascontiguousarray(obj))
            return {"__array__": key}
        return {"__small__": obj.tolist(), "dtype": str(obj.dtype), "shape": list(obj.shape)}
    if isinstance(obj, (np.integer,)):
        return int(obj)
    if isinstance(obj, (np.floating,)):
        return float(obj)
    if isinstance(obj, (np.bool_,)):
        return bool(obj)
    if obj is None or isinstance(obj, (bool, int, float, str)):
        return obj
    if hasattr(obj, "to_dict"):          # pandas objects
        return _encode(obj.to_dict(), path, arrays)
    return repr(obj)                     # models etc.: a description only


def _decode(obj: Any, arrays: Dict[str, np.ndarray]) -> Any:
    if isinstance(obj, dict):
        if "__array__" in obj:
            return arrays[obj["__array__"]]
        if "__small__" in obj:
            return np.array(obj["__small__"], dtype=obj["dtype"]).reshape(obj["shape"])
        return {k: _decode(v, arrays) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_decode(v, arrays) for v in obj]
    return obj


def save_results(prefix: str, obj: Dict[str, Any]) -> None:
    """Atomically write ``prefix``.json / .safetensors."""
    from safetensors.torch import save_file
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    arrays: Dict[str, torch.Tensor] = {}
    tree = _encode(obj, "", arrays)
    if arrays:
        save_file(arrays, prefix + ".safetensors.part")
        os.replace(prefix + ".safetensors.part", prefix + ".safetensors")
    with open(prefix + ".json.part", "w") as fh:
        json.dump(tree, fh)
    os.replace(prefix + ".json.part", prefix + ".json")


def load_results(prefix: str) -> Dict[str, Any]:
    from safetensors.torch import load_file
    arrays = {}
    if os.path.exists(prefix + ".safetensors"):
        arrays = {k: v.numpy() for k, v in load_file(prefix + ".safetensors").items()}
    with open(prefix + ".json") as fh:
        return _decode(json.load(fh), arrays)


def exists(prefix: str) -> bool:
    return os.path.exists(prefix + ".json")
