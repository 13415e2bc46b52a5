"""Weight I/O in the reference's formats.

* ``.pt`` training checkpoints: ``{"epoch", "model_state_dict", "optimizer_state_dict",
  "global_step"}`` written by ``torch.save`` (FullPrecision/QuantizationAwareTraining.py:301-313)
  and read back with ``strict=False`` (:192-202).  Loading uses ``weights_only=True`` — nothing
  in the file is executed.
* per-key JSON export: one ``weight_export/{key}.json`` file per state_dict entry holding the
  tensor as nested lists (FullPrecision/exportWeights.py:55-70).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterable, Mapping, Optional

import numpy as np


def load_checkpoint(path: str) -> Dict[str, np.ndarray]:
    """State dict (numpy) from a reference ``.pt`` file: a training checkpoint dict or a bare state_dict."""
    import torch

    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict) and "model_state_dict" in obj:
        obj = obj["model_state_dict"]
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: not a state dict")
    return {k: (v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)) for k, v in obj.items()}


def save_checkpoint(path: str, state: Mapping[str, object], epoch: int = 0, global_step: int = 0,
                    optimizer_state: Optional[dict] = None) -> None:
    """Write the reference's checkpoint dict (QuantizationAwareTraining.py:305-313)."""
    import torch

    sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state.items()}
    torch.save({"epoch": epoch, "model_state_dict": sd, "optimizer_state_dict": optimizer_state or {},
                "global_step": global_step}, path)


def export_json(state: Mapping[str, object], directory: str) -> None:
    """``{directory}/{key}.json`` per entry, nested lists (exportWeights.py:62-70)."""
    os.makedirs(directory, exist_ok=True)
    for k, v in state.items():
        arr = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        with open(os.path.join(directory, f"{k}.json"), "w") as f:
            json.dump(arr.tolist(), f)


def import_json(directory: str, keys: Optional[Iterable[str]] = None) -> Dict[str, np.ndarray]:
    """Inverse of :func:`export_json` (all ``*.json`` files, or the given keys)."""
    if keys is None:
        keys = [f[:-5] for f in sorted(os.listdir(directory)) if f.endswith(".json")]
    out = {}
    for k in keys:
        with open(os.path.join(directory, f"{k}.json")) as f:
            v = json.load(f)
        a = np.asarray(v)
        out[k] = a.astype(np.int64) if k.endswith("num_batches_tracked") else a.astype(np.float32)
    return out
