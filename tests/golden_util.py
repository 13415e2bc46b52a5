"""Loading the committed golden fixtures (tests/golden/*.npz).

Fixtures hold inputs, ProbSparse index draws, outputs and activations produced by
the reference itself (tests/golden/make_golden.py); weights are regenerated here
from the recorded schema + seed with the engine's synthetic recipe.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from channelestimationtransformer_amd.weights import synthetic_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@dataclass
class Case:
    name: str
    meta: dict
    z: Dict[str, np.ndarray]
    state: Dict[str, np.ndarray]
    idx: List[np.ndarray]

    @property
    def cfg(self):
        return self.meta["cfg"]

    def acts(self):
        return {k[4:]: v for k, v in self.z.items() if k.startswith("act_")}


def case_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("data_"))


def layerwise_name(name: str) -> bool:
    """Fixture cases whose shapes only the layer-wise engine carries (d_model != 128, n_heads != 8,
    d_ff > 128, more than 48 decoder rows); their names say so."""
    return any(t in name for t in ("_d64_", "_h5_", "_d256_", "_d512_"))


def load_case(name: str) -> Case:
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as f:
        z = {k: f[k] for k in f.files}
    meta = json.loads(str(z.pop("meta")))
    spec = [(k, tuple(s), kd) for k, s, kd in meta["keys"]]
    state = synthetic_state_dict(spec, meta["weight_seed"], lsq_bits=meta["cfg"].get("num_bits", 8))
    idx = [z[f"idx{k}"] for k in range(meta["n_randint"])]
    return Case(name, meta, z, state, idx)


def informer_oracle_config(cfg: dict, lsq_bits=None, stack=True):
    """Effective oracle flags for the callers' 19/20-positional-argument construction."""
    from oracle.informer_np import InformerConfig

    return InformerConfig(enc_in=cfg["enc_in"], dec_in=cfg["dec_in"], c_out=cfg["c_out"], seq_len=cfg["seq_len"],
                          label_len=cfg["label_len"], pred_len=cfg["pred_len"], factor=cfg["factor"],
                          d_model=cfg["d_model"], n_heads=cfg["n_heads"], e_layers=tuple(cfg["e_layers"]) if stack else (int(cfg["e_layers"]),),
                          d_layers=cfg["d_layers"], d_ff=cfg["d_ff"], attn=cfg["attn"],
                          activation="gelu" if cfg["output_attention"] != "relu" else "relu",
                          output_attention=bool(cfg["distil"]), distil=True, mix=True, stack=stack,
                          lsq_bits=lsq_bits)


def oracle_for(case: Case, dtype=np.float64):
    from oracle.informer_np import InformerOracle
    from oracle.transformer_np import TransformerConfig, TransformerOracle

    cfg = case.cfg
    if case.meta["model"] == "transformer":
        tc = TransformerConfig(16, 16, cfg["seq_len"], cfg["pred_len"], cfg["label_len"], cfg["d_model"],
                               cfg["d_layers"], cfg["n_heads"], cfg["d_ff"])
        return TransformerOracle(tc, case.state, dtype)
    bits = cfg.get("num_bits") if case.meta["model"] == "informer_lsq" else None
    return InformerOracle(informer_oracle_config(cfg, bits, stack=case.meta["model"] != "informer"), case.state,
                          dtype)


def rel_nmse(a, b):
    """``Σ(a-b)² / Σb²`` — the parity metric of the north star (relative fp32 NMSE)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.sum((a - b) ** 2) / np.sum(b ** 2))
