"""ProbSparse index sampling with the reference's RNG protocol.

The reference draws ``index_sample = torch.randint(L_K, (L_Q, U_part))`` from the
GLOBAL torch CPU generator once per ProbAttention call, in forward order
(``FullPrecision/InformerModel/attn.py:96-98``).  torch's CPU
``randint`` is ``mt19937() % range`` drawn sequentially, so:

* :func:`draw_indices` with ``seed=None`` consumes the global generator exactly
  as the reference forward would (drop-in parity with callers that seed torch);
* with a ``seed`` it uses a private generator;
* the engine's native sampler (``cet_seed`` in the C ABI, an mt19937 in C++)
  reproduces the same stream without Python — tested against this module.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


def draw_indices(shapes: Sequence[Tuple[int, Tuple[int, int]]], seed: Optional[int] = None,
                 generator=None) -> List[np.ndarray]:
    """One ``randint(L_K, (L_Q, U))`` per entry of ``shapes`` → int32 arrays."""
    import torch

    if seed is not None:
        generator = torch.Generator().manual_seed(int(seed))
    out = []
    for lk, shp in shapes:
        if generator is None:
            r = torch.randint(int(lk), tuple(shp))
        else:
            r = torch.randint(int(lk), tuple(shp), generator=generator)
        out.append(r.numpy().astype(np.int32))
    return out
