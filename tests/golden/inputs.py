"""Deterministic inputs shared by the golden generator and the tests (numpy PCG64 seeds).

Inputs are regenerated, never stored, so the fixtures stay KB-sized.
"""

from __future__ import annotations

import numpy as np


def make_inputs(B: int, C: int, T: int, seed: int):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, C, T), dtype=np.float32)
    y = rng.integers(0, 4, size=B, dtype=np.int64)
    return x, y


def make_masks(B: int, F2: int, T: int, seed: int, p: float):
    """Keep-masks for the two dropout layers: [B,F2,T//4] and [B,F2,(T//4)//8], uint8 (1 = keep)."""
    rng = np.random.default_rng(10_000 + seed)
    T1 = T // 4
    T2 = T1 // 8
    m2 = (rng.random((B, F2, T1)) >= p).astype(np.uint8)
    m3 = (rng.random((B, F2, T2)) >= p).astype(np.uint8)
    return m2, m3
