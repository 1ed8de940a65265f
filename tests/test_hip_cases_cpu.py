"""CPU check of the test-side restatement of the on-device dropout generator (tests/hip_cases.py):
its vectorised uint32 arithmetic equals a scalar Python restatement of eegnet_common.h keep_mul."""

from __future__ import annotations

import numpy as np

from hip_cases import device_masks, mix_key


def _keep_scalar(idx, key, pthr):
    m = 0xFFFFFFFF
    h = (idx * 0x9E3779B1 + key) & m
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & m
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & m
    h ^= h >> 16
    return int((h >> 8) >= pthr)


def test_generator_restatement_matches_scalar():
    B, F2, T, p = 3, 16, 257, 0.25
    seed, off = 0xDEADBEEF1234, 99
    m2, m3 = device_masks(B, F2, T, seed, off, p)
    key = mix_key(seed, off)
    k0, k1 = key & 0xFFFFFFFF, ((key >> 32) ^ 0x5BD1E995) & 0xFFFFFFFF
    pthr = int(p * 16777216)
    T1, T2 = T // 4, T // 32
    for b, o, q in [(0, 0, 0), (2, 15, T1 - 1), (1, 7, 33)]:
        assert m2[b, o, q] == _keep_scalar((b * F2 + o) * T1 + q, k0, pthr)
    for b, o, t in [(0, 0, 0), (2, 15, T2 - 1), (1, 3, 5)]:
        assert m3[b, o, t] == _keep_scalar(b * F2 * T2 + o * T2 + t, k1, pthr)
    assert abs(m2.mean() - 0.75) < 0.05
