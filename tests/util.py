"""Shared test helpers: the seeded splitmix64 byte generator used by the golden fixtures,
the parity tests, smoke() and bench.py ("all use a seeded splitmix64 PRNG")."""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(seed: int, n: int) -> bytes:
    """concat_i LE64(mix(seed + (i+1)*golden)), truncated to n bytes."""
    if n <= 0:
        return b""
    k = (n + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(1, k + 1, dtype=np.uint64) * _GOLDEN + np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    return _mix(idx).astype("<u8").tobytes()[:n]


def splitmix_array(seed: int, n: int) -> np.ndarray:
    return np.frombuffer(splitmix_bytes(seed, n), dtype=np.uint8).copy()
