"""Host-side helpers for BLS12-377 Fr element arrays.

Elements live in numpy ``uint64`` arrays of shape (..., 4): little-endian
limbs in Montgomery form (R = 2^256) -- ark-ff's in-memory ``Bls12_377Fr``
(bin/src/config.rs:9) and the element format of include/lsp.h.
"""
from __future__ import annotations

import numpy as np

MODULUS = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
GENERATOR = 22
TWO_ADICITY = 47
_R = pow(2, 256, MODULUS)
_RINV = pow(_R, MODULUS - 2, MODULUS)


def to_mont(values) -> np.ndarray:
    """Python ints -> (n, 4) uint64 Montgomery limbs."""
    vals = [int(v) % MODULUS * _R % MODULUS for v in values]
    out = np.empty((len(vals), 4), dtype=np.uint64)
    raw = b"".join(v.to_bytes(32, "little") for v in vals)
    out[:] = np.frombuffer(raw, dtype=np.uint64).reshape(-1, 4) if vals else out
    return out


def from_mont(arr: np.ndarray) -> list:
    """(n, 4) uint64 Montgomery limbs -> Python ints."""
    a = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1, 4)
    raw = a.tobytes()
    return [int.from_bytes(raw[32 * i:32 * i + 32], "little") * _RINV % MODULUS for i in range(a.shape[0])]


def from_be_bytes_mod_order(b: bytes) -> int:
    """FF_Bls12_377Fr::from_be_bytes_mod_order (trace/src/permutation.rs:102)."""
    return int.from_bytes(b, "big") % MODULUS


def two_adic_generator(bits: int) -> int:
    root = pow(GENERATOR, (MODULUS - 1) >> TWO_ADICITY, MODULUS)
    return pow(root, 1 << (TWO_ADICITY - bits), MODULUS)


def empty(n: int) -> np.ndarray:
    return np.zeros((n, 4), dtype=np.uint64)
