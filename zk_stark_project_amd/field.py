"""f128 field constants and host-side packing helpers.

winter-math 0.12 `fields::f128::BaseElement` (reference: src/aggregation/air.rs:10):
p = 2^128 - 45*2^40 + 1, GENERATOR = 3, TWO_ADICITY = 40.
Elements cross the C-ABI as 16-byte canonical little-endian values; in numpy
they are `(..., 2)` arrays of little-endian uint64 [lo, hi].
"""
from __future__ import annotations

import numpy as np

P = 2**128 - 45 * 2**40 + 1
GENERATOR = 3
TWO_ADICITY = 40
ELEMENT_BYTES = 16
_MASK64 = (1 << 64) - 1


def felt_new(v: int) -> int:
    """`BaseElement::new(u128)`: reduce a u128 by one conditional subtraction."""
    v &= (1 << 128) - 1
    return v - P if v >= P else v


def inv(a: int) -> int:
    """winter-math `inv` (inv(0) = 0)."""
    return 0 if a % P == 0 else pow(a, P - 2, P)


def to_bytes(vals) -> bytes:
    return b"".join(int(v).to_bytes(16, "little") for v in vals)


def from_bytes(b: bytes) -> list[int]:
    a = np.frombuffer(b, dtype="<u8").reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in a]


def pack(vals) -> np.ndarray:
    """list of ints -> (len, 2) uint64 array."""
    out = np.empty((len(vals), 2), dtype=np.uint64)
    for i, v in enumerate(vals):
        v = int(v)
        out[i, 0] = v & _MASK64
        out[i, 1] = v >> 64
    return out


def unpack(a: np.ndarray) -> list[int]:
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in a]
