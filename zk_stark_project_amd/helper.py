"""Host-side mirror of the parts of /root/reference/src/helper.rs that feed the
proving path (trace building and public inputs). These are trace-construction
helpers that run on the host in the reference too; they are not the hot path.
"""
from __future__ import annotations

import math

from .field import P, felt_new

# src/helper.rs:18-22
AC = 6   # number of activations
FE = 9   # features per activation
C = 8    # number of clients
MAX = (1 << 128) - 1  # helper.rs:15 (u128::MAX)


def f64_to_felt(x: float) -> int:
    """helper.rs:25-27 — `Felt::new((x * 1e6).round() as u128)`.

    Rust `f64::round` rounds half away from zero; `as u128` saturates
    (negative and NaN -> 0; overflow -> u128::MAX), then `Felt::new` reduces."""
    y = x * 1e6
    if y != y or y <= 0:          # NaN, negatives and -0.0 saturate to 0
        return 0
    if math.isinf(y) or y >= 2.0**128:
        return felt_new(MAX)
    r = math.floor(y)
    if y - r >= 0.5:              # exact for floats: half away from zero
        r += 1
    return felt_new(int(r))


def encode_signed(x: int) -> tuple[int, int]:
    """helper.rs:38-45 — (value, sign) with negatives as u128::MAX - |x| + 1 (mod p)."""
    if x >= 0:
        return felt_new(x), 0
    return felt_new((MAX - (-x) + 1) & MAX), 1


def transpose(matrix):
    """helper.rs:197-211 — row-major Vec<Vec<Felt>> -> column-major."""
    if not matrix:
        return []
    cols = len(matrix[0])
    for row in matrix:
        assert len(row) == cols, "All rows must have equal length"
    return [[row[j] for row in matrix] for j in range(cols)]


def get_round_constants():
    """helper.rs:404-406."""
    return [f64_to_felt(float(i)) for i in range(1, 65)]


def mimc_cipher(inp: int, round_constant: int, z: int) -> int:
    """helper.rs:213-220 — 64 rounds of x <- (x + rc + z)^7, returns x + z."""
    x = inp
    for _ in range(64):
        x = pow((x + round_constant + z) % P, 7, P)
    return (x + z) % P


def mimc_hash_matrix(w, b, round_constants) -> int:
    """helper.rs:222-233."""
    z = f64_to_felt(0.0)
    n = len(round_constants)
    for i in range(len(w)):
        for j in range(len(w[i])):
            z = mimc_cipher(w[i][j], round_constants[j % n], z)
        z = mimc_cipher(b[i], round_constants[i % n], z)
    return z
