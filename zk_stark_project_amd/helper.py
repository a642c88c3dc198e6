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


# --------------------------------------------------------------------------
# signed fixed-point arithmetic over the field (src/signed.rs), used by the
# training trace builder. Semantics are reproduced exactly, including
# sub_generic(a, 0, b, 0) returns a + b.
SIGNED_MAX = felt_new(MAX)  # signed.rs:3 Felt::new(u128::MAX)


def _cleanse(v: int, s: int) -> int:
    """signed.rs:11-14."""
    return ((1 - s) * v + s * (SIGNED_MAX - v + 1)) % P


def add_generic(a: int, s_a: int, b: int, s_b: int) -> tuple[int, int]:
    """signed.rs:16-25."""
    a_c, b_c = _cleanse(a, s_a), _cleanse(b, s_b)
    ind = s_a * s_b % P
    c = (ind * (SIGNED_MAX + 1 - a_c - b_c) + (1 - ind) * (a + b)) % P
    return c, ind


def sub_generic(a: int, s_a: int, b: int, s_b: int) -> tuple[int, int]:
    """signed.rs:27-30 — a + (-b), with the reference's sign handling."""
    return add_generic(a, s_a, b, (1 - s_b) % P)


def mul_generic(a: int, s_a: int, b: int, s_b: int) -> tuple[int, int]:
    """signed.rs:32-39."""
    prod = _cleanse(a, s_a) * _cleanse(b, s_b) % P
    sign = (s_a + s_b - s_a * s_b * 2) % P
    return (sign * (SIGNED_MAX - prod + 1) + (1 - sign) * prod) % P, sign


def div_generic(a: int, s_a: int, b: int, s_b: int) -> tuple[int, int]:
    """signed.rs:41-48 (field inverse; inv(0) = 0)."""
    from .field import inv
    q = _cleanse(a, s_a) * inv(_cleanse(b, s_b)) % P
    sign = (s_a + s_b - s_a * s_b * 2) % P
    return (sign * (SIGNED_MAX + 1 - q) + (1 - sign) * q) % P, sign


# felt-only wrappers (signed.rs:53-64), re-exported by helper.rs:3 as
# add / subtract / multiply / divide with argument order (a, b, s_a, s_b)
def add(a, b, s_a, s_b):
    return add_generic(a, s_a, b, s_b)


def subtract(a, b, s_a, s_b):
    return sub_generic(a, s_a, b, s_b)


def multiply(a, b, s_a, s_b):
    return mul_generic(a, s_a, b, s_b)


def divide(a, b, s_a, s_b):
    return div_generic(a, s_a, b, s_b)


def _rust_round_i128(y: float) -> int:
    """`(y).round() as i128`: half away from zero; NaN -> 0; saturating."""
    if y != y:
        return 0
    if math.isinf(y) or abs(y) >= 2.0**127:
        return (1 << 127) - 1 if y > 0 else -(1 << 127)
    r = math.floor(abs(y))
    if abs(y) - r >= 0.5:
        r += 1
    return r if y >= 0 else -r


def f64_to_signed_felt(x: float, scale: float) -> tuple[int, int]:
    """helper.rs:48-51."""
    return encode_signed(_rust_round_i128(x * scale))


def label_to_one_hot(label: float, ac: int, precision: float):
    """helper.rs:150-162."""
    v, s = [0] * ac, [0] * ac
    idx = 0 if label < 1.0 else max(int(label) - 1, 0)
    if idx < ac:
        v[idx], s[idx] = f64_to_signed_felt(precision, 1.0)
    return v, s


def split_state_with_sign(row, ac: int, fe: int):
    """helper.rs:165-195 — [v0,s0,v1,s1,...] -> (w, b, w_sign, b_sign)."""
    assert len(row) == 2 * ac * (fe + 1), "split_state_with_sign: bad row length"
    w = [[row[2 * (j * fe + i)] for i in range(fe)] for j in range(ac)]
    ws = [[row[2 * (j * fe + i) + 1] for i in range(fe)] for j in range(ac)]
    b = [row[2 * (ac * fe + j)] for j in range(ac)]
    bs = [row[2 * (ac * fe + j) + 1] for j in range(ac)]
    return w, b, ws, bs


def mse_prime(y_true, y_pred, y_pred_sign, pr):
    """helper.rs:245-269."""
    ac = len(y_true)
    ac_f = f64_to_felt(float(ac))
    res, res_s = [0] * ac, [0] * ac
    for i in range(ac):
        t, ts = subtract(y_pred[i], y_true[i], y_pred_sign[i], 0)
        t2, t2s = multiply(t, f64_to_felt(2.0), ts, 0)
        res[i], res_s[i] = divide(t2, ac_f, t2s, 0)
    return res, res_s


def forward_propagation_layer(w, b, x, w_sign, b_sign, x_sign, pr):
    """helper.rs:282-330."""
    ac, fe = len(b), len(x)
    wx, wxs = [0] * ac, [0] * ac
    for j in range(ac):
        t, ts = 0, 0
        for i in range(fe):
            ti, tis = multiply(w[j][i], x[i], w_sign[j][i], x_sign[i])
            t, ts = add(t, ti, ts, tis)
        wx[j], wxs[j] = divide(t, pr, ts, 0)
    out, out_s = [0] * ac, [0] * ac
    for j in range(ac):
        out[j], out_s[j] = add(wx[j], b[j], wxs[j], b_sign[j])
    return out, out_s


def backward_propagation_layer(w, b, x, output_error, learning_rate, pr, w_sign, b_sign, x_sign,
                               output_error_sign):
    """helper.rs:345-400 (updates in place and returns copies, like the reference)."""
    ac, fe = len(b), len(x)
    for i in range(ac):
        t, ts = divide(output_error[i], learning_rate, output_error_sign[i], 0)
        b[i], b_sign[i] = subtract(b[i], t, b_sign[i], ts)
    for j in range(fe):
        for i in range(ac):
            prod, ps = multiply(output_error[i], x[j], output_error_sign[i], x_sign[j])
            t, ts = divide(prod, learning_rate, ps, 0)
            grad, gs = divide(t, pr, ts, 0)
            w[i][j], w_sign[i][j] = subtract(w[i][j], grad, w_sign[i][j], gs)
    return [r[:] for r in w], b[:], [r[:] for r in w_sign], b_sign[:]


# ---------------------------------------------------------- CLI-side inputs
def read_dataset(file_path: str):
    """helper.rs:55-80 — CSV rows of width 46 (features = columns 18..27, label = 45)
    or 10 (features = 0..9, label = 9); unparsable cells read as 0.0."""
    import csv
    feats, labs = [], []
    with open(file_path, newline="") as fh:
        for rec in csv.reader(fh):
            if not rec:
                continue
            row = []
            for cell in rec:
                try:
                    row.append(float(cell.strip()))
                except ValueError:
                    row.append(0.0)
            if len(row) == 46:
                feats.append(row[18:27])
                labs.append(row[45])
            elif len(row) == 10:
                feats.append(row[:9])
                labs.append(row[9])
            else:
                raise ValueError(f"Unexpected CSV width {len(row)}")
    return feats, labs


class EdgeDevice:
    """helper.rs:83-106 — one device's data; next_batch samples p distinct rows."""

    def __init__(self, features, labels, rng=None):
        import random
        self.features, self.labels = features, labels
        self._rng = rng or random.Random()

    def next_batch(self, p: int):
        n = len(self.labels)
        idx = self._rng.sample(range(n), min(p, n))
        return [list(self.features[i]) for i in idx], [self.labels[i] for i in idx]


def generate_initial_model(fe: int, ac: int, sigma: float, rng=None):
    """helper.rs:108-131 — N(0, sigma) weights as (w, w_sign, b, b_sign), scale 1e6.
    The reference draws from `thread_rng`; `rng` (random.Random) makes it reproducible."""
    import random
    rng = rng or random.Random()
    w = [[0] * fe for _ in range(ac)]
    ws = [[0] * fe for _ in range(ac)]
    b, bs = [0] * ac, [0] * ac
    for j in range(ac):
        for i in range(fe):
            w[j][i], ws[j][i] = f64_to_signed_felt(rng.gauss(0.0, sigma), 1e6)
        b[j], bs[j] = f64_to_signed_felt(rng.gauss(0.0, sigma), 1e6)
    return w, ws, b, bs
