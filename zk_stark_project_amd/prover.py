"""Host-side mirror of the reference's `Prover` plug-ins.

`GlobalUpdateProver` follows /root/reference/src/aggregation/prover.rs:15-249
(same constructor arguments, trace construction and public inputs);
`MimcProver` is the prover for the builder-defined MiMC AIR (SURVEY.md
Appendix B). `prove(trace)` hands the trace to libzkp.so (HIP, gfx950) through
the C-ABI in include/zkp.h — there is no CPU fallback.
"""
from __future__ import annotations

import secrets

import numpy as np

from . import _native
from .air import (AIR_GLOBAL_UPDATE, AIR_MIMC, D_STATE, GlobalUpdateAir, GlobalUpdateInputs,
                  MimcAir, MimcInputs)
from .field import P, inv, pack, unpack
from .helper import AC, FE, get_round_constants, mimc_hash_matrix
from .options import ProofOptions


class TraceTable:
    """winterfell `TraceTable<Felt>` (column-major). Storage: uint64 array of
    shape (width, length, 2) = canonical 16-byte LE felts, exactly the C-ABI layout."""

    MIN_TRACE_LENGTH = 8
    MAX_TRACE_WIDTH = 255

    def __init__(self, columns: np.ndarray):
        columns = np.ascontiguousarray(columns, dtype=np.uint64)
        if columns.ndim != 3 or columns.shape[2] != 2:
            raise ValueError("trace must have shape (width, length, 2)")
        w, n, _ = columns.shape
        if not 0 < w <= self.MAX_TRACE_WIDTH:
            raise ValueError("trace width must be in [1, 255]")
        if n < self.MIN_TRACE_LENGTH or n & (n - 1):
            raise ValueError("trace length must be a power of two >= 8")
        self.data = columns

    @classmethod
    def init(cls, columns):
        """`TraceTable::init(Vec<Vec<Felt>>)` from python ints (column-major)."""
        return cls(np.stack([pack(c) for c in columns]))

    def width(self) -> int:
        return self.data.shape[0]

    def length(self) -> int:
        return self.data.shape[1]

    def get(self, col: int, row: int) -> int:
        lo, hi = self.data[col, row]
        return int(lo) | (int(hi) << 64)

    def to_bytes(self) -> bytes:
        return self.data.tobytes()


class Proof:
    """Serialized proof (≙ winterfell `Proof`; bytes ≙ `Proof::to_bytes()`)."""

    def __init__(self, data: bytes, transcript=None):
        self.data = data
        self.transcript = transcript

    def to_bytes(self) -> bytes:
        return self.data

    def __len__(self):
        return len(self.data)


class Prover:
    """Base: subclasses provide AIR_ID, get_pub_inputs(trace) and options()."""

    AIR = None

    def __init__(self, options: ProofOptions, ctx: "_native.Context | None" = None):
        self._options = options
        self._ctx = ctx

    def options(self) -> ProofOptions:
        return self._options

    def context(self) -> "_native.Context":
        if self._ctx is None:
            self._ctx = _native.Context.default()
        return self._ctx

    def get_pub_inputs(self, trace: TraceTable):
        raise NotImplementedError

    def prove(self, trace: TraceTable) -> Proof:
        """`Prover::prove(&self, trace) -> Result<Proof, ProverError>`."""
        pub = self.get_pub_inputs(trace).to_elements()
        data, transcript = self.context().prove(self.AIR.AIR_ID, trace.data, pub, self._options)
        return Proof(data, transcript)


# --------------------------------------------------------------------- MiMC
def mimc_trace_columns(seed: int, n: int) -> np.ndarray:
    """x_{i+1} = (x_i + K[i % 64])^7 (host trace builder; serial chain)."""
    return _native.mimc_trace(seed, n).reshape(1, n, 2)


class MimcProver(Prover):
    AIR = MimcAir

    def build_trace(self, seed: int, n: int) -> TraceTable:
        return TraceTable(mimc_trace_columns(seed, n))

    def get_pub_inputs(self, trace: TraceTable) -> MimcInputs:
        return MimcInputs(trace.get(0, 0), trace.get(0, trace.length() - 1))


# --------------------------------------------------------------- aggregation
def _flatten(w, b):
    out = [x for row in w for x in row]
    out.extend(b)
    return out


def _unflatten(state, ac, fe):
    return [list(state[i * fe:(i + 1) * fe]) for i in range(ac)], list(state[ac * fe:])


class GlobalUpdateProver(Prover):
    """src/aggregation/prover.rs:15-249."""

    AIR = GlobalUpdateAir

    def __init__(self, options, raw_global_w, raw_global_b, local_w, local_b, k,
                 trace_length: int | None = None, blinding=None, ctx=None):
        super().__init__(options, ctx)
        uns_padded_steps = len(local_w) + 2
        padded = max(1 << (uns_padded_steps - 1).bit_length(), 8)  # prover.rs:64
        if trace_length is not None:
            if trace_length < padded or trace_length & (trace_length - 1):
                raise ValueError("trace_length must be a power of two >= the unpadded length")
            padded = trace_length
        self.raw_global_w, self.raw_global_b = raw_global_w, raw_global_b
        self.local_w, self.local_b = local_w, local_b
        self.k = k % P
        self.trace_length = padded
        if blinding is None:  # prover.rs:68-72 — random u64 blinding
            blinding = [secrets.randbits(64) for _ in range(D_STATE)]
        self.blinding = [b % P for b in blinding]
        raw = _flatten(raw_global_w, raw_global_b)
        masked = [(r + m) % P for r, m in zip(raw, self.blinding)]
        self.masked_global_w, self.masked_global_b = _unflatten(masked, AC, FE)

    def compute_iterative_trace_augmented(self):
        """prover.rs:98-154 — the unpadded rows (padding = repeat the last row)."""
        kinv = inv(self.k)
        raw = _flatten(self.raw_global_w, self.raw_global_b)
        cur = _flatten(self.masked_global_w, self.masked_global_b)
        rows = [cur + [0] * D_STATE]
        for i in range(len(self.local_w)):
            loc = _flatten(self.local_w[i], self.local_b[i])
            upd = [(l - g) % P for g, l in zip(raw, loc)]
            cur = [(c + u * kinv) % P for c, u in zip(cur, upd)]
            rows.append(cur + upd)
        rows.append(cur + [0] * D_STATE)
        return rows

    def build_trace(self) -> TraceTable:
        """prover.rs:157-160: TraceTable::init(transpose(rows)), padded by repetition."""
        rows = self.compute_iterative_trace_augmented()
        w, n = 2 * D_STATE, self.trace_length
        packed = np.stack([pack(col) for col in zip(*rows)])  # (w, steps, 2)
        out = np.empty((w, n, 2), dtype=np.uint64)
        out[:, :len(rows)] = packed
        out[:, len(rows):] = packed[:, -1:]
        return TraceTable(out)

    def get_pub_inputs(self, trace: TraceTable | None = None) -> GlobalUpdateInputs:
        """prover.rs:163-190."""
        rows = self.compute_iterative_trace_augmented()
        steps = len(self.local_w) + 2
        final = rows[steps - 1][:D_STATE]
        new_w, new_b = _unflatten(final, AC, FE)
        digest = mimc_hash_matrix(new_w, new_b, get_round_constants())
        return GlobalUpdateInputs(self.masked_global_w, self.masked_global_b, new_w, new_b,
                                  self.k, digest, steps)
