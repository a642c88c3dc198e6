"""Host-side mirror of the reference's `Prover` plug-ins.

`GlobalUpdateProver` follows /root/reference/src/aggregation/prover.rs:15-249
and `TrainingUpdateProver` /root/reference/src/training/prover.rs:18-301
(same constructor arguments, trace construction and public inputs);
`MimcProver` is the prover for the builder-defined MiMC AIR (SURVEY.md
Appendix B). `prove(trace)` hands the trace to libzkp.so (HIP, gfx950) through
the C-ABI in include/zkp.h — there is no CPU fallback.
"""
from __future__ import annotations

import secrets

import numpy as np

from . import _native
from .air import (AIR_GLOBAL_UPDATE, AIR_MIMC, D_STATE, TU_STATE, GlobalUpdateAir, GlobalUpdateInputs,
                  MimcAir, MimcInputs, TrainingUpdateAir, TrainingUpdateInputs)
from .field import P, inv, pack, unpack
from .helper import (AC, FE, backward_propagation_layer, forward_propagation_layer, get_round_constants,
                     mimc_hash_matrix, mse_prime, split_state_with_sign)
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

    def build_trace_device(self, ctx=None, d_out=None):
        """build_trace() on the GPU (zkp_build_global_update_trace): returns the device
        pointer of the 120 x n column-major trace in HBM (caller frees it with
        ctx.free; d_out = an existing allocation of 120 * n * 16 bytes to reuse) and
        keeps the final state for get_pub_inputs()."""
        ctx = ctx or self.context()
        raw = _flatten(self.raw_global_w, self.raw_global_b)
        local = [_flatten(w, b) for w, b in zip(self.local_w, self.local_b)]
        n = self.trace_length
        d = d_out if d_out is not None else ctx.alloc(2 * D_STATE * n * 16)
        try:
            self._final_state = ctx.build_global_update_trace(raw, self.blinding, local, self.k, n, d)
        except Exception:
            if d_out is None:
                ctx.free(d)
            raise
        return d

    def get_pub_inputs(self, trace: TraceTable | None = None) -> GlobalUpdateInputs:
        """prover.rs:163-190 (the final state comes from the device builder when it ran)."""
        steps = len(self.local_w) + 2
        final = getattr(self, "_final_state", None)
        if final is None:
            final = self.compute_iterative_trace_augmented()[steps - 1][:D_STATE]
        new_w, new_b = _unflatten(final, AC, FE)
        digest = mimc_hash_matrix(new_w, new_b, get_round_constants())
        return GlobalUpdateInputs(self.masked_global_w, self.masked_global_b, new_w, new_b,
                                  self.k, digest, steps)


# ------------------------------------------------------------------ training
class TrainingUpdateProver(Prover):
    """src/training/prover.rs:18-301 — masked trace of `batch_size` SGD steps.

    The reference samples its masks with `thread_rng` (prover.rs:117-126,
    188-196); here they come from `mask_seed` (random when None) so a trace can
    be rebuilt for parity tests."""

    AIR = TrainingUpdateAir

    def __init__(self, options, initial_w, initial_b, w_sign, b_sign, x_batch, x_batch_sign, y_batch,
                 learning_rate, precision, batch_size, mask_seed=None, ctx=None):
        super().__init__(options, ctx)
        if not (len(x_batch) == len(x_batch_sign) == len(y_batch) == batch_size):
            raise ValueError("batch data does not match batch_size")  # prover.rs:57-59
        ac, fe = len(initial_b), len(initial_w[0])
        state_cells = ac * fe + ac
        self.initial_w, self.initial_b = initial_w, initial_b
        self.w_sign, self.b_sign = w_sign, b_sign
        self.x_batch, self.x_batch_sign, self.y_batch = x_batch, x_batch_sign, y_batch
        self.learning_rate, self.precision = learning_rate % P, precision % P
        self.batch_size = batch_size
        self.trace_length = max(1 << (2 * state_cells * batch_size - 1).bit_length(), 16)  # prover.rs:63
        self.mask_seed = secrets.randbits(63) if mask_seed is None else mask_seed
        self._raw_rows = None

    def _raw_states(self):
        """The unmasked flattened state [v0,s0,v1,s1,...] after each processed sample."""
        if self._raw_rows is None:
            ac, fe = len(self.initial_b), len(self.initial_w[0])
            raw = []
            for row, srow in zip(self.initial_w, self.w_sign):
                for v, s in zip(row, srow):
                    raw += [v % P, s % P]
            for v, s in zip(self.initial_b, self.b_sign):
                raw += [v % P, s % P]
            states = [raw]
            for step in range(1, self.batch_size + 1):  # prover.rs:139-181
                w, b, ws, bs = split_state_with_sign(raw, ac, fe)
                k = step - 1
                out, out_s = forward_propagation_layer(w, b, self.x_batch[k], ws, bs, self.x_batch_sign[k],
                                                       self.precision)
                err, err_s = mse_prime(self.y_batch[k], out, out_s, self.precision)
                w2, b2, w2s, b2s = backward_propagation_layer(w, b, self.x_batch[k], err, self.learning_rate,
                                                              self.precision, ws, bs, self.x_batch_sign[k],
                                                              err_s)
                raw = []
                for rv, sv in zip(w2, w2s):
                    for v, s in zip(rv, sv):
                        raw += [v, s]
                for v, s in zip(b2, b2s):
                    raw += [v, s]
                states.append(raw)
            self._raw_rows = states
        return self._raw_rows

    def build_trace(self) -> TraceTable:
        """prover.rs:90-218: row t = [raw_t + mask_t || mask_t]; raw stops changing after batch_size."""
        n, half = self.trace_length, TU_STATE
        states = self._raw_states()
        rng = np.random.default_rng(self.mask_seed)
        masks = rng.integers(0, 1 << 64, size=(n, half), dtype=np.uint64, endpoint=False)
        cols = np.zeros((2 * half, n, 2), dtype=np.uint64)
        cols[half:, :, 0] = masks.T
        for t in range(n):
            raw = states[min(t, len(states) - 1)]
            mrow = masks[t].tolist()
            cols[:half, t] = pack([(r + m) % P for r, m in zip(raw, mrow)])
        return TraceTable(cols)

    def get_pub_inputs(self, trace: TraceTable) -> TrainingUpdateInputs:
        """prover.rs:236-270."""
        half = trace.width() // 2
        rows = trace.length()
        return TrainingUpdateInputs(
            [trace.get(c, 0) for c in range(half)], [trace.get(c, rows - 1) for c in range(half)],
            self.trace_length - 1, [list(r) for r in self.x_batch], [list(r) for r in self.y_batch],
            self.learning_rate, self.precision, self.batch_size)


# ------------------------------------------------------------------ verifier
def verify(air, proof, pub_inputs, acceptable_options) -> None:
    """`winterfell::verify::<AIR, Blake3_256, DefaultRandomCoin, MerkleTree>(proof, pub_inputs,
    &AcceptableOptions::OptionSet(..))` as called at /root/reference/src/main.rs:251-257, 430-436, 478-484.

    `air` is an AIR class (MimcAir, GlobalUpdateAir, TrainingUpdateAir) or its id; `proof` a Proof or
    its bytes; `pub_inputs` an inputs object (to_elements()) or the element list; `acceptable_options`
    a ProofOptions or a list of them (OptionSet). Raises `_native.VerifierError` on rejection. Runs in
    libzkp.so on the host (no device needed)."""
    air_id = air if isinstance(air, int) else air.AIR_ID
    data = proof.to_bytes() if isinstance(proof, Proof) else bytes(proof)
    pub = pub_inputs.to_elements() if hasattr(pub_inputs, "to_elements") else list(pub_inputs)
    opts = acceptable_options if isinstance(acceptable_options, (list, tuple)) else [acceptable_options]
    last = None
    for o in opts:
        try:
            _native.verify(air_id, data, pub, o)
            return
        except _native.VerifierError as e:
            last = e
            if e.kind != "UnacceptableProofOptions":
                raise
    raise last
