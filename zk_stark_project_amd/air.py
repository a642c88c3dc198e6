"""AIR descriptions mirrored from the reference (public inputs + metadata).

The constraint arithmetic itself runs on the GPU (csrc/kernels.hip);
these classes carry what `Air::new` / `get_assertions` / `to_elements` carry
in the reference so callers build identical public inputs.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from .field import P
from .helper import AC, FE

AIR_MIMC = 1
AIR_GLOBAL_UPDATE = 2
AIR_TRAINING_UPDATE = 3

D_STATE = AC * FE + AC  # 60 (src/aggregation/air.rs:94)


@dataclass
class Assertion:
    """winterfell `Assertion::single(column, step, value)`."""
    column: int
    step: int
    value: int


# --------------------------------------------------------------------- MiMC
@dataclass
class MimcInputs:
    """Public inputs of the builder-defined MiMC AIR."""
    seed: int
    result: int

    def to_elements(self):
        return [self.seed % P, self.result % P]


class MimcAir:
    """x' = (x + K)^7 with K the 64-cycle periodic column `get_round_constants()`
    (src/helper.rs:213-217, 404-406); assertions at rows 0 and n-1."""
    AIR_ID = AIR_MIMC
    WIDTH = 1
    TRANSITION_DEGREE = 7
    CYCLE = 64

    def __init__(self, trace_length: int, pub_inputs: MimcInputs, options):
        if trace_length < 64 or trace_length & (trace_length - 1):
            raise ValueError("MiMC AIR needs a power-of-two trace length >= 64")
        self.trace_length = trace_length
        self.pub_inputs = pub_inputs
        self.options = options

    def get_assertions(self):
        return [Assertion(0, 0, self.pub_inputs.seed),
                Assertion(0, self.trace_length - 1, self.pub_inputs.result)]


# --------------------------------------------------------------- aggregation
@dataclass
class GlobalUpdateInputs:
    """src/aggregation/air.rs:14-81."""
    global_w: list
    global_b: list
    new_global_w: list
    new_global_b: list
    k: int
    digest: int
    steps: int

    def to_elements(self):
        """air.rs:57-81 — 123 elements; k is element 120."""
        e = []
        for i in range(AC):
            for j in range(FE):
                e.append(self.global_w[i][j])
        for i in range(AC):
            e.append(self.global_b[i])
        for i in range(AC):
            for j in range(FE):
                e.append(self.new_global_w[i][j])
        for i in range(AC):
            e.append(self.new_global_b[i])
        e.append(self.k)
        e.append(self.digest)
        e.append(self.steps % P)
        return e

    def to_bytes(self) -> bytes:
        """`Serializable::write_into` (air.rs:33-55): the same 123 felts, 16 B LE each."""
        return b"".join(int(v).to_bytes(16, "little") for v in self.to_elements())


class GlobalUpdateAir:
    """src/aggregation/air.rs:89-151: width 2d = 120, d = 60 degree-1 transition
    constraints `k*next[i] - k*cur[i] - next[i+d]`, 2d assertions at row steps-1."""
    AIR_ID = AIR_GLOBAL_UPDATE
    WIDTH = 2 * D_STATE
    TRANSITION_DEGREE = 1
    CYCLE = 0

    def __init__(self, trace_length: int, pub_inputs: GlobalUpdateInputs, options):
        self.trace_length = trace_length
        self.pub_inputs = pub_inputs
        self.options = options

    def get_assertions(self):
        final = [self.pub_inputs.new_global_w[i][j] for i in range(AC) for j in range(FE)]
        final += list(self.pub_inputs.new_global_b)
        last = self.pub_inputs.steps - 1
        out = [Assertion(i, last, final[i]) for i in range(D_STATE)]
        out += [Assertion(i, last, 0) for i in range(D_STATE, 2 * D_STATE)]
        return out


# ------------------------------------------------------------------ training
TU_STATE = 2 * (AC * FE + AC)   # 120: flattened [v, s] pairs (src/training/prover.rs:98-103)
TU_WIDTH = 2 * TU_STATE         # 240: masked state || masks


@dataclass
class TrainingUpdateInputs:
    """src/training/air.rs:18-99."""
    initial_masked: list
    final_masked: list
    steps: int
    x_batch: list        # BS x FE
    y_batch: list        # BS x AC
    learning_rate: int
    precision: int
    batch_size: int

    def to_elements(self):
        """air.rs:74-98: initial || final || f64(steps) || f64(bs) || x || y || lr || precision."""
        from .helper import f64_to_felt
        e = list(self.initial_masked) + list(self.final_masked)
        e.append(f64_to_felt(float(self.steps)))
        e.append(f64_to_felt(float(self.batch_size)))
        for row in self.x_batch:
            e.extend(row)
        for row in self.y_batch:
            e.extend(row)
        e.append(self.learning_rate)
        e.append(self.precision)
        return e

    def to_bytes(self) -> bytes:
        """`Serializable::write_into` (air.rs:38-70): the same elements, 16 B LE each."""
        return b"".join(int(v).to_bytes(16, "little") for v in self.to_elements())


class TrainingUpdateAir:
    """src/training/air.rs:101-292: width 240, 240 degree-1 transition constraints
    that evaluate to zero (current_step() == 0), masked state asserted
    at row 0 and row trace_length - 1 (240 assertions)."""
    AIR_ID = AIR_TRAINING_UPDATE
    WIDTH = TU_WIDTH
    TRANSITION_DEGREE = 1
    CYCLE = 0

    def __init__(self, trace_length: int, pub_inputs: TrainingUpdateInputs, options):
        if len(pub_inputs.x_batch) != pub_inputs.batch_size or len(pub_inputs.y_batch) != pub_inputs.batch_size:
            raise ValueError("batch data does not match batch_size in public inputs")  # air.rs:120-123
        self.trace_length = trace_length
        self.pub_inputs = pub_inputs
        self.options = options

    def get_assertions(self):
        half = self.WIDTH // 2
        last = self.trace_length - 1
        out = [Assertion(i, 0, self.pub_inputs.initial_masked[i]) for i in range(half)]
        out += [Assertion(i, last, self.pub_inputs.final_masked[i]) for i in range(half)]
        return out
