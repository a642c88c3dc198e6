"""winterfell 0.12 `ProofOptions` mirror (validated like `ProofOptions::new`).

The reference's parameter set is
`ProofOptions::new(40, 16, 21, FieldExtension::None, 16, 7, Algebraic, Algebraic)`
(/root/reference/src/main.rs:98-107; also tests/integration_tests.rs:69-75).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from enum import IntEnum


class FieldExtension(IntEnum):
    NONE = 1
    QUADRATIC = 2
    CUBIC = 3


class BatchingMethod(IntEnum):
    LINEAR = 0
    ALGEBRAIC = 1
    HORNER = 2


class ProofOptionsC(ctypes.Structure):
    """`zkp_proof_options` from include/zkp.h."""
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "num_queries", "blowup_factor", "grinding_factor", "field_extension",
        "fri_folding_factor", "fri_remainder_max_degree", "batching_constraints", "batching_deep")]


@dataclass(frozen=True)
class ProofOptions:
    num_queries: int
    blowup_factor: int
    grinding_factor: int
    field_extension: int = FieldExtension.NONE
    fri_folding_factor: int = 16
    fri_remainder_max_degree: int = 7
    batching_constraints: int = BatchingMethod.ALGEBRAIC
    batching_deep: int = BatchingMethod.ALGEBRAIC

    def __post_init__(self):
        # ProofOptions::new assertions (winter-air 0.12)
        if not 0 < self.num_queries <= 255:
            raise ValueError("number of queries must be in [1, 255]")
        b = self.blowup_factor
        if b < 2 or b > 128 or b & (b - 1):
            raise ValueError("blowup factor must be a power of two in [2, 128]")
        if self.grinding_factor > 32:
            raise ValueError("grinding factor cannot exceed 32")
        if self.fri_folding_factor not in (2, 4, 8, 16):
            raise ValueError("FRI folding factor must be 2, 4, 8 or 16")
        r = self.fri_remainder_max_degree
        if r > 255 or (r + 1) & r:
            raise ValueError("FRI remainder max degree must be one less than a power of two")

    @classmethod
    def reference(cls) -> "ProofOptions":
        """/root/reference/src/main.rs:98-107."""
        return cls(40, 16, 21, FieldExtension.NONE, 16, 7, BatchingMethod.ALGEBRAIC, BatchingMethod.ALGEBRAIC)

    def with_blowup(self, blowup: int) -> "ProofOptions":
        return ProofOptions(self.num_queries, blowup, self.grinding_factor, self.field_extension,
                            self.fri_folding_factor, self.fri_remainder_max_degree,
                            self.batching_constraints, self.batching_deep)

    def to_c(self) -> ProofOptionsC:
        return ProofOptionsC(self.num_queries, self.blowup_factor, self.grinding_factor,
                             int(self.field_extension), self.fri_folding_factor,
                             self.fri_remainder_max_degree, int(self.batching_constraints),
                             int(self.batching_deep))
