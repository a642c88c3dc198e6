"""MI355X-native STARK prover for the winterfell-based AIRs of
FireMines/zk_stark_project (HIP/gfx950 kernels behind include/zkp.h)."""
from .field import P, GENERATOR, TWO_ADICITY
from .options import ProofOptions, FieldExtension, BatchingMethod
from .air import (MimcAir, MimcInputs, GlobalUpdateAir, GlobalUpdateInputs, TrainingUpdateAir,
                  TrainingUpdateInputs, AIR_MIMC, AIR_GLOBAL_UPDATE, AIR_TRAINING_UPDATE)
from .prover import TraceTable, Proof, Prover, MimcProver, GlobalUpdateProver, TrainingUpdateProver, verify
from ._native import VerifierError
from . import helper

__all__ = ["P", "GENERATOR", "TWO_ADICITY", "ProofOptions", "FieldExtension", "BatchingMethod",
           "MimcAir", "MimcInputs", "GlobalUpdateAir", "GlobalUpdateInputs", "AIR_MIMC",
           "AIR_GLOBAL_UPDATE", "AIR_TRAINING_UPDATE", "TraceTable", "Proof", "Prover",
           "MimcProver", "GlobalUpdateProver", "TrainingUpdateAir", "TrainingUpdateInputs",
           "TrainingUpdateProver", "helper", "verify", "VerifierError"]
