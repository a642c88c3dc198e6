"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; it is the checker, never the thing measured or shipped.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")


class ProofOptionsC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "num_queries", "blowup_factor", "grinding_factor", "field_extension",
        "fri_folding_factor", "fri_remainder_max_degree", "batching_constraints", "batching_deep")]


class Felt(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


class Transcript(ctypes.Structure):
    _fields_ = [
        ("trace_root", ctypes.c_uint8 * 32),
        ("constraint_root", ctypes.c_uint8 * 32),
        ("fri_roots", (ctypes.c_uint8 * 32) * 16),
        ("remainder_commitment", ctypes.c_uint8 * 32),
        ("num_fri_layers", ctypes.c_uint32),
        ("num_composition_columns", ctypes.c_uint32),
        ("pow_nonce", ctypes.c_uint64),
        ("z", Felt),
        ("num_unique_queries", ctypes.c_uint32),
        ("query_positions", ctypes.c_uint64 * 255),
    ]


class Timings(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "t_lde", "t_eval", "t_comp", "t_deep", "t_fri", "t_grind", "t_query", "t_total")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_prove.restype = ctypes.c_int
        L.oracle_prove.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64,
                                   ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ProofOptionsC),
                                   ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(Transcript), ctypes.POINTER(Timings)]
        L.oracle_verify.restype = ctypes.c_int
        L.oracle_verify.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                    ctypes.c_uint64, ctypes.POINTER(ProofOptionsC)]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_blake3.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_f128_op.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_root_of_unity.argtypes = [ctypes.c_uint, ctypes.c_char_p]
        L.oracle_mimc_cipher.argtypes = [ctypes.c_char_p] * 4
        L.oracle_mimc_trace.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_trace_lde.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                       ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_merkle_rows.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_grind.restype = ctypes.c_uint64
        L.oracle_grind.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_set_threads.restype = None
        L.oracle_mimc_hash_matrix.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p,
                                              ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p]
        L.oracle_mimc_hash_matrix.restype = None
        L.oracle_gu_trace.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64,
                                      ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_gu_trace.restype = ctypes.c_int
        L.oracle_time_mimc_cipher.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_time_mimc_cipher.restype = ctypes.c_double
        L.oracle_time_mimc_hash_matrix.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                                                   ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32,
                                                   ctypes.c_uint64, ctypes.c_char_p]
        L.oracle_time_mimc_hash_matrix.restype = ctypes.c_double
        _lib = L
    return _lib


def fb(v: int) -> bytes:
    return int(v).to_bytes(16, "little")


def opts_c(o) -> ProofOptionsC:
    return ProofOptionsC(o.num_queries, o.blowup_factor, o.grinding_factor, o.field_extension,
                         o.fri_folding_factor, o.fri_remainder_max_degree,
                         o.batching_constraints, o.batching_deep)


def prove(air_id: int, trace_cols: bytes, width: int, n: int, pub: bytes, opts, timings=False):
    L = lib()
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    tr = Transcript()
    tm = Timings()
    oc = opts_c(opts)
    rc = L.oracle_prove(air_id, trace_cols, width, n, pub, len(pub) // 16, ctypes.byref(oc),
                        ctypes.byref(out), ctypes.byref(olen), ctypes.byref(tr), ctypes.byref(tm))
    if rc != 0:
        raise RuntimeError(f"oracle_prove failed: {rc}")
    proof = ctypes.string_at(out, olen.value)
    L.oracle_free(out)
    if timings:
        return proof, tr, tm
    return proof, tr


def verify(air_id: int, proof: bytes, pub: bytes, opts) -> int:
    oc = opts_c(opts)
    return lib().oracle_verify(air_id, proof, len(proof), pub, len(pub) // 16, ctypes.byref(oc))


def blake3(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_blake3(data, len(data), out)
    return out.raw


def f128(op: str, a: int, b: int = 0) -> int:
    code = {"add": 0, "sub": 1, "mul": 2, "inv": 3, "exp": 4, "new": 5}[op]
    out = ctypes.create_string_buffer(16)
    lib().oracle_f128_op(code, a.to_bytes(16, "little"), b.to_bytes(16, "little"), out)
    return int.from_bytes(out.raw, "little")


def root_of_unity(log_n: int) -> int:
    out = ctypes.create_string_buffer(16)
    lib().oracle_root_of_unity(log_n, out)
    return int.from_bytes(out.raw, "little")


def mimc_cipher(x: int, rc: int, z: int) -> int:
    out = ctypes.create_string_buffer(16)
    lib().oracle_mimc_cipher(fb(x), fb(rc), fb(z), out)
    return int.from_bytes(out.raw, "little")


def mimc_trace(x0: int, n: int) -> bytes:
    out = ctypes.create_string_buffer(16 * n)
    lib().oracle_mimc_trace(fb(x0), n, out)
    return out.raw


def trace_lde(trace_cols: bytes, width: int, n: int, blowup: int):
    lde = ctypes.create_string_buffer(16 * width * n * blowup)
    root = ctypes.create_string_buffer(32)
    lib().oracle_trace_lde(trace_cols, width, n, blowup, lde, root)
    return lde.raw, root.raw


def merkle_rows(cols: bytes, width: int, rows: int) -> bytes:
    root = ctypes.create_string_buffer(32)
    lib().oracle_merkle_rows(cols, width, rows, root)
    return root.raw


def grind(seed: bytes, bits: int) -> int:
    return lib().oracle_grind(seed, bits)


def felts_from_bytes(b: bytes):
    a = np.frombuffer(b, dtype="<u8").reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in a]


class Stages(ctypes.Structure):
    """oracle_stages (oracle/stark_oracle.c): stage values of one oracle proof."""
    _fields_ = [("coeffs", ctypes.c_void_p), ("comp_evals", ctypes.c_void_p), ("ood", ctypes.c_void_p),
                ("deep_coeffs", ctypes.c_void_p), ("alphas", ctypes.c_void_p), ("remainder", ctypes.c_void_p),
                ("n_coeffs", ctypes.c_uint32), ("n_layers", ctypes.c_uint32), ("n_remainder", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


def prove_stages(air_id: int, trace_cols: bytes, width: int, n: int, pub: bytes, opts, ce: int, C: int):
    """Oracle proof + its stage values: dict of byte strings (16 B LE felts) keyed
    coeffs, comp_evals (n*ce, natural CE order), ood (2w + C), deep_coeffs (w + C),
    alphas (one per FRI layer), remainder."""
    L = lib()
    L.oracle_prove_stages.restype = ctypes.c_int
    L.oracle_prove_stages.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64,
                                      ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ProofOptionsC),
                                      ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(Stages)]
    bufs = {"coeffs": ctypes.create_string_buffer(16 * 1024), "comp_evals": ctypes.create_string_buffer(16 * n * ce),
            "ood": ctypes.create_string_buffer(16 * (2 * width + C)),
            "deep_coeffs": ctypes.create_string_buffer(16 * (width + C)),
            "alphas": ctypes.create_string_buffer(16 * 16), "remainder": ctypes.create_string_buffer(16 * 256)}
    sd = Stages(*[ctypes.cast(bufs[k], ctypes.c_void_p) for k in
                  ("coeffs", "comp_evals", "ood", "deep_coeffs", "alphas", "remainder")], 0, 0, 0, 0)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    oc = opts_c(opts)
    rc = L.oracle_prove_stages(air_id, trace_cols, width, n, pub, len(pub) // 16, ctypes.byref(oc),
                               ctypes.byref(out), ctypes.byref(olen), ctypes.byref(sd))
    if rc != 0:
        raise RuntimeError(f"oracle_prove_stages failed: {rc}")
    proof = ctypes.string_at(out, olen.value)
    L.oracle_free(out)
    res = {"coeffs": bufs["coeffs"].raw[:16 * sd.n_coeffs], "comp_evals": bufs["comp_evals"].raw,
           "ood": bufs["ood"].raw, "deep_coeffs": bufs["deep_coeffs"].raw,
           "alphas": bufs["alphas"].raw[:16 * sd.n_layers], "remainder": bufs["remainder"].raw[:16 * sd.n_remainder]}
    return proof, res


def mimc_hash_matrix(w, b, rc) -> int:
    """helper.rs:222-233 on the oracle (C)."""
    out = ctypes.create_string_buffer(16)
    wb = b"".join(fb(v) for row in w for v in row)
    lib().oracle_mimc_hash_matrix(wb, len(w), len(w[0]) if w else 0, b"".join(fb(v) for v in b),
                                  b"".join(fb(v) for v in rc), len(rc), out)
    return int.from_bytes(out.raw, "little")


def gu_trace(raw, blinding, local, k: int, n: int):
    """GlobalUpdateProver trace (src/aggregation/prover.rs:98-160) on the oracle:
    -> (column-major 120 x n trace bytes, final state ints). raw/blinding: 60 ints,
    local: ndev lists of 60 ints (flattened w then b)."""
    ndev = len(local)
    out = ctypes.create_string_buffer(120 * n * 16)
    fin = ctypes.create_string_buffer(60 * 16)
    rc = lib().oracle_gu_trace(b"".join(fb(v) for v in raw), b"".join(fb(v) for v in blinding),
                               b"".join(fb(v) for row in local for v in row) or b"\0" * 16, ndev, fb(k), n,
                               out, fin)
    if rc != 0:
        raise ValueError("oracle_gu_trace: n < ndev + 2")
    return out.raw, [int.from_bytes(fin.raw[16 * i:16 * i + 16], "little") for i in range(60)]


def time_mimc_cipher(x: int, rc: int, iters: int):
    """C1 mimc_cipher timing (one host thread): (seconds per call, chained output)."""
    out = ctypes.create_string_buffer(16)
    sec = lib().oracle_time_mimc_cipher(fb(x), fb(rc), iters, out)
    return sec, int.from_bytes(out.raw, "little")


def time_mimc_hash_matrix(w, b, rc, iters: int):
    """C1 mimc_hash_matrix timing (one host thread): (seconds per call, last digest)."""
    out = ctypes.create_string_buffer(16)
    sec = lib().oracle_time_mimc_hash_matrix(b"".join(fb(v) for row in w for v in row), len(w), len(w[0]),
                                             b"".join(fb(v) for v in b), b"".join(fb(v) for v in rc), len(rc),
                                             iters, out)
    return sec, int.from_bytes(out.raw, "little")
