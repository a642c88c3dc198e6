"""ctypes binding of libzkp.so (the HIP/gfx950 prover behind include/zkp.h).

The library is built in-tree by __graft_entry__.build() / `make -C
zk_stark_project_amd/csrc`. There is no CPU fallback: if the library or a
gfx950 device is missing every compute call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time

import numpy as np

from .options import ProofOptions

HERE = os.path.dirname(os.path.abspath(__file__))
# ZKP_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("ZKP_LIB") or os.path.join(HERE, "libzkp.so")

ZKP_OK = 0
STATUS = {
    1: "invalid proof options", 2: "unsupported field extension", 3: "invalid trace shape",
    4: "invalid public inputs", 5: "HIP device error", 6: "grinding nonce not found",
    7: "out of device memory", 8: "unsupported AIR", 9: "invalid argument",
}


class ZkpError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"zkp error {code} ({STATUS.get(code, '?')}): {msg}")
        self.code = code


class Felt(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


class Transcript(ctypes.Structure):
    """`zkp_transcript` (include/zkp.h)."""
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

    def summary(self) -> dict:
        return {
            "trace_root": bytes(self.trace_root).hex(),
            "constraint_root": bytes(self.constraint_root).hex(),
            "fri_roots": [bytes(self.fri_roots[i]).hex() for i in range(self.num_fri_layers)],
            "remainder_commitment": bytes(self.remainder_commitment).hex(),
            "pow_nonce": int(self.pow_nonce),
            "z": int(self.z.lo) | (int(self.z.hi) << 64),
            "num_composition_columns": int(self.num_composition_columns),
            "query_positions": [int(self.query_positions[i]) for i in range(self.num_unique_queries)],
        }


# symbols declared in include/zkp.h (checked by tests/test_abi.py)
EXPORTED = [
    "zkp_ctx_create", "zkp_ctx_destroy", "zkp_last_error", "zkp_free", "zkp_prove",
    "zkp_prove_device", "zkp_device_alloc", "zkp_device_free", "zkp_copy_to_device",
    "zkp_copy_to_host", "zkp_trace_lde_commit", "zkp_merkle_commit_rows", "zkp_grind",
    "zkp_set_profiling", "zkp_kernel_stats", "zkp_reset_stats", "zkp_kernel_stats_table",
    "zkp_build_mimc_trace", "zkp_prove_sharded", "zkp_comm_local_group", "zkp_comm_rccl_unique_id",
    "zkp_comm_rccl_create", "zkp_comm_destroy", "zkp_comm_rank", "zkp_comm_world", "zkp_comm_backend_world", "zkp_comm_check",
    "zkp_prove_sharded_device",
    "zkp_verify", "zkp_build_global_update_trace", "zkp_set_profiling_kernel",
    "zkp_session_create", "zkp_session_destroy", "zkp_session_trace_lde", "zkp_eval_constraints",
    "zkp_composition_commit", "zkp_ood_frame", "zkp_deep_fri", "zkp_query", "zkp_comm_host_create",
    "zkp_session_shape",
    "zkp_channel_create", "zkp_channel_destroy", "zkp_channel_commit", "zkp_channel_commit_felts",
    "zkp_channel_draw", "zkp_channel_seed", "zkp_channel_query_positions", "zkp_ctx_trim",
]

# zkp_host_transport callbacks (include/zkp.h)
HOST_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
HOST_ABORT = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class HostTransport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("all_to_all", HOST_A2A), ("all_gather", HOST_A2A),
                ("abort", HOST_ABORT)]


# int (*zkp_fri_channel)(void* user, uint32_t layer, const uint8_t root[32], zkp_felt* alpha)
FRI_CHANNEL = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint8),
                               ctypes.c_void_p)

# zkp_verify_status (include/zkp.h) -> winter-verifier `VerifierError` variant
VERIFY_STATUS = {
    32: "InconsistentBaseField", 33: "UnacceptableProofOptions", 34: "ProofDeserializationError",
    35: "InvalidPublicInputs", 36: "InconsistentOodConstraintEvaluations",
    37: "TraceQueryDoesNotMatchCommitment", 38: "ConstraintQueryDoesNotMatchCommitment",
    39: "QuerySeedProofOfWorkVerificationFailed", 40: "FriVerificationFailed", 41: "RandomCoinError",
}


class VerifierError(ValueError):
    """winter-verifier `VerifierError` (the variant name is in .kind)."""

    def __init__(self, code: int):
        self.code = code
        self.kind = VERIFY_STATUS.get(code, STATUS.get(code, "unknown"))
        super().__init__(f"proof rejected: {self.kind} (status {code})")

_lib = None
_lock = threading.Lock()


def load():
    """Load libzkp.so, raising loudly if it was not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                              "(make -C zk_stark_project_amd/csrc); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        pu8 = ctypes.POINTER(ctypes.c_uint8)
        L.zkp_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
        L.zkp_ctx_destroy.argtypes = [vp]
        L.zkp_ctx_destroy.restype = None
        L.zkp_ctx_trim.argtypes = [vp]
        L.zkp_last_error.argtypes = [vp]
        L.zkp_last_error.restype = ctypes.c_char_p
        L.zkp_free.argtypes = [vp]
        L.zkp_free.restype = None
        from .options import ProofOptionsC
        popt = ctypes.POINTER(ProofOptionsC)
        for name, trace_t in (("zkp_prove", vp), ("zkp_prove_device", vp)):
            f = getattr(L, name)
            f.argtypes = [vp, i32, trace_t, u32, u64, vp, u64, popt, ctypes.POINTER(pu8),
                          ctypes.POINTER(u64), ctypes.POINTER(Transcript)]
        L.zkp_device_alloc.argtypes = [vp, u64, ctypes.POINTER(vp)]
        L.zkp_device_free.argtypes = [vp, vp]
        L.zkp_copy_to_device.argtypes = [vp, vp, vp, u64]
        L.zkp_copy_to_host.argtypes = [vp, vp, vp, u64]
        L.zkp_trace_lde_commit.argtypes = [vp, vp, u32, u64, u32, vp, ctypes.c_char_p]
        L.zkp_merkle_commit_rows.argtypes = [vp, vp, u32, u64, ctypes.c_char_p]
        L.zkp_grind.argtypes = [vp, ctypes.c_char_p, u32, ctypes.POINTER(u64)]
        L.zkp_set_profiling.argtypes = [vp, i32]
        L.zkp_set_profiling_kernel.argtypes = [vp, ctypes.c_char_p]
        L.zkp_kernel_stats.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double)]
        L.zkp_reset_stats.argtypes = [vp]
        L.zkp_kernel_stats_table.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p)]
        L.zkp_build_mimc_trace.argtypes = [ctypes.c_char_p, u64, vp]
        L.zkp_build_mimc_trace.restype = i32
        for name in ("zkp_prove_sharded", "zkp_prove_sharded_device"):
            getattr(L, name).argtypes = [vp, vp, i32, vp, u32, u64, vp, u64, popt, ctypes.POINTER(pu8),
                                         ctypes.POINTER(u64), ctypes.POINTER(Transcript)]
        L.zkp_comm_local_group.argtypes = [i32, ctypes.POINTER(vp)]
        L.zkp_comm_rccl_unique_id.argtypes = [ctypes.c_char_p]
        L.zkp_comm_rccl_create.argtypes = [vp, ctypes.c_char_p, i32, i32, ctypes.POINTER(vp)]
        L.zkp_comm_destroy.argtypes = [vp]
        L.zkp_comm_destroy.restype = None
        L.zkp_comm_rank.argtypes = [vp]
        L.zkp_comm_world.argtypes = [vp]
        L.zkp_comm_backend_world.argtypes = [vp]
        L.zkp_comm_check.argtypes = [vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]
        L.zkp_verify.argtypes = [i32, ctypes.c_char_p, u64, vp, u64, popt]
        L.zkp_verify.restype = i32
        L.zkp_build_global_update_trace.argtypes = [vp, vp, vp, vp, u64, Felt, u64, vp, vp]
        L.zkp_comm_host_create.argtypes = [i32, i32, ctypes.POINTER(HostTransport), ctypes.POINTER(vp)]
        L.zkp_session_create.argtypes = [vp, i32, u32, u64, vp, u64, popt, ctypes.POINTER(vp)]
        L.zkp_session_destroy.argtypes = [vp]
        L.zkp_session_destroy.restype = None
        L.zkp_session_shape.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.zkp_session_trace_lde.argtypes = [vp, vp, ctypes.c_char_p]
        L.zkp_eval_constraints.argtypes = [vp, vp, u32, vp]
        L.zkp_composition_commit.argtypes = [vp, vp, ctypes.c_char_p, ctypes.POINTER(u32)]
        L.zkp_ood_frame.argtypes = [vp, Felt, vp, vp]
        L.zkp_deep_fri.argtypes = [vp, vp, FRI_CHANNEL, vp, vp, ctypes.POINTER(u64), ctypes.c_char_p]
        L.zkp_query.argtypes = [vp, ctypes.POINTER(u64), u64, ctypes.POINTER(pu8), ctypes.POINTER(u64)]
        L.zkp_channel_create.argtypes = [i32, u32, u64, vp, u64, popt, ctypes.POINTER(vp)]
        L.zkp_channel_destroy.argtypes = [vp]
        L.zkp_channel_destroy.restype = None
        L.zkp_channel_commit.argtypes = [vp, ctypes.c_char_p]
        L.zkp_channel_commit_felts.argtypes = [vp, vp, u64]
        L.zkp_channel_draw.argtypes = [vp, u32, u32, vp]
        L.zkp_channel_seed.argtypes = [vp, ctypes.c_char_p]
        L.zkp_channel_query_positions.argtypes = [vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u32)]
        _lib = L
        return L


def mimc_trace(seed: int, n: int) -> np.ndarray:
    """Host MiMC trace builder (serial chain) -> (n, 2) uint64."""
    L = load()
    out = np.empty((n, 2), dtype=np.uint64)
    rc = L.zkp_build_mimc_trace(int(seed).to_bytes(16, "little"), n, out.ctypes.data)
    if rc:
        raise ZkpError(rc, "zkp_build_mimc_trace")
    return out


def verify_status(air_id: int, proof: bytes, pub, options: ProofOptions) -> int:
    """zkp_verify (host-only, no device): 0 or a zkp_verify_status code."""
    L = load()
    pub_np = np.array([[v & (2**64 - 1), v >> 64] for v in pub], dtype=np.uint64).reshape(-1, 2)
    return L.zkp_verify(int(air_id), bytes(proof), len(proof), pub_np.ctypes.data if len(pub) else None,
                        len(pub), ctypes.byref(options.to_c()))


def verify(air_id: int, proof: bytes, pub, options: ProofOptions) -> None:
    """`winterfell::verify` with `AcceptableOptions::OptionSet(vec![options])`; raises VerifierError."""
    rc = verify_status(air_id, proof, pub, options)
    if rc:
        raise VerifierError(rc)


class Comm:
    """Owns one `zkp_comm` (one rank of a coset-sharded proof group)."""

    def __init__(self, ptr: int):
        self.lib = load()
        self.ptr = ctypes.c_void_p(ptr)

    @property
    def rank(self) -> int:
        return int(self.lib.zkp_comm_rank(self.ptr))

    @property
    def world(self) -> int:
        return int(self.lib.zkp_comm_world(self.ptr))

    @property
    def backend_world(self) -> int:
        """Ranks as the transport counts them (RCCL: ncclCommCount)."""
        return int(self.lib.zkp_comm_backend_world(self.ptr))

    def close(self):
        if self.ptr:
            self.lib.zkp_comm_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def local_group(world: int) -> list:
    """`world` communicators of one in-process group (ranks run as threads)."""
    L = load()
    arr = (ctypes.c_void_p * world)()
    rc = L.zkp_comm_local_group(world, arr)
    if rc:
        raise ZkpError(rc, "zkp_comm_local_group")
    return [Comm(arr[i]) for i in range(world)]


def host_comm(rank: int, world: int, all_to_all, all_gather, abort=None) -> Comm:
    """`zkp_comm` over a caller transport: all_to_all(send_ptr, recv_ptr, block_bytes) and
    all_gather(send_ptr, recv_ptr, bytes) are blocking collectives on host memory."""
    L = load()

    def wrap(fn):
        def cb(user, send, recv, nbytes):
            try:
                fn(send, recv, int(nbytes))
                return 0
            except Exception:  # noqa: BLE001 — reported to the library as a failed collective
                import traceback
                traceback.print_exc()
                return 1
        return HOST_A2A(cb)
    t = HostTransport(None, wrap(all_to_all), wrap(all_gather),
                      HOST_ABORT(lambda user: abort() if abort else None))
    p = ctypes.c_void_p()
    rc = L.zkp_comm_host_create(world, rank, ctypes.byref(t), ctypes.byref(p))
    if rc:
        raise ZkpError(rc, "zkp_comm_host_create")
    c = Comm(p.value)
    c._transport = t  # keeps the callbacks alive as long as the communicator
    return c


def rccl_unique_id() -> bytes:
    L = load()
    buf = ctypes.create_string_buffer(128)
    rc = L.zkp_comm_rccl_unique_id(buf)
    if rc:
        raise ZkpError(rc, "zkp_comm_rccl_unique_id")
    return buf.raw


class Context:
    """Owns one `zkp_ctx` (one HIP device, its streams and HBM buffers)."""

    _default = None

    def __init__(self, device: int = 0):
        self.lib = load()
        self.ptr = ctypes.c_void_p()
        rc = self.lib.zkp_ctx_create(device, ctypes.byref(self.ptr))
        if rc:
            raise ZkpError(rc, "zkp_ctx_create")

    @classmethod
    def default(cls) -> "Context":
        if cls._default is None:
            cls._default = cls(0)
        return cls._default

    def trim(self):
        """zkp_ctx_trim: free the idle stage-session context kept for the next session."""
        self._check(self.lib.zkp_ctx_trim(self.ptr), "zkp_ctx_trim")

    def close(self):
        if self.ptr:
            self.lib.zkp_ctx_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc:
            msg = self.lib.zkp_last_error(self.ptr) or b""
            raise ZkpError(rc, f"{what}: {msg.decode(errors='replace')}")

    def prove(self, air_id: int, trace: np.ndarray, pub, options: ProofOptions, device_ptr=None):
        """trace: (width, n, 2) uint64 host array (ignored when device_ptr is given)."""
        w, n = int(trace.shape[0]), int(trace.shape[1])
        pubb = b"".join(int(v).to_bytes(16, "little") for v in pub)
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen = ctypes.c_uint64()
        tr = Transcript()
        oc = options.to_c()
        if device_ptr is None:
            trace = np.ascontiguousarray(trace, dtype=np.uint64)
            rc = self.lib.zkp_prove(self.ptr, air_id, trace.ctypes.data, w, n, pubb, len(pub),
                                    ctypes.byref(oc), ctypes.byref(out), ctypes.byref(olen), ctypes.byref(tr))
        else:
            rc = self.lib.zkp_prove_device(self.ptr, air_id, device_ptr, w, n, pubb, len(pub),
                                           ctypes.byref(oc), ctypes.byref(out), ctypes.byref(olen),
                                           ctypes.byref(tr))
        self._check(rc, "zkp_prove")
        data = ctypes.string_at(out, olen.value)
        self.lib.zkp_free(out)
        return data, tr

    def prove_sharded(self, comm: "Comm", air_id: int, trace, pub, options: ProofOptions, shape=None):
        """One rank of a coset-sharded proof (collective over `comm`). `trace` is a
        (width, n, 2) uint64 host array, or a device pointer with shape=(width, n)."""
        pubb = b"".join(int(v).to_bytes(16, "little") for v in pub)
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen = ctypes.c_uint64()
        tr = Transcript()
        oc = options.to_c()
        if shape is None:
            w, n = int(trace.shape[0]), int(trace.shape[1])
            trace = np.ascontiguousarray(trace, dtype=np.uint64)
            rc = self.lib.zkp_prove_sharded(self.ptr, comm.ptr, air_id, trace.ctypes.data, w, n, pubb, len(pub),
                                            ctypes.byref(oc), ctypes.byref(out), ctypes.byref(olen),
                                            ctypes.byref(tr))
        else:
            w, n = shape
            rc = self.lib.zkp_prove_sharded_device(self.ptr, comm.ptr, air_id, trace, w, n, pubb, len(pub),
                                                   ctypes.byref(oc), ctypes.byref(out), ctypes.byref(olen),
                                                   ctypes.byref(tr))
        self._check(rc, f"zkp_prove_sharded(rank {comm.rank}/{comm.world})")
        data = ctypes.string_at(out, olen.value)
        self.lib.zkp_free(out)
        return data, tr

    def comm_check(self, comm: "Comm", block_bytes: int = 1 << 20):
        """zkp_comm_check (collective): verified all-to-all + all-gather of
        `block_bytes` blocks; returns (all_to_all_ms, all_gather_ms) on this rank."""
        ta, tg = ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.zkp_comm_check(self.ptr, comm.ptr, block_bytes, ctypes.byref(ta), ctypes.byref(tg)),
                    "zkp_comm_check")
        return ta.value, tg.value

    def rccl_comm(self, unique_id: bytes, world: int, rank: int) -> "Comm":
        p = ctypes.c_void_p()
        self._check(self.lib.zkp_comm_rccl_create(self.ptr, unique_id, world, rank, ctypes.byref(p)),
                    "zkp_comm_rccl_create")
        return Comm(p.value)

    def prove_device(self, air_id, d_trace, width, n, pub, options):
        shape = np.empty((width, n, 0))
        return self.prove(air_id, shape, pub, options, device_ptr=d_trace)

    # -- device memory ------------------------------------------------------
    def alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        self._check(self.lib.zkp_device_alloc(self.ptr, nbytes, ctypes.byref(p)), "zkp_device_alloc")
        return p.value

    def free(self, d_ptr: int):
        self._check(self.lib.zkp_device_free(self.ptr, d_ptr), "zkp_device_free")

    def to_device(self, d_ptr: int, host: np.ndarray):
        host = np.ascontiguousarray(host)
        self._check(self.lib.zkp_copy_to_device(self.ptr, d_ptr, host.ctypes.data, host.nbytes),
                    "zkp_copy_to_device")

    def to_host(self, host: np.ndarray, d_ptr: int):
        self._check(self.lib.zkp_copy_to_host(self.ptr, host.ctypes.data, d_ptr, host.nbytes),
                    "zkp_copy_to_host")

    # -- stage entry points -------------------------------------------------
    def build_global_update_trace(self, raw, blinding, local, k: int, n: int, d_out: int):
        """zkp_build_global_update_trace: GlobalUpdate trace into HBM at d_out; returns the final
        masked state (60 ints)."""
        def arr(vals):
            a = np.array([[v & (2**64 - 1), v >> 64] for v in vals], dtype=np.uint64).reshape(-1, 2)
            return np.ascontiguousarray(a)
        r, b = arr(raw), arr(blinding)
        loc = arr([v for row in local for v in row]) if local else np.zeros((1, 2), dtype=np.uint64)
        final = np.zeros((60, 2), dtype=np.uint64)
        kf = Felt(k & (2**64 - 1), k >> 64)
        rc = self.lib.zkp_build_global_update_trace(self.ptr, r.ctypes.data, b.ctypes.data, loc.ctypes.data,
                                                    len(local), kf, n, d_out, final.ctypes.data)
        self._check(rc, "zkp_build_global_update_trace")
        return [int(lo) | (int(hi) << 64) for lo, hi in final]

    def trace_lde_commit(self, trace: np.ndarray, blowup: int, want_lde: bool = True):
        trace = np.ascontiguousarray(trace, dtype=np.uint64)
        w, n = trace.shape[0], trace.shape[1]
        lde = np.empty((w, n * blowup, 2), dtype=np.uint64) if want_lde else None
        root = ctypes.create_string_buffer(32)
        self._check(self.lib.zkp_trace_lde_commit(self.ptr, trace.ctypes.data, w, n, blowup,
                                                  lde.ctypes.data if want_lde else None, root),
                    "zkp_trace_lde_commit")
        return lde, root.raw

    def merkle_commit_rows(self, cols: np.ndarray) -> bytes:
        cols = np.ascontiguousarray(cols, dtype=np.uint64)
        root = ctypes.create_string_buffer(32)
        self._check(self.lib.zkp_merkle_commit_rows(self.ptr, cols.ctypes.data, cols.shape[0],
                                                    cols.shape[1], root), "zkp_merkle_commit_rows")
        return root.raw

    def grind(self, seed: bytes, bits: int) -> int:
        nonce = ctypes.c_uint64()
        self._check(self.lib.zkp_grind(self.ptr, seed, bits, ctypes.byref(nonce)), "zkp_grind")
        return nonce.value

    # -- profiling ----------------------------------------------------------
    def set_profiling(self, on: bool, kernel: str | None = None):
        """Bracket launches with HIP events (all of them, or only those named `kernel`)."""
        self._check(self.lib.zkp_set_profiling_kernel(self.ptr, kernel.encode() if kernel else None),
                    "zkp_set_profiling_kernel")
        self._check(self.lib.zkp_set_profiling(self.ptr, 1 if on else 0), "zkp_set_profiling")

    def reset_stats(self):
        self._check(self.lib.zkp_reset_stats(self.ptr), "zkp_reset_stats")

    def kernel_stats(self, name: str):
        n = ctypes.c_uint64()
        ms = ctypes.c_double()
        self._check(self.lib.zkp_kernel_stats(self.ptr, name.encode(), ctypes.byref(n), ctypes.byref(ms)),
                    "zkp_kernel_stats")
        return n.value, ms.value

    def stats_table(self) -> dict:
        p = ctypes.c_char_p()
        self._check(self.lib.zkp_kernel_stats_table(self.ptr, ctypes.byref(p)), "zkp_kernel_stats_table")
        txt = p.value.decode()
        self.lib.zkp_free(ctypes.cast(p, ctypes.c_void_p))
        out = {}
        for line in txt.splitlines():
            name, cnt, ms, nbytes = line.split()
            out[name] = {"launches": int(cnt), "ms": float(ms), "bytes": float(nbytes)}
        return out


def _felts(vals) -> np.ndarray:
    return np.ascontiguousarray(np.array([[int(v) & (2**64 - 1), int(v) >> 64] for v in vals],
                                         dtype=np.uint64).reshape(-1, 2))


def _ints(a: np.ndarray) -> list:
    return [int(lo) | (int(hi) << 64) for lo, hi in a.reshape(-1, 2)]


class Session:
    """One proof driven stage by stage (`zkp_session`, include/zkp.h): the plug-in
    hooks a winter-prover fork calls from its own `generate_proof` with its own
    channel. Stages: trace_lde -> eval_constraints -> composition_commit ->
    ood_frame -> deep_fri -> query."""

    def __init__(self, ctx: "Context", air_id: int, width: int, n: int, pub, options: ProofOptions):
        self.ctx, self.lib, self.width, self.n = ctx, ctx.lib, width, n
        self.ptr = ctypes.c_void_p()
        self._pub = _felts(pub) if len(pub) else None
        self._opts = options.to_c()
        ctx._check(self.lib.zkp_session_create(ctx.ptr, air_id, width, n,
                                               self._pub.ctypes.data if self._pub is not None else None,
                                               len(pub), ctypes.byref(self._opts), ctypes.byref(self.ptr)),
                   "zkp_session_create")
        # the AIR's own shape (not re-derived here): evals_out holds n*ce values
        ce, nc, nl = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        ctx._check(self.lib.zkp_session_shape(self.ptr, ctypes.byref(ce), ctypes.byref(nc), ctypes.byref(nl)),
                   "zkp_session_shape")
        self.ce, self.fri_layers = ce.value, nl.value
        self.num_columns = None

    def close(self):
        if self.ptr:
            self.lib.zkp_session_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trace_lde(self, trace: np.ndarray) -> bytes:
        """trace: (width, n, 2) uint64 column-major -> trace commitment root."""
        trace = np.ascontiguousarray(trace, dtype=np.uint64)
        root = ctypes.create_string_buffer(32)
        self.ctx._check(self.lib.zkp_session_trace_lde(self.ptr, trace.ctypes.data, root), "zkp_session_trace_lde")
        return root.raw

    def eval_constraints(self, coeffs, want_evals: bool = True):
        """composition coefficients -> n*ce evaluations (natural CE-domain order) or None."""
        c = _felts(coeffs)
        out = None
        if want_evals:
            out = np.zeros((self.n * self.ce, 2), dtype=np.uint64)
        self.ctx._check(self.lib.zkp_eval_constraints(self.ptr, c.ctypes.data, len(coeffs),
                                                      out.ctypes.data if out is not None else None),
                        "zkp_eval_constraints")
        return out

    def composition_commit(self, evals: np.ndarray | None = None) -> bytes:
        root = ctypes.create_string_buffer(32)
        nc = ctypes.c_uint32()
        e = np.ascontiguousarray(evals, dtype=np.uint64) if evals is not None else None
        self.ctx._check(self.lib.zkp_composition_commit(self.ptr, e.ctypes.data if e is not None else None, root,
                                                        ctypes.byref(nc)), "zkp_composition_commit")
        self.num_columns = nc.value
        return root.raw

    def ood_frame(self, z: int):
        """-> (trace_ood: 2*width ints [T(z) | T(zg)], comp_ood: C ints)."""
        t = np.zeros((2 * self.width, 2), dtype=np.uint64)
        c = np.zeros((self.num_columns, 2), dtype=np.uint64)
        self.ctx._check(self.lib.zkp_ood_frame(self.ptr, Felt(z & (2**64 - 1), z >> 64), t.ctypes.data,
                                               c.ctypes.data), "zkp_ood_frame")
        return _ints(t), _ints(c)

    def deep_fri(self, deep_coeffs, channel):
        """channel(layer, root: bytes) -> alpha (int). Returns (remainder ints, remainder commitment)."""
        g = _felts(deep_coeffs)
        err = []

        def cb(user, layer, root, alpha_p):
            try:
                a = int(channel(int(layer), bytes(root[:32])))
                ctypes.cast(alpha_p, ctypes.POINTER(Felt))[0] = Felt(a & (2**64 - 1), a >> 64)
                return 0
            except Exception as e:  # noqa: BLE001 — re-raised after the call
                err.append(e)
                return 1
        fn = FRI_CHANNEL(cb)
        rem = np.zeros((256, 2), dtype=np.uint64)
        rlen = ctypes.c_uint64(256)
        commit = ctypes.create_string_buffer(32)
        rc = self.lib.zkp_deep_fri(self.ptr, g.ctypes.data, fn, None, rem.ctypes.data, ctypes.byref(rlen), commit)
        if err:
            raise err[0]
        self.ctx._check(rc, "zkp_deep_fri")
        return _ints(rem[:rlen.value]), commit.raw

    def query(self, positions) -> bytes:
        pos = (ctypes.c_uint64 * len(positions))(*positions)
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen = ctypes.c_uint64()
        self.ctx._check(self.lib.zkp_query(self.ptr, pos, len(positions), ctypes.byref(out), ctypes.byref(olen)),
                        "zkp_query")
        data = ctypes.string_at(out, olen.value)
        self.lib.zkp_free(out)
        return data


class Channel:
    """`zkp_channel` (include/zkp.h): winter-prover's ProverChannel over
    DefaultRandomCoin<Blake3_256>, seeded as generate_proof seeds it. Host-only."""

    def __init__(self, air_id: int, width: int, n: int, pub, options: ProofOptions):
        self.lib = load()
        self.options = options
        self.ptr = ctypes.c_void_p()
        pb = _felts(pub) if len(pub) else None
        rc = self.lib.zkp_channel_create(air_id, width, n, pb.ctypes.data if pb is not None else None, len(pub),
                                         ctypes.byref(options.to_c()), ctypes.byref(self.ptr))
        if rc:
            raise ZkpError(rc, "zkp_channel_create")

    def close(self):
        if self.ptr:
            self.lib.zkp_channel_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ok(self, rc, what):
        if rc:
            raise ZkpError(rc, what)

    def commit(self, root: bytes):
        self._ok(self.lib.zkp_channel_commit(self.ptr, bytes(root)), "zkp_channel_commit")

    def commit_felts(self, vals):
        a = _felts(vals)
        self._ok(self.lib.zkp_channel_commit_felts(self.ptr, a.ctypes.data, len(vals)), "zkp_channel_commit_felts")

    def draw(self) -> int:
        out = np.zeros((1, 2), dtype=np.uint64)
        self._ok(self.lib.zkp_channel_draw(self.ptr, 0, 0, out.ctypes.data), "zkp_channel_draw")
        return _ints(out)[0]

    def draw_coeffs(self, method: int, count: int) -> list:
        out = np.zeros((count, 2), dtype=np.uint64)
        self._ok(self.lib.zkp_channel_draw(self.ptr, method, count, out.ctypes.data), "zkp_channel_draw")
        return _ints(out)

    def seed(self) -> bytes:
        b = ctypes.create_string_buffer(32)
        self._ok(self.lib.zkp_channel_seed(self.ptr, b), "zkp_channel_seed")
        return b.raw

    def query_positions(self, nonce: int) -> list:
        out = (ctypes.c_uint64 * 256)()
        nu = ctypes.c_uint32()
        self._ok(self.lib.zkp_channel_query_positions(self.ptr, nonce, out, ctypes.byref(nu)),
                 "zkp_channel_query_positions")
        return [int(out[i]) for i in range(nu.value)]


def prove_by_stages(ctx: "Context", air_id: int, trace: np.ndarray, pub, options: ProofOptions,
                    num_coeffs: int, times: dict | None = None) -> dict:
    """One proof through the stage hooks, in generate_proof's order, with the host
    channel drawing every coefficient (what a winter-prover fork's `Prover::prove`
    does with its own channel). Returns the commitments, z, nonce, positions and the
    query section; they equal zkp_prove's for the same trace. `times` (optional)
    accumulates the wall-clock ms of each stage call under its entry point's name."""
    w, n = int(trace.shape[0]), int(trace.shape[1])
    clock = [time.perf_counter()]

    def lap(name):
        if times is not None:
            t = time.perf_counter()
            times[name] = times.get(name, 0.0) + (t - clock[0]) * 1e3
            clock[0] = t
    ch = Channel(air_id, w, n, pub, options)
    s = Session(ctx, air_id, w, n, pub, options)
    lap("create")
    try:
        troot = s.trace_lde(trace)
        lap("trace_lde")
        ch.commit(troot)
        s.eval_constraints(ch.draw_coeffs(options.batching_constraints, num_coeffs), want_evals=False)
        lap("eval_constraints")
        croot = s.composition_commit()
        lap("composition_commit")
        ch.commit(croot)
        z = ch.draw()
        tood, cood = s.ood_frame(z)
        lap("ood_frame")
        ch.commit_felts(tood)
        ch.commit_felts(cood)
        gam = ch.draw_coeffs(options.batching_deep, w + s.num_columns)
        roots = []

        def fri_channel(layer, root):
            roots.append(root)
            ch.commit(root)
            return ch.draw()
        rem, rcommit = s.deep_fri(gam, fri_channel)
        lap("deep_fri")
        ch.commit(rcommit)
        nonce = ctx.grind(ch.seed(), options.grinding_factor) if options.grinding_factor else 1
        lap("grind")
        pos = ch.query_positions(nonce)
        queries = s.query(pos)
        lap("query")
    finally:
        s.close()
        ch.close()
    return {"trace_root": troot, "constraint_root": croot, "z": z, "fri_roots": roots, "remainder": rem,
            "remainder_commitment": rcommit, "pow_nonce": nonce, "query_positions": pos, "queries": queries}
