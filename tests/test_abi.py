"""CPU checks of the C-ABI boundary: libzkp.so loads, exports every function
include/zkp.h declares, and fails loudly (no CPU fallback) without a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "zk_stark_project_amd", "libzkp.so")


def header_functions():
    src = open(os.path.join(ROOT, "include", "zkp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\s*\*)\s+(zkp_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "zk_stark_project_amd", "csrc")])
    return ctypes.CDLL(LIB)


def test_exports_every_declared_symbol(lib):
    names = header_functions()
    assert len(names) >= 18
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (zkp_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        getattr(lib, n)
    from zk_stark_project_amd import _native
    assert sorted(_native.EXPORTED) == names


def test_no_cpu_fallback_without_gpu(lib):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    from zk_stark_project_amd import _native
    with pytest.raises(_native.ZkpError) as e:
        _native.Context(0)
    assert e.value.code == 5  # ZKP_ERR_DEVICE


def test_mimc_trace_builder_matches_oracle(lib):
    """zkp_build_mimc_trace is a host trace-construction helper (not the prover)."""
    import oracle_ref as O
    from zk_stark_project_amd import _native
    t = _native.mimc_trace(42 * 10**6, 256)
    assert t.tobytes() == O.mimc_trace(42 * 10**6, 256)


def test_null_arguments_rejected(lib):
    lib.zkp_prove.restype = ctypes.c_int
    assert lib.zkp_prove(None, 1, None, 1, 64, None, 0, None, None, None, None) == 9  # ZKP_ERR_ARGUMENT
    lib.zkp_build_mimc_trace.restype = ctypes.c_int
    assert lib.zkp_build_mimc_trace(None, 8, None) == 9


def test_comm_world_and_backend_world(lib):
    """zkp_comm_world / zkp_comm_backend_world on a caller-transport group (host only, no
    collective runs): the transport's own count equals the group size; a null comm is -1."""
    from zk_stark_project_amd import _native
    comm = _native.host_comm(1, 4, lambda s, r, b: None, lambda s, r, b: None)
    try:
        assert (comm.rank, comm.world, comm.backend_world) == (1, 4, 4)
    finally:
        comm.close()
    lib.zkp_comm_backend_world.restype = ctypes.c_int
    assert lib.zkp_comm_backend_world(None) == -1
