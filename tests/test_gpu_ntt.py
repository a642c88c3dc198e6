"""Field-op fast paths and the NTT rounds' exact recomputation on the GPU.

The product and sum forms skip the exact canonical select unless a lane needs it
(felt_dev.hpp canon_rare / add_sum, and the NTT rounds' deferred check that redoes
a round with the exact forms). Random data reaches those branches about once per
2^32 operations, so the proof-level parity tests never take them; these native
checks drive them on purpose (values at p - 1 against small values, products whose
residue sits at the top of the range or below 2^128 - p) and compare with the host's
portable arithmetic and a host DFT. Binaries built by __graft_entry__.build()
(tests/native/Makefile)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def run(binary, *args, timeout=240):
    path = os.path.join(HERE, binary)
    assert os.path.exists(path), f"{path} not built (run __graft_entry__.build())"
    r = subprocess.run([path, *args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def test_field_op_edge_cases():
    out = run("ubench_bfly", "--check")
    assert "all equal to the host's portable arithmetic" in out


def test_ntt_exact_redo_rounds():
    out = run("ntt_check")
    assert "0 mismatching" in out, out


def test_eval_mimc_exact_redo():
    """k_eval_mimc's exact recomputation, driven on purpose (tests/native/eval_check.cpp):
    every output equals the host's exact arithmetic and the redo branch was taken."""
    out = run("eval_check")
    assert ", 0 mismatching," in out, out
    redo = int(out.strip().splitlines()[-1].split(",")[-1].split()[0])
    assert redo > 0, out
