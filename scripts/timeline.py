"""Per-launch timeline of one MiMC 2^20 proof (diagnostics only; run on the GPU box).

ZKP_TIMELINE=1 makes the library print (start, duration, gap) of every bracketed
launch of a profiled call on stderr.  This proves three warm-up proofs and then
one profiled proof.  Usage: python3 scripts/timeline.py [log_n]
"""
import os
import sys

os.environ["ZKP_TIMELINE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zk_stark_project_amd import AIR_MIMC, MimcProver, ProofOptions, _native  # noqa: E402


def main():
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 1 << log_n
    ctx = _native.Context(0)
    opts = ProofOptions(40, 8, 21)
    prover = MimcProver(opts, ctx)
    trace = prover.build_trace(42 * 10**6, n)
    pub = prover.get_pub_inputs(trace).to_elements()
    d_trace = ctx.alloc(trace.data.nbytes)
    ctx.to_device(d_trace, trace.data)
    for _ in range(3):
        ctx.prove_device(AIR_MIMC, d_trace, 1, n, pub, opts)
    ctx.set_profiling(True)
    ctx.prove_device(AIR_MIMC, d_trace, 1, n, pub, opts)
    ctx.set_profiling(False)


if __name__ == "__main__":
    main()
