#!/usr/bin/env python3
"""bench.py — STARK proofs/s on MI355X for the MiMC AIR 2^20-step trace.

Metric (BASELINE.json): "STARK proofs/sec + prove-time ms, MiMC AIR 2^20-step
trace, 1/2/4/8 MI355X". Workload = BASELINE.json configs[1]:
MiMC AIR, n = 2^20, x0 = 42e6, ProofOptions(40, 8, 21,
None, 16, 7, Algebraic, Algebraic).

A "step" is SURVEY.md §8(d)'s "prove": `zkp_prove` wall-clock from the host
trace (a pageable numpy array, built before timing) to the serialized proof
bytes, PCIe upload included. `value` = proofs/s and `ms_per_step` = mean
ms/proof of those calls; `step_ms` gives their median and min (BASELINE.md:35).
Extra keys: `trace_resident` (the same proof by `zkp_prove_device` with the
trace already in HBM; never `value`), `first_proof_ms` (first proof of a
fresh context: domain tables built cold), `sustained` (proofs/s over a few
seconds), `c3` (BASELINE configs[2]: the aggregation AIR, 64 updates, 2^18 x
120, reference options, with its own roofline and oracle byte check) and
`reference_flow` (/root/reference/src/main.rs:374-493, the reference binary's
proof step: 8 TrainingUpdate proofs at bs = 50 and the GlobalUpdate proof,
cold and warm, beside the oracle).

Multi-GPU: one process per GPU (torchrun). Default `--mode replicas`: each
rank proves its own independent 2^20 trace on its own device (weak scaling,
no data-path collective); value = total proofs of all ranks / max-over-ranks
wall time. With N > 1 the line also carries `sharded`: ONE C4 proof (MiMC
2^22, BASELINE configs[3]) split over all ranks by LDE coset, collectives over
the library's RCCL communicator (xGMI). `--mode sharded` makes that the
headline (strong scaling; `--air agg` = configs[4] C5). See DESIGN.md §5-6.

`roofline`: the dominant kernel's SURVEY.md §8(d) algorithmic bytes per launch
(Appendix C stage bytes / that kernel's launches per proof) ÷ its average
HIP-event launch time on the prover's stream, measured live in the timed
region; `whole_proof_frac` = §8(d) bytes per proof ÷ ms_per_step ÷ 8 TB/s.
`cpu_baseline`: the C oracle restating the winterfell CPU path on the host
cores (rank 0, N=1 only, bounded sample).
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CLOCK_GHZ, SIMDS = 2.4, 1024
# measured SIMD cycles per wave64 VALU instruction on gfx950 (tests/native/ubench_valu.hip,
# profiles/r02_ubench_valu.txt): plain 2-operand 32-bit ops (v_add_u32, v_xor, v_mov, shifts)
# issue every 2 cycles; carry in/out, 3-operand, multiply and 64-bit ops every 4
VALU_CYCLES_FAST, VALU_CYCLES_SLOW = 2.0, 4.0
E, H = 16, 32  # felt and digest bytes

# launch name (zkp_kernel_stats_table) -> kernel symbol in the rocprofv3 PMC
# summaries that scripts/profile_round.sh writes (profiles/r0*_pmc_*.json)
KERNEL_SYMBOL = {
    "ntt_dit": "void k_ntt8<true,", "ntt_dif": "void k_ntt8<false,", "deep": "k_deep",
    "merkle_lde": ("void k_merkle_lane<0,", "void k_merkle_lane<4,", "void k_merkle_leaf2<"), "eval_mimc": "k_eval_mimc",
    "eval_linear": ("void k_eval_linear<", "void k_eval_linear_pts<"),
}
# launch name -> SURVEY.md Appendix C stages whose algorithmic bytes that kernel moves.
# ntt_dit is charged per column it actually extends (kernel_stage_bytes): the trace
# columns that are interpolated and extended (GlobalUpdate pairing derives the other
# half) and the composition columns (the derived last column, LastCol, is written by
# the leaf pass, not by an NTT)
KERNEL_STAGES = {
    "ntt_dit": ("lde", "comp_lde"), "ntt_dif": ("intt", "comp_intt"), "deep": ("deep",),
    "eval_mimc": ("eval",), "eval_linear": ("eval",),
}
UBENCH_BFLY = "profiles/r04_ubench_bfly.json"  # tests/native/ubench_bfly.hip on the box: the butterfly floor
PMC_TAGS = ("r06", "r05", "r04", "r03", "r02_final", "r02", "r01")  # newest committed PMC summaries first (scripts/profile_round.sh)


def stage_bytes(w: int, n: int, B: int, ce: int, C: int, rem: int = 7, F: int = 16) -> dict:
    """algorithmic bytes per proof, per stage (winterfell's
    materialize-every-stage dataflow; fusion does not change these figures)."""
    N = n * B
    s = {
        "intt": 2 * w * n * E,
        "lde": w * n * E + w * N * E,
        "trace_merkle": w * N * E + 2 * N * H,
        "eval": w * n * ce * E + n * ce * E,
        "comp_intt": 2 * n * ce * E,
        "comp_lde": C * n * E + C * N * E,
        "comp_merkle": C * N * E + 2 * N * H,
        "ood": (w + C) * n * E,
        "deep": (w + C) * n * E + 2 * n * E + N * E,
    }
    fri, D = 0, N
    while D > (rem + 1) * B:
        fri += 2 * D * E + 2 * (D // F) * H + (D // F) * E
        D //= F
    s["fri"] = fri
    return s


def lde_columns(wl: dict, R: int) -> tuple:
    """(trace columns, composition columns) that ntt_dit's launches extend per proof."""
    w, C, ce, B = wl["width"], wl["C"], wl["ce"], wl["opts"].blowup_factor
    comp = C - 1 if (ce == B and 2 <= C <= 8) else C  # LastCol: derived in the composition leaf pass
    trace = w
    if wl.get("paired"):  # GlobalUpdate: columns 0..59 (rounded up to a multiple of the ranks) are extended
        d = w // 2
        trace = d if R == 1 else -(-d // R) * R
    return trace, comp


def kernel_stage_bytes(kernel: str, sb: dict, wl: dict, R: int):
    """Appendix C bytes per proof that `kernel` is charged with, and a source note."""
    stages = KERNEL_STAGES.get(kernel)
    if not stages:
        return None, None
    if kernel != "ntt_dit":
        return sum(sb[s] for s in stages), f"stages {'+'.join(stages)}"
    n, N = wl["n"], wl["n"] * wl["opts"].blowup_factor
    tcols, ccols = lde_columns(wl, R)
    per_col = n * E + N * E  # Appendix C lde / comp_lde per column
    return ((tcols + ccols) * per_col,
            f"stages lde+comp_lde for the columns ntt_dit extends: {tcols} trace + {ccols} composition column(s) "
            f"x (nE + NE) (of w = {wl['width']}, C = {wl['C']})")


def floor_rate():
    """G butterflies/s of the committed butterfly micro-benchmark, or None."""
    path = os.path.join(ROOT, UBENCH_BFLY)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("gbfly_per_s")


def zkp_env() -> dict:
    """Every ZKP_* switch set in this process's environment (A/B switches of the library)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("ZKP_")}


def load_pmc(kind: str, air: str, kernel: str):
    prefix = KERNEL_SYMBOL.get(kernel)
    for tag in PMC_TAGS:
        name = {"mimc": f"{tag}_pmc_{kind}_mimc_c2.json", "agg": f"{tag}_pmc_{kind}_agg_c3.json"}[air]
        path = os.path.join(ROOT, "profiles", name)
        if os.path.exists(path):
            break
    if not prefix or not os.path.exists(path):
        return None, name
    with open(path) as f:
        recs = {k: v for k, v in json.load(f).items() if k.startswith(prefix)}  # prefix: str or tuple of str
    if not sum(v["launches"] for v in recs.values()):
        return None, name
    return recs, name


def pmc_traffic(kernel: str, air: str, mode: str):
    """HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected) of `kernel`
    from the committed PMC summary of the same workload, or None. A launch name may
    cover several template instances (the NTT pass kernels are templated on their
    stage count): their traffic is averaged over all their launches."""
    if mode != "replicas":
        return None, None
    recs, name = load_pmc("traffic", air, kernel)
    if not recs:
        return None, None
    launches = sum(v["launches"] for v in recs.values())
    traffic = sum(v["traffic_per_launch"] * v["launches"] for v in recs.values()) / launches
    syms = ", ".join(sorted(recs))
    return traffic, f"profiles/{name} ({syms}; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"


def valu_side(kernel: str, air: str, mode: str):
    """VALU issue of `kernel` from the committed SQ PMC summary of the same workload
    (the path is INT-VALU-bound). Reported against the 2-cycle wave64
    issue rate of the SIMD (MI355X_MICROARCH.md) and against the instruction mix's own
    issue cost (the kernel's static ISA mix over the measured 2- and 4-cycle classes)."""
    if mode != "replicas":
        return None
    recs, name = load_pmc("sq", air, kernel)
    if not recs:
        return None
    launches = sum(v["launches"] for v in recs.values())
    us = sum(v["avg_us"] * v["launches"] for v in recs.values())
    insts = sum(v["valu_insts_per_launch"] * v["launches"] for v in recs.values())
    cyc_avail = us * 1e3 * CLOCK_GHZ * SIMDS
    out = {"valu_insts_per_launch": round(insts / launches), "issue_util_2cyc": round(insts * 2 / cyc_avail, 3),
           "peak": "1 wave64 VALU instruction / 2 cycles / SIMD (MI355X_MICROARCH.md:54)",
           "source": f"profiles/{name} (rocprofv3 --pmc SQ_INSTS_VALU..., {', '.join(sorted(recs))})"}
    mix = isa_mix()
    slow = {k: mix.get(k) for k in recs}
    if mix and all(s is not None for s in slow.values()):
        sf = sum(slow[k] * v["valu_insts_per_launch"] * v["launches"] for k, v in recs.items()) / insts
        cyc = insts * (sf * VALU_CYCLES_SLOW + (1 - sf) * VALU_CYCLES_FAST)
        out["slow_class_frac"] = round(sf, 3)
        out["issue_util_mix"] = round(cyc / cyc_avail, 3)
        out["mix_note"] = ("share of 4-cycle VALU instructions (carry, multiply, 3-operand, 64-bit) from the kernel's "
                           "ISA mix (scripts/isa_mix.py); issue_util_mix = insts x mix cycles / SIMD cycles")
    return out


def isa_mix() -> dict:
    """kernel symbol (as the rocprofv3 summaries name it) -> share of 4-cycle VALU
    instructions in its gfx950 ISA (profiles/r0*_isa_mix.json, scripts/isa_mix.py)."""
    for name in ("r05_isa_mix.json", "r04_isa_mix.json", "r02_isa_mix.json"):  # newest first
        path = os.path.join(ROOT, "profiles", name)
        if os.path.exists(path):
            break
    else:
        return {}
    with open(path) as f:
        d = json.load(f)
    return {k.replace("(anonymous namespace)::", "").split("(")[0]: v["slow_frac"] for k, v in d.items()}


def host_cpus() -> int:
    """CPUs this job may use on the host: the cgroup cpu.max quota when one is set
    (the GPU box gives each job a share of a larger machine), else the scheduler
    affinity. os.cpu_count() reports the whole machine either way."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def c1_leg(ctx) -> dict:
    """BASELINE configs[0] / SURVEY §8(d) C1: benches/bench_mimc.rs:17-60 restated —
    mimc_cipher(x, rc, 0) with x, rc = the first two next_u64 of StdRng::from_seed([24; 32])
    (tests/golden/mimc.json, ChaCha12 restated) and mimc_hash_matrix over the bench's
    6x9 of 42.0 and 6 of 1.0, timed on one host thread by the C oracle; plus a MiMC-AIR
    STARK at n = 2^10 (blowup 8, options of C2) on the CPU oracle and on the GPU."""
    import oracle_ref
    from zk_stark_project_amd import AIR_MIMC, MimcProver, ProofOptions, helper
    with open(os.path.join(ROOT, "tests", "golden", "mimc.json")) as f:
        kat = json.load(f)
    bc = kat["bench_mimc_cipher"]
    x, rc = int(bc["x"]), int(bc["rc"])
    assert oracle_ref.mimc_cipher(x, rc, 0) == int(bc["out"])
    cipher_s, _ = oracle_ref.time_mimc_cipher(x, rc, 200000)
    w = [[helper.f64_to_felt(42.0)] * 9] * 6
    b = [helper.f64_to_felt(1.0)] * 6
    rcs = helper.get_round_constants()
    _, d = oracle_ref.time_mimc_hash_matrix(w, b, rcs, 1)
    assert d == int(kat["mimc_hash_matrix_bench"])
    hash_s, _ = oracle_ref.time_mimc_hash_matrix(w, b, rcs, 2000)
    opts = ProofOptions(40, 8, 21)
    prover = MimcProver(opts, ctx)
    n = 1 << 10
    trace = prover.build_trace(42 * 10**6, n)
    pub = prover.get_pub_inputs(trace).to_elements()
    pb = b"".join(v.to_bytes(16, "little") for v in pub)
    t0 = time.perf_counter()
    cproof, _ = oracle_ref.prove(AIR_MIMC, trace.to_bytes(), 1, n, pb, opts)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    ctx.prove(AIR_MIMC, trace.data, pub, opts)  # warm the 2^10 domain tables
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        gproof, _ = ctx.prove(AIR_MIMC, trace.data, pub, opts)
    gpu_ms = (time.perf_counter() - t0) * 1e3 / reps
    return {"workload": "benches/bench_mimc.rs (BASELINE configs[0]) + MiMC AIR 2^10 STARK, blowup 8",
            "mimc_cipher_ns": round(cipher_s * 1e9, 1), "mimc_hash_matrix_us": round(hash_s * 1e6, 2),
            "cipher_inputs": "StdRng::from_seed([24; 32]) next_u64 x2 (tests/golden/mimc.json)",
            "helpers_on": "C oracle, 1 host thread",
            "stark_2e10_cpu_ms": round(cpu_ms, 2), "cpu_threads": oracle_ref.lib().oracle_num_threads(),
            "stark_2e10_gpu_ms": round(gpu_ms, 3), "proof_bytes_identical": cproof == gproof}


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"os_cpu_count": os.cpu_count(), "job_cpus": host_cpus(), "model": model,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=None, help="trace length 2^k (default: the config's)")
    ap.add_argument("--mode", choices=["replicas", "sharded"], default="replicas")
    ap.add_argument("--blowup", type=int, default=8)
    ap.add_argument("--sustain-s", type=float, default=3.0, help="seconds of back-to-back proofs for `sustained`")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-sharded-leg", action="store_true", help="N>1 replicas: skip the C4 sharded proof")
    ap.add_argument("--sharded-leg", action="store_true",
                    help="run the C4 sharded leg at N = 1 too (a world-1 RCCL rehearsal of its collectives and checks)")
    ap.add_argument("--stats", action="store_true", help="print the per-kernel table to stderr")
    ap.add_argument("--no-concurrent", dest="concurrent", action="store_false",
                    help="N=1: skip the leg with 3 proofs in flight on the GPU")
    ap.add_argument("--no-c3", dest="c3", action="store_false",
                    help="N=1 MiMC line: skip the C3 leg (BASELINE configs[2])")
    ap.add_argument("--no-reference-flow", dest="reference_flow", action="store_false",
                    help="N=1 MiMC line: skip the reference binary's proof step (main.rs:374-493)")
    ap.add_argument("--no-rank-emulation", dest="rank_emulation", action="store_false",
                    help="N=1 MiMC line: skip the emulated rank of the 8-GPU C4 proof")
    ap.add_argument("--no-tampered", dest="tampered", action="store_false",
                    help="skip the tampered-trace proofs (keeps PMC passes to valid proofs)")
    ap.add_argument("--air", choices=["mimc", "agg"], default="mimc",
                    help="mimc = C2 (default, the BASELINE metric); agg = C3 GlobalUpdate (64 updates, 2^18 rows)")
    return ap.parse_args()


def make_workload(air: str, sharded: bool, log_n, blowup: int, seed_rank: int, ctx):
    from zk_stark_project_amd import AIR_GLOBAL_UPDATE, AIR_MIMC, GlobalUpdateProver, MimcProver, ProofOptions
    from zk_stark_project_amd.helper import f64_to_felt
    if air == "mimc":
        log_n = log_n or (22 if sharded else 20)
        n = 1 << log_n
        opts = ProofOptions(40, blowup, 21)  # (40, 8, 21, None, 16, 7, Algebraic, Algebraic)
        prover = MimcProver(opts, ctx)
        trace = prover.build_trace(42 * 10**6 + seed_rank, n)  # independent trace per replica
        cfg = "BASELINE configs[3], domain-sharded" if sharded else "BASELINE configs[1]"
        return dict(air_id=AIR_MIMC, width=1, n=n, log_n=log_n, opts=opts, trace=trace, prover=prover, ce=8, C=6,
                    paired=False, workload=f"MiMC AIR 2^{log_n}-step trace, blowup={blowup} ({cfg})")
    import random
    log_n = log_n or (20 if sharded else 18)
    n = 1 << log_n
    opts = ProofOptions.reference()  # (40, 16, 21, None, 16, 7, Algebraic, Algebraic)
    rnd = random.Random(1 + seed_rank)
    r = lambda: rnd.randrange(2**64)  # noqa: E731
    ndev = 256 if sharded else 64
    prover = GlobalUpdateProver(opts, [[r() for _ in range(9)] for _ in range(6)], [r() for _ in range(6)],
                                [[[r() for _ in range(9)] for _ in range(6)] for _ in range(ndev)],
                                [[r() for _ in range(6)] for _ in range(ndev)], f64_to_felt(ndev),
                                trace_length=n, blinding=[r() for _ in range(60)], ctx=ctx)
    trace = prover.build_trace()
    cfg = "BASELINE configs[4], domain-sharded" if sharded else "BASELINE configs[2]"
    return dict(air_id=AIR_GLOBAL_UPDATE, width=120, n=n, log_n=log_n, opts=opts, trace=trace, prover=prover,
                ce=2, C=1, paired=True, workload=f"GlobalUpdate AIR, {ndev} updates padded to 2^{log_n} rows, w=120 ({cfg})")


WATCHDOG_EXIT = 3  # exit status of every rank when the sharded leg hangs


def watchdog(done: threading.Event, timeout_s: float, rank: int, on_timeout=None, exit_fn=os._exit):
    """Ends the process with WATCHDOG_EXIT unless `done` is set within timeout_s: a
    hung collective must not look like a clean run (rank 0 first prints the
    headline line it already has, with the error, so the measurement survives)."""
    if done.wait(timeout_s):
        return
    print(json.dumps({"error": f"sharded leg exceeded {timeout_s:.0f} s on rank {rank}"}), file=sys.stderr, flush=True)
    if on_timeout is not None:
        on_timeout()
    sys.stdout.flush()
    sys.stderr.flush()
    exit_fn(WATCHDOG_EXIT)


def sharded_leg(ctx, rank: int, world: int, dist, local_rank: int, on_timeout=None, timeout_s: float = 120.0):
    """One C4 proof (MiMC 2^22, B = 8) split over all `world` ranks by LDE coset over
    RCCL; timed like the headline (barrier + device sync, max over ranks). Runs after
    the headline line is built: a watchdog bounds it, and on a hung collective rank 0
    prints the headline (with the sharded error) before every rank exits."""
    import torch
    from zk_stark_project_amd.replicas import timed_replicas
    from zk_stark_project_amd.sharded import rccl_group_comm

    done = threading.Event()
    threading.Thread(target=watchdog, args=(done, timeout_s, rank, on_timeout), daemon=True).start()
    wl = make_workload("mimc", True, None, 8, 0, ctx)
    pub = wl["prover"].get_pub_inputs(wl["trace"]).to_elements()
    comm = rccl_group_comm(ctx, rank, world)
    try:
        # fabric check first (zkp_comm_check: verified RCCL all-to-all + all-gather of
        # 64 MiB blocks) — the per-rank xGMI rates DESIGN.md §6's model assumes
        blk = 64 << 20
        a2a_ms, ag_ms = ctx.comm_check(comm, blk)
        moved = (world - 1) * blk / 1e9
        fabric = {"block_MiB": blk >> 20, "all_to_all_ms": round(a2a_ms, 3), "all_gather_ms": round(ag_ms, 3),
                  "all_to_all_GBps_per_rank": round(moved / (a2a_ms / 1e3), 1),
                  "all_gather_GBps_per_rank": round(moved / (ag_ms / 1e3), 1)}
        rccl_ranks = comm.backend_world  # ncclCommCount: the ranks RCCL itself joined
        steps = 10
        host = wl["trace"].data
        d_tr = ctx.alloc(host.nbytes)
        ctx.to_device(d_tr, host)

        def once():  # every rank holds the trace in its HBM
            return ctx.prove_sharded(comm, wl["air_id"], d_tr, pub, wl["opts"], shape=(wl["width"], wl["n"]))

        def once_host():  # each rank uploads its row slice of the host trace (all-gather)
            return ctx.prove_sharded(comm, wl["air_id"], host, pub, wl["opts"])
        elapsed, _, (proof, _) = timed_replicas(once, steps, 2, dist=dist, device_sync=torch.cuda.synchronize,
                                                device=f"cuda:{local_rank}")
        el_host, _, _ = timed_replicas(once_host, steps, 1, dist=dist, device_sync=torch.cuda.synchronize,
                                       device=f"cuda:{local_rank}")
        check = sharded_self_check(ctx, wl, pub, proof, rank, world, dist, local_rank)
    finally:
        comm.close()
    done.set()
    return {"metric": "STARK proofs/sec + prove-time ms, MiMC AIR 2^22-step trace, one proof domain-sharded over "
                      "all GPUs", "workload": wl["workload"], "value": round(steps / elapsed, 3), "unit": "proofs/s",
            "ms_per_proof": round(elapsed / steps * 1e3, 3), "steps": steps, "warmup": 2, "scaling": "strong",
            "step": "zkp_prove_sharded from the trace in every rank's HBM",
            "pcie_inclusive": {"ms_per_proof": round(el_host / steps * 1e3, 3),
                               "proofs_per_s": round(steps / el_host, 3),
                               "step": "zkp_prove_sharded from the host trace: each rank uploads its row slice"},
            "parallelism": f"coset-sharded{world} (RCCL)", "rccl_comm_count": rccl_ranks,
            "proof_bytes": len(proof), "fabric": fabric, **check,
            "bytes_per_proof_8d": sum(stage_bytes(1, 1 << 22, 8, 8, 6).values())}


def emulate_rank(ctx, wl, world: int, rank: int = 0, steps: int = 3) -> dict:
    """Device work of ONE rank of a `world`-rank coset-sharded proof, run alone on this GPU:
    `zkp_prove_sharded` over a loopback caller transport (every collective fills each
    receive block with this rank's own data through host memory), so the rank's kernels
    have exactly the shapes and counts of a `world`-GPU run while no other rank shares the
    device. Device time = the union of the proof's kernel intervals over all its streams
    (the library's per-launch HIP events, `host_device_busy`), beside their plain sum. The
    exchanged data is not a real peer's, so the proof bytes are meaningless (a host-replay
    rejection still leaves the kernel statistics)."""
    import ctypes
    from zk_stark_project_amd import _native
    width, n, opts = wl["width"], wl["n"], wl["opts"]
    pub = wl["prover"].get_pub_inputs(wl["trace"]).to_elements()
    d = ctx.alloc(wl["trace"].data.nbytes)
    ctx.to_device(d, wl["trace"].data)
    R, r = world, rank
    moved = {"a2a": 0, "ag": 0, "calls": 0}

    def a2a(send, recv, block):
        moved["a2a"] += (R - 1) * block
        moved["calls"] += 1
        for s in range(R):
            ctypes.memmove(recv + s * block, send + r * block, block)

    def ag(send, recv, nbytes):
        moved["ag"] += (R - 1) * nbytes
        moved["calls"] += 1
        if nbytes == 16:
            # the shortcut checks' flags (LastCol, GlobalUpdate pairing): the loopback data
            # makes them fail, and a valid proof's flags are zero, so report zeros and time
            # the path a valid proof takes (not a second, unshortcut proof)
            ctypes.memset(recv, 0, R * nbytes)
            return
        for s in range(R):
            ctypes.memmove(recv + s * nbytes, send, nbytes)

    comm = _native.host_comm(r, R, a2a, ag) if R > 1 else _native.local_group(1)[0]

    def once():
        try:
            ctx.prove_sharded(comm, wl["air_id"], d, pub, opts, shape=(width, n))
            return "ok"
        except _native.ZkpError as e:  # the loopback data may fail the host replay
            return f"rejected ({e})"
    try:
        once()  # warm: domain tables, buffers
        ctx.reset_stats()
        ctx.set_profiling(True)
        for k in moved:
            moved[k] = 0
        t0 = time.perf_counter()
        status = [once() for _ in range(steps)][-1]
        wall = (time.perf_counter() - t0) / steps * 1e3
        st = ctx.stats_table()
        ctx.set_profiling(False)
    finally:
        comm.close()
        ctx.free(d)
    busy = st.pop("host_device_busy", {"ms": 0.0})
    kern = {k: v for k, v in st.items() if not k.startswith("host_")}
    return {"world": R, "rank": r, "status": status.split(" (")[0],
            "device_busy_ms_per_proof": round(busy["ms"] / steps, 3),
            "kernel_event_sum_ms_per_proof": round(sum(v["ms"] for v in kern.values()) / steps, 3),
            "launches_per_proof": sum(v["launches"] for v in kern.values()) / steps,
            "wall_ms_with_host_loopback": round(wall, 3),
            "exchange_MiB_in_per_proof": round((moved["a2a"] + moved["ag"]) / steps / 2**20, 1),
            "collectives_per_proof": moved["calls"] / steps,
            "by_kernel_ms": {k: round(v["ms"] / steps, 4) for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["ms"])}}


def rank_emulation_leg(ctx, world: int = 8, steps: int = 3) -> dict:
    """One rank of the 8-rank C4 proof (BASELINE configs[3]: MiMC 2^22, blowup 8, domain-
    sharded; the single proof /root/reference/src/main.rs:468 would split) on this one GPU
    (`emulate_rank`), beside the whole world-1 proof by the same method. The exchange is
    priced separately: its volume at 7 xGMI links x 50-64 GB/s, as the
    lower and upper bound of the exposed part (all hidden / none hidden)."""
    wl = make_workload("mimc", True, None, 8, 0, ctx)
    one = emulate_rank(ctx, wl, world, 0, steps)
    w1 = emulate_rank(ctx, wl, 1, 0, steps)
    xgmi_lo, xgmi_hi = 7 * 50e9, 7 * 64e9
    ex_ms = (one["exchange_MiB_in_per_proof"] * 2**20 / xgmi_hi * 1e3,
             one["exchange_MiB_in_per_proof"] * 2**20 / xgmi_lo * 1e3)
    busy, busy1 = one["device_busy_ms_per_proof"], w1["device_busy_ms_per_proof"]
    return {"workload": wl["workload"], "rank": one, "world1": {k: w1[k] for k in (
                "device_busy_ms_per_proof", "kernel_event_sum_ms_per_proof", "launches_per_proof")},
            "ideal_rank_busy_ms": round(busy1 / world, 3),
            "rank_busy_over_ideal": round(busy / (busy1 / world), 3) if busy1 else None,
            "xgmi_exchange_ms_if_serialized": [round(x, 3) for x in ex_ms],
            "modelled_speedup_vs_world1": [round(busy1 / (busy + ex_ms[1]), 2), round(busy1 / busy, 2)],
            "model": "speed-up = world-1 device busy / (rank device busy + exchange): exchange fully exposed at "
                     "50 GB/s per link .. fully hidden; measured on one GPU, the exchange is not"}


NUM_COEFFS = {"mimc": 3, "agg": 180}  # ConstraintCompositionCoefficients: transitions + assertions


def session_leg(ctx, wl, pub, tr, steps: int) -> dict:
    """ms per proof through the stage hooks (zkp_session_* + zkp_channel_*, the route
    of DESIGN.md §1 that keeps winterfell's Prover::prove), host trace in, openings
    out; checked against the zkp_prove transcript of the same trace."""
    from zk_stark_project_amd import _native
    air = "mimc" if wl["air_id"] == 1 else "agg"

    def once():
        return _native.prove_by_stages(ctx, wl["air_id"], wl["trace"].data, pub, wl["opts"], NUM_COEFFS[air])
    got = once()  # warm (the session context's domain tables)
    stage_ms = {}
    t0 = time.perf_counter()
    for _ in range(steps):
        got = _native.prove_by_stages(ctx, wl["air_id"], wl["trace"].data, pub, wl["opts"], NUM_COEFFS[air],
                                      times=stage_ms)
    ms = (time.perf_counter() - t0) / steps * 1e3
    want = tr.summary()
    same = (got["trace_root"].hex() == want["trace_root"] and got["constraint_root"].hex() == want["constraint_root"]
            and [r.hex() for r in got["fri_roots"]] == want["fri_roots"] and got["z"] == want["z"]
            and got["pow_nonce"] == want["pow_nonce"] and got["query_positions"] == want["query_positions"])
    return {"session_ms": round(ms, 3), "steps": steps, "equals_zkp_prove_transcript": same,
            "stage_ms": {k: round(v / steps, 3) for k, v in stage_ms.items()},
            "route": "zkp_session_trace_lde -> zkp_eval_constraints -> zkp_composition_commit -> zkp_ood_frame -> "
                     "zkp_deep_fri -> zkp_grind -> zkp_query, coefficients from zkp_channel (host)"}


def concurrent_leg(wl, pub, want: bytes, in_flight: int = 3, seconds: float = 1.5) -> dict:
    """Proofs/s on this GPU with `in_flight` proofs at once: that many host threads,
    each with its own zkp_ctx (own streams and HBM buffers) and its own copy of the
    trace in HBM, proving back to back (ctypes drops the GIL inside zkp_prove_device).
    One proof's latency-bound phases (tree tops, FRI tail, coin steps, grinding's
    search end) then overlap another's bandwidth-bound kernels. Reported beside the
    headline, which keeps one proof in flight."""
    from zk_stark_project_amd import _native
    ctxs = [_native.Context(0) for _ in range(in_flight)]
    host = wl["trace"].data
    dts = []
    for c in ctxs:
        d = c.alloc(host.nbytes)
        c.to_device(d, host)
        dts.append(d)
    same = True
    for c, d in zip(ctxs, dts):  # warm: each context's domain tables
        p, _ = c.prove_device(wl["air_id"], d, wl["width"], wl["n"], pub, wl["opts"])
        same = same and p == want
    counts = [0] * in_flight
    stop = threading.Event()

    def worker(i):
        nonlocal same
        while not stop.is_set():
            p, _ = ctxs[i].prove_device(wl["air_id"], dts[i], wl["width"], wl["n"], pub, wl["opts"])
            same = same and p == want
            counts[i] += 1
    th = [threading.Thread(target=worker, args=(i,)) for i in range(in_flight)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    time.sleep(seconds)
    stop.set()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    total = sum(counts)
    return {"in_flight": in_flight, "proofs": total, "seconds": round(dt, 3),
            "proofs_per_s": round(total / dt, 3), "ms_per_proof_amortized": round(dt / total * 1e3, 3),
            "latency_ms_per_proof": round(dt / max(1, min(counts)) * 1e3, 3),
            "proof_bytes_identical": same,
            "step": "zkp_prove_device from HBM, one zkp_ctx and host thread per proof in flight"}


def sharded_self_check(ctx, wl, pub, proof, rank: int, world: int, dist, local_rank: int) -> dict:
    """After the timed sharded proofs (outside the timed region): every rank checks its
    last proof with the product verifier (zkp_verify) and hashes its bytes; rank 0 also
    proves the same trace on its one GPU (zkp_prove) and compares. The flags and
    hashes are all-gathered, so the line says whether every rank's RCCL proof is the
    world-1 proof, byte for byte."""
    import hashlib
    import torch
    from zk_stark_project_amd._native import verify_status
    ok = verify_status(wl["air_id"], proof, pub, wl["opts"]) == 0
    exact = True
    if rank == 0:
        ref, _ = ctx.prove(wl["air_id"], wl["trace"].data, pub, wl["opts"])
        exact = ref == proof
    h = int.from_bytes(hashlib.blake2b(proof, digest_size=7).digest(), "little")
    mine = torch.tensor([h, int(ok), int(exact)], dtype=torch.int64, device=f"cuda:{local_rank}")
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    rows = [t.tolist() for t in allv]
    same = all(r[0] == rows[0][0] for r in rows)
    return {"verified": all(r[1] for r in rows), "bit_exact_vs_world1": bool(rows[0][2]) and same,
            "ranks_identical": same,
            "self_check": "zkp_verify on every rank; rank 0's world-1 zkp_prove of the same trace vs the sharded "
                          "bytes; every rank's proof hash all-gathered"}

def measure(ctx, headline, steps: int, warmup: int, dist=None, sync=None, device=None) -> dict:
    """One workload's timing: the first proof of a fresh shape (domain tables built cold),
    two untimed proofs with every launch bracketed by HIP events (the per-kernel table,
    which names the dominant kernel), the rest of the warm-up, then `steps` timed proofs
    in which only the dominant kernel's launches carry events (its roofline is measured
    live at ~no event overhead)."""
    from zk_stark_project_amd.replicas import timed_replicas
    t0 = time.perf_counter()
    headline()
    first_ms = (time.perf_counter() - t0) * 1e3
    ctx.reset_stats()
    ctx.set_profiling(True)
    for _ in range(2):
        headline()
    ctx.set_profiling(False)
    kernels = {k: v for k, v in ctx.stats_table().items() if not k.startswith("host_")}
    dom_name = max(kernels.items(), key=lambda kv: kv[1]["ms"])[0]
    for _ in range(max(warmup - 1, 0)):  # the rest of the W warm-up steps (the first proof was one)
        headline()
    ctx.reset_stats()
    ctx.set_profiling(True, kernel=dom_name)
    times = []
    elapsed, _, (proof, tr) = timed_replicas(headline, steps, 0, dist=dist, device_sync=sync, device=device,
                                              times=times)
    ctx.set_profiling(False)
    return {"first_ms": first_ms, "kernels": kernels, "dom_name": dom_name, "elapsed": elapsed, "times": times,
            "proof": proof, "tr": tr, "stats": ctx.stats_table()}


def step_summary(times) -> dict:
    """Per-step wall times of the timed region (ms): mean, median, min, max."""
    ts = sorted(t * 1e3 for t in times)
    k = len(ts)
    med = ts[k // 2] if k % 2 else (ts[k // 2 - 1] + ts[k // 2]) / 2
    return {"mean": round(sum(ts) / k, 3), "median": round(med, 3), "min": round(ts[0], 3),
            "max": round(ts[-1], 3), "n": k}


def launches_of(kernels: dict) -> dict:
    """Every launch of the two profiled proofs (HIP events per launch, side stream included)."""
    total_ms = sum(v["ms"] for v in kernels.values())
    return {"per_proof": sum(v["launches"] for v in kernels.values()) / 2,
            "kernel_ms_per_proof": round(total_ms / 2, 3),
            "by_kernel_ms": {k: round(v["ms"] / 2, 4) for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["ms"])}}


def roofline_of(m: dict, wl: dict, R: int, steps: int, ms: float, air: str, mode: str) -> dict:
    """The dominant kernel's roofline: SURVEY.md §8(d) algorithmic bytes per launch ÷ its
    average HIP-event duration in the timed region; PMC traffic and VALU issue from the
    committed summaries of the same workload; the NTT's butterfly floor."""
    kernels, stats, dom_name = m["kernels"], m["stats"], m["dom_name"]
    B, n = wl["opts"].blowup_factor, wl["n"]
    sb = stage_bytes(wl["width"], n, B, wl["ce"], wl["C"])
    bytes_per_proof = sum(sb.values())
    total_ms = sum(v["ms"] for v in kernels.values())
    dom = stats[dom_name]  # HIP events of the timed region
    dom_avg_ms = dom["ms"] / dom["launches"]
    launches_per_proof = dom["launches"] / steps
    kbytes, ksrc = kernel_stage_bytes(dom_name, sb, wl, R)
    alg = kbytes / R / launches_per_proof if kbytes else None
    # the NTT's butterfly floor: butterflies of the extended columns' coset NTTs at the
    # micro-benchmark's register-resident rate, against the kernel's time per proof
    valu_floor = None
    if dom_name == "ntt_dit" and floor_rate():
        tcols, ccols = lde_columns(wl, R)
        bfly = (tcols + ccols) * B / R * (n // 2) * wl["log_n"]
        kernel_ms = dom_avg_ms * launches_per_proof
        floor_ms = bfly / (floor_rate() * 1e9) * 1e3
        valu_floor = {"butterflies_per_proof": bfly, "floor_gbfly_per_s": floor_rate(), "floor_ms": round(floor_ms, 4),
                      "kernel_ms_per_proof": round(kernel_ms, 4), "valu_floor_frac": round(floor_ms / kernel_ms, 3),
                      "source": f"{UBENCH_BFLY} (tests/native/ubench_bfly.hip, the library's butterfly forms)"}
    traffic, traffic_src = pmc_traffic(dom_name, air, mode)
    return {
        "bound": "hbm",
        "kernel": dom_name,
        "achieved": round(alg / (dom_avg_ms * 1e-3) / 1e9, 2) if alg else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(alg / (dom_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if alg else None,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "algorithmic_bytes_per_launch": alg,
        "algorithmic_bytes_source": (f"SURVEY.md §8(d)/Appendix C {ksrc} = {kbytes} B per proof / "
                                     f"{launches_per_proof:g} launches" if kbytes else None),
        "traffic_over_algorithmic": round(traffic / alg, 2) if traffic and alg else None,
        "traffic_model_per_launch": dom["bytes"] / dom["launches"],
        "avg_launch_ms": round(dom_avg_ms, 5),
        "launches_per_proof": launches_per_proof,
        "share_of_device_time": round(kernels[dom_name]["ms"] / total_ms, 3) if total_ms else None,
        "whole_proof_frac": round(bytes_per_proof / R / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "bytes_per_proof_8d": bytes_per_proof,
        "valu": valu_side(dom_name, air, mode),
        "valu_floor_frac": valu_floor["valu_floor_frac"] if valu_floor else None,
        "valu_floor": valu_floor,
    }


def c3_leg(ctx, steps: int, warmup: int, check: bool) -> dict:
    """BASELINE configs[2] / SURVEY §8(d) C3 on the same GPU: the GlobalUpdate AIR over 64
    device updates padded to 2^18 rows x 120 columns (/root/reference/src/aggregation/
    prover.rs:98-160), the reference's options (src/main.rs:98-107: 40, 16, 21, None, 16,
    7, Algebraic, Algebraic). Same step as the headline (zkp_prove from the host trace),
    its own roofline, and — after the timed region — the proof checked byte for byte
    against the C oracle's proof of the same trace."""
    wl = make_workload("agg", False, None, 16, 0, ctx)
    pub = wl["prover"].get_pub_inputs(wl["trace"]).to_elements()
    host = wl["trace"].data
    d_tr = ctx.alloc(host.nbytes)
    ctx.to_device(d_tr, host)
    try:
        m = measure(ctx, lambda: ctx.prove(wl["air_id"], host, pub, wl["opts"]), steps, warmup)
        el_in, _, _ = timed_replicas_plain(
            lambda: ctx.prove_device(wl["air_id"], d_tr, wl["width"], wl["n"], pub, wl["opts"]), steps)
    finally:
        ctx.free(d_tr)
    tampered = tampered_leg(ctx, wl, pub, el_in / steps * 1e3)
    fresh = fresh_buffer_leg(ctx, wl, pub)
    ms = m["elapsed"] / steps * 1e3
    out = {"workload": wl["workload"], "options": "(40, 16, 21, None, 16, 7, Algebraic, Algebraic) (src/main.rs:98-107)",
           "value": round(steps / m["elapsed"], 3), "unit": "proofs/s", "ms_per_step": round(ms, 3),
           "steps": steps, "step_ms": step_summary(m["times"]),
           "step": "zkp_prove: host trace (pageable numpy) -> proof bytes, PCIe upload included",
           "trace_resident": {"ms_per_proof": round(el_in / steps * 1e3, 3), "proofs_per_s": round(steps / el_in, 3)},
           "first_proof_ms": round(m["first_ms"], 3),
           "roofline": roofline_of(m, wl, 1, steps, ms, "agg", "replicas"),
           "tampered": tampered, "fresh_host_buffer": fresh, "launches": launches_of(m["kernels"]),
           "proof_bytes": len(m["proof"])}
    if check:
        import oracle_ref
        t0 = time.perf_counter()
        ref, _ = oracle_ref.prove(wl["air_id"], wl["trace"].to_bytes(), wl["width"], wl["n"],
                                  b"".join(v.to_bytes(16, "little") for v in pub), wl["opts"])
        out["oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        out["oracle_threads"] = oracle_ref.lib().oracle_num_threads()
        out["proof_bytes_identical"] = ref == m["proof"]
    return out


def timed_replicas_plain(fn, steps: int):
    """`steps` back-to-back calls after one warm-up call (single rank): (elapsed, None, last)."""
    from zk_stark_project_amd.replicas import timed_replicas
    return timed_replicas(fn, steps, 1)


def fresh_buffer_leg(ctx, wl, pub, reps: int = 3) -> dict:
    """The headline step on a trace in host pages never uploaded before (a caller's next
    trace): the timed steps reuse one host array, whose pages the runtime has already
    locked for DMA after the first upload; a fresh buffer pays that again (≈ 2 ms for
    C3's 503 MB). Copies made before timing; proof bytes must not change."""
    import numpy as np
    host = wl["trace"].data
    copies = [np.array(host, copy=True) for _ in range(reps)]
    want, _ = ctx.prove(wl["air_id"], host, pub, wl["opts"])
    ms, same = [], True
    for h in copies:
        t0 = time.perf_counter()
        p, _ = ctx.prove(wl["air_id"], h, pub, wl["opts"])
        ms.append((time.perf_counter() - t0) * 1e3)
        same = same and p == want
    return {"ms_per_proof": round(sum(ms) / len(ms), 3), "proofs": reps, "proof_bytes_identical": same,
            "step": "zkp_prove from a freshly allocated copy of the host trace (pageable numpy)"}


def tampered_leg(ctx, wl, pub, valid_ms: float, reps: int = 5) -> dict:
    """A device-resident trace that breaks its AIR (MiMC: one transition; GlobalUpdate:
    one derived column entry, so a pair fails) proved like the headline's
    `trace_resident` step. The proof's exact shortcuts rest on a valid trace
    (DESIGN.md §2): such a trace is caught by the early trace check and proven without
    them in the same call, not by a second proof."""
    bad = wl["trace"].data.copy()
    n = wl["n"]
    if wl["air_id"] == 1:
        bad[0, n // 2, 0] ^= 1  # row n/2 no longer follows from row n/2 - 1
    else:
        bad[wl["width"] // 2 + 3, n // 3, 0] ^= 1  # column 63 breaks its pairing with column 3
    d = ctx.alloc(bad.nbytes)
    try:
        ctx.to_device(d, bad)
        ctx.prove_device(wl["air_id"], d, wl["width"], n, pub, wl["opts"])  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.prove_device(wl["air_id"], d, wl["width"], n, pub, wl["opts"])
        ms = (time.perf_counter() - t0) / reps * 1e3
    finally:
        ctx.free(d)
    return {"ms_per_proof": round(ms, 3), "over_valid_trace_resident": round(ms / valid_ms, 3), "proofs": reps,
            "tamper": "one MiMC transition broken" if wl["air_id"] == 1 else "one GlobalUpdate pair broken"}


REF_FLOW_DEVICES, REF_FLOW_BS = 8, 50


REF_FLOW_IN_FLIGHT = 4


def reference_flow_concurrent(device: int, jobs, opts, want, in_flight: int = REF_FLOW_IN_FLIGHT) -> dict:
    """The same proof step with its proofs in flight together: `in_flight` host threads, each
    with its own zkp_ctx (streams, HBM buffers), take the 9 proofs of the step from a queue
    (the reference's per-device loop, src/main.rs:379-439, as a parallel map; the GlobalUpdate
    proof of :441-493 first — its trace needs the devices' updates, not their proofs); each
    proof verified. One small proof's latency-bound phases
    (tree tops, transcript steps, the FRI tail) overlap another's transforms. Not the drop-in
    call sequence: a Rust caller gets it from a parallel iterator over the devices, one
    context per worker."""
    import queue
    from zk_stark_project_amd import _native
    ctxs = [_native.Context(device) for _ in range(in_flight)]
    try:
        for c in ctxs:  # warm: each context's domain tables and buffers at both shapes
            for air, tr, pub in (jobs[0], jobs[-1]):
                c.prove(air, tr.data, pub, opts)
        out = [None] * len(jobs)
        verify = [True]

        def run_all():
            # every proof of the step is independent of the others' proofs (the aggregation's
            # trace needs the devices' updates, which exist before any proof): the GlobalUpdate
            # proof goes first in the queue, so it does not run alone at the end
            q = queue.Queue()
            for k in [len(jobs) - 1] + list(range(len(jobs) - 1)):
                q.put(k)
            errs = []

            def worker(c):
                while True:
                    try:
                        k = q.get_nowait()
                    except queue.Empty:
                        return
                    try:
                        air, tr, pub = jobs[k]
                        p, _ = c.prove(air, tr.data, pub, opts)
                        if verify[0]:
                            _native.verify(air, p, pub, opts)
                        out[k] = p
                    except Exception as e:  # noqa: BLE001 — re-raised below
                        errs.append(e)
                        return
            th = [threading.Thread(target=worker, args=(c,)) for c in ctxs]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errs:
                raise errs[0]
        run_all()  # warm
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            run_all()
        ms = (time.perf_counter() - t0) / reps * 1e3
        verify[0] = False  # the proofs alone, as the sequential leg's prove_ms_total
        t0 = time.perf_counter()
        for _ in range(reps):
            run_all()
        prove_ms = (time.perf_counter() - t0) / reps * 1e3
    finally:
        for c in ctxs:
            c.close()
    return {"in_flight": in_flight, "flow_ms": round(ms, 3), "prove_ms_total": round(prove_ms, 3),
            "repetitions": reps,
            "proofs_identical_to_sequential": out == want,
            "step": f"the GlobalUpdate proof and the {len(jobs) - 1} TrainingUpdate proofs from {in_flight} host threads "
                    "(one zkp_ctx each); flow_ms: each verified (zkp_verify on the proving thread), prove_ms_total: "
                    "the proofs alone; means over the repetitions"}


def reference_flow_leg(device: int, check: bool) -> dict:
    """The reference binary's proof step (/root/reference/src/main.rs:374-493, `--step proof
    --bs 50`): one TrainingUpdate proof per device (bs = 50 samples: n = 8192 rows, w = 240,
    src/training/prover.rs:63), each verified, then the GlobalUpdate proof over the
    devices' last-row values (8 updates: n = 16), verified; the reference's options
    (src/main.rs:98-107, blowup 16). The harness (verification/time_memory_analytics/
    analyze.py:476-482) reads the aggregation's "proof: Tms".

    Timed on a FRESH zkp_ctx — every shape's domain tables and buffers built on first use,
    as the reference's fresh process does — (`cold`), then again on the same context
    (`warm`). The 8 synthetic devices hold 60 seeded rows of 9 features + a label
    (the Device_* CSV layout, helper.rs:55-80). Traces are built once beforehand by the
    host mirror of the trace builders (Python; `trace_build_ms`), outside the proof
    timings, like the reference times `proof:` apart from `trace:`. With `check`, every
    proof is compared with the C oracle's proof of the same trace (`oracle_ms` per proof)."""
    import random
    from zk_stark_project_amd import AIR_GLOBAL_UPDATE, AIR_TRAINING_UPDATE, _native, cli
    from zk_stark_project_amd.helper import FE, EdgeDevice
    from zk_stark_project_amd.options import ProofOptions
    opts = ProofOptions.reference()
    rng, drng = random.Random(2024), random.Random(99)
    devs = [EdgeDevice([[drng.uniform(-2, 2) for _ in range(FE)] for _ in range(60)],
                       [float(drng.randrange(1, 9)) for _ in range(60)], random.Random(rng.getrandbits(64)))
            for _ in range(REF_FLOW_DEVICES)]
    t0 = time.perf_counter()
    jobs = []
    for d in devs:
        tp = cli._training_prover(opts, cli._zk_batch(d, REF_FLOW_BS), REF_FLOW_BS, rng, None)
        tr = tp.build_trace()
        jobs.append((AIR_TRAINING_UPDATE, tr, tp.get_pub_inputs(tr).to_elements()))
    agg = cli._aggregator(opts, [tr.get(0, tr.length() - 1) for _, tr, _ in jobs], rng, None)
    agg_tr = agg.build_trace()
    jobs.append((AIR_GLOBAL_UPDATE, agg_tr, agg.get_pub_inputs(agg_tr).to_elements()))
    build_ms = (time.perf_counter() - t0) * 1e3

    def run(ctx):
        proofs, prove_ms = [], []
        t_all = time.perf_counter()
        for air, tr, pub in jobs:
            t1 = time.perf_counter()
            p, _ = ctx.prove(air, tr.data, pub, opts)
            prove_ms.append((time.perf_counter() - t1) * 1e3)
            _native.verify(air, p, pub, opts)  # main.rs:430-436, 478-484 (zkp_verify, host)
            proofs.append(p)
        total = (time.perf_counter() - t_all) * 1e3
        return proofs, {"training_proof_ms": [round(x, 3) for x in prove_ms[:-1]],
                        "aggregation_proof_ms": round(prove_ms[-1], 3),
                        "prove_ms_total": round(sum(prove_ms), 3), "flow_ms": round(total, 3)}

    t0 = time.perf_counter()
    ctx = _native.Context(device)
    create_ms = (time.perf_counter() - t0) * 1e3
    create_phases = {k[len("host_ctx_"):]: round(v["ms"], 3) for k, v in ctx.stats_table().items()
                     if k.startswith("host_ctx_")}
    try:
        proofs, cold = run(ctx)
        cold["ctx_create_ms"] = round(create_ms, 3)
        cold["ctx_create_phases_ms"] = create_phases  # zkp_ctx_create's own wall clock by phase
        proofs2, warm = run(ctx)
        # the TrainingUpdate proofs once more with every launch bracketed by HIP events:
        # where a reference-shape proof's time goes (profiled separately: the events
        # themselves cost a few us per launch)
        ctx.reset_stats()
        ctx.set_profiling(True)
        for air, tr, pub in jobs[:-1]:
            ctx.prove(air, tr.data, pub, opts)
        tu_stats = ctx.stats_table()
        ctx.set_profiling(False)
        concurrent = [reference_flow_concurrent(device, jobs, opts, proofs, k) for k in (4, REF_FLOW_DEVICES)]
    finally:
        ctx.close()
    ntu = len(jobs) - 1
    tu_busy = tu_stats.pop("host_device_busy", {"ms": 0.0})["ms"] / ntu
    tu_kern = {k: v for k, v in tu_stats.items() if not k.startswith("host_")}
    w_tu, n_tu = jobs[0][1].width(), jobs[0][1].length()
    tu_ms = sum(warm["training_proof_ms"]) / ntu
    tu_bytes = sum(stage_bytes(w_tu, n_tu, opts.blowup_factor, 2, 1).values())
    tu_profile = {
        "shape": f"n = {n_tu}, w = {w_tu}, blowup {opts.blowup_factor}, ce = 2, C = 1",
        "warm_ms_per_proof": round(tu_ms, 3),
        "device_busy_ms_per_proof": round(tu_busy, 3),
        "launches_per_proof": sum(v["launches"] for v in tu_kern.values()) / ntu,
        "by_kernel": {k: {"launches": v["launches"] / ntu, "ms": round(v["ms"] / ntu, 4)}
                      for k, v in sorted(tu_kern.items(), key=lambda kv: -kv[1]["ms"])},
        # the prover's host-side stage clock (wall ms per proof, the device work inside included)
        "host_stages_ms": {k[len("host_"):]: round(v["ms"] / ntu, 4) for k, v in sorted(tu_stats.items())
                           if k.startswith("host_") and not k.startswith("host_ctx_")},
        "bytes_per_proof_8d": tu_bytes,
        "whole_proof_frac": round(tu_bytes / (tu_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "whole_proof_frac_note": "SURVEY.md §8(d)/Appendix C bytes of one TrainingUpdate proof / its warm wall ms "
                                 "(upload and host replay included) / 8 TB/s"}
    out = {"workload": f"src/main.rs:374-493 --step proof --bs {REF_FLOW_BS}: {REF_FLOW_DEVICES} TrainingUpdate proofs "
                       f"(n = {jobs[0][1].length()}, w = {jobs[0][1].width()}) + GlobalUpdate proof "
                       f"(n = {agg_tr.length()}, w = {agg_tr.width()}), blowup 16, each verified",
           "cold": cold, "warm": warm, "warm_concurrent": concurrent, "training_proof_profile": tu_profile,
           "trace_build_ms": round(build_ms, 1),
           "cold_context": "fresh zkp_ctx: domain tables, twiddles and buffers built on first use of each shape",
           "proof_bytes": [len(p) for p in proofs], "warm_equals_cold": proofs == proofs2}
    if check:
        import oracle_ref
        ms, same = [], True
        for (air, tr, pub), p in zip(jobs, proofs):
            t1 = time.perf_counter()
            ref, _ = oracle_ref.prove(air, tr.to_bytes(), tr.width(), tr.length(),
                                      b"".join(v.to_bytes(16, "little") for v in pub), opts)
            ms.append(round((time.perf_counter() - t1) * 1e3, 1))
            same = same and ref == p
        out["oracle"] = {"training_proof_ms": ms[:-1], "aggregation_proof_ms": ms[-1], "prove_ms_total": round(sum(ms), 1),
                         "threads": oracle_ref.lib().oracle_num_threads()}
        out["proof_bytes_identical"] = same
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1 or args.sharded_leg:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        if world > 1:
            tdist.init_process_group("nccl")
        else:  # world-1 rehearsal outside torchrun
            tdist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1)
        dist = tdist

    def cuda_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()

    from zk_stark_project_amd import _native
    from zk_stark_project_amd.replicas import aggregate_rate, timed_replicas

    ctx = _native.Context(local_rank)
    sharded = args.mode == "sharded"
    wl = make_workload(args.air, sharded, args.log_n, args.blowup, 0 if sharded else rank, ctx)
    air_id, width, n, opts, trace = wl["air_id"], wl["width"], wl["n"], wl["opts"], wl["trace"]
    pub = wl["prover"].get_pub_inputs(trace).to_elements()
    host_trace = trace.data  # (width, n, 2) uint64, pageable host memory
    d_trace = ctx.alloc(host_trace.nbytes)
    ctx.to_device(d_trace, host_trace)

    comm = None
    if sharded:
        from zk_stark_project_amd.sharded import rccl_group_comm
        comm = rccl_group_comm(ctx, rank, world) if world > 1 else _native.local_group(1)[0]

        if args.air == "agg":
            # C5: each rank builds the GlobalUpdate trace in its own HBM from the
            # device updates (zkp_build_global_update_trace, prover.rs:98-160), so
            # no rank uploads the 2 GiB trace; the step = trace build + proof
            d_built = ctx.alloc(host_trace.nbytes)

            def prove_once():
                wl["prover"].build_trace_device(ctx, d_out=d_built)
                return ctx.prove_sharded(comm, air_id, d_built, pub, opts, shape=(width, n))
        else:
            def prove_once():  # host trace -> proof (each rank uploads its row slice; all-gather)
                return ctx.prove_sharded(comm, air_id, host_trace, pub, opts)

        def prove_dev():
            return ctx.prove_sharded(comm, air_id, d_trace, pub, opts, shape=(width, n))
    else:
        def prove_once():  # zkp_prove: host trace -> proof (uploads included)
            return ctx.prove(air_id, host_trace, pub, opts)

        def prove_dev():  # zkp_prove_device: trace resident in HBM
            return ctx.prove_device(air_id, d_trace, width, n, pub, opts)

    # the headline step: SURVEY.md §8(d)'s "prove" — zkp_prove from the host trace,
    # uploads included (C5: the trace built on every rank's device from the updates,
    # then the sharded proof); the trace-resident proof is reported beside it
    headline, second = prove_once, prove_dev
    sync = cuda_sync if dist is not None else None
    m = measure(ctx, headline, args.steps, args.warmup, dist=dist, sync=sync, device=f"cuda:{local_rank}")
    elapsed, proof, tr, kernels, dom_name = m["elapsed"], m["proof"], m["tr"], m["kernels"], m["dom_name"]
    # the same proof with the trace already in HBM (zkp_prove_device / a device-resident
    # sharded proof): reported beside the headline, never as `value`
    el_in, _, _ = timed_replicas(second, args.steps, 1, dist=dist, device_sync=sync, device=f"cuda:{local_rank}")
    # sustained: back-to-back headline proofs for a few seconds (clock / thermal steadiness)
    sus_n, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < args.sustain_s:
        headline()
        sus_n += 1
    sus_s = time.perf_counter() - t1
    tampered = tampered_leg(ctx, wl, pub, el_in / args.steps * 1e3) \
        if (world == 1 and not sharded and args.tampered) else None
    fresh = fresh_buffer_leg(ctx, wl, pub) if (world == 1 and not sharded and args.tampered) else None
    # the stage-hook route (a winter-prover fork keeping Prover::prove): the same proof
    # through zkp_session_* with the host channel drawing every coefficient
    session = None if sharded else session_leg(ctx, wl, pub, tr, min(args.steps, 10))
    # several proofs in flight on this one GPU (a proof service's throughput)
    concurrent = concurrent_leg(wl, pub, proof) if (world == 1 and not sharded and args.concurrent) else None
    # BASELINE configs[2] (C3) on the same GPU, and the reference binary's own proof step
    if world == 1 and not args.no_verify:
        import oracle_ref  # their byte checks run the oracle on every CPU of this job's host share
        oracle_ref.lib().oracle_set_threads(host_cpus())
    c3 = c3_leg(ctx, args.steps, args.warmup, not args.no_verify) if (
        world == 1 and not sharded and args.air == "mimc" and args.c3) else None
    ref_flow = reference_flow_leg(local_rank, not args.no_verify) if (
        world == 1 and not sharded and args.air == "mimc" and args.reference_flow) else None
    # one rank of the 8-GPU C4 proof, emulated on this GPU (driver-observable per-rank cost)
    rank_emu = rank_emulation_leg(ctx) if (
        world == 1 and not sharded and args.air == "mimc" and args.rank_emulation) else None
    # the oracle's verifier (CPU) runs after every timed region, so the GPU does not
    # sit idle (and clock down) just before the timed steps
    verified = None
    if rank == 0 and not args.no_verify:
        import oracle_ref  # tests/ checker: the oracle's verifier accepts the GPU proof
        verified = oracle_ref.verify(air_id, proof, b"".join(v.to_bytes(16, "little") for v in pub), opts) == 0

    if comm is not None:
        comm.close()
    run_sharded = (world > 1 or args.sharded_leg) and not sharded and not args.no_sharded_leg
    if rank != 0:
        failed = False
        if run_sharded:  # collective with rank 0's leg below
            try:
                sharded_leg(ctx, rank, world, dist, local_rank)
            except Exception as e:  # noqa: BLE001 — rank 0 reports the leg; this rank exits non-zero
                print(json.dumps({"error": f"sharded leg failed on rank {rank}: {type(e).__name__}: {e}"}),
                      file=sys.stderr, flush=True)
                failed = True
        if dist is not None:
            dist.destroy_process_group()
        if failed:
            sys.exit(1)
        return

    R = world if sharded else 1
    B = opts.blowup_factor
    host_stages = {k: v for k, v in m["stats"].items() if k.startswith("host_")}
    ms = elapsed / args.steps * 1e3
    roofline = roofline_of(m, wl, R, args.steps, ms, args.air, args.mode)

    cpu = None
    c1 = None
    if world == 1 and not args.no_cpu_baseline and not sharded:
        import oracle_ref
        # the whole host share this job may use (cgroup quota / affinity), not an inherited
        # OMP_NUM_THREADS: the oracle's OpenMP regions run on every CPU available to it
        oracle_ref.lib().oracle_set_threads(host_cpus())
        if args.air == "mimc":
            c1 = c1_leg(ctx)
        tb = trace.to_bytes()
        pb = b"".join(v.to_bytes(16, "little") for v in pub)
        # bounded sample: whole proofs of the same workload until >= 10 s of CPU work (at most 5)
        t1 = time.perf_counter()
        count, same = 0, True
        while True:
            cproof, _ = oracle_ref.prove(air_id, tb, width, n, pb, opts)
            count += 1
            same = same and cproof == proof
            dt = time.perf_counter() - t1
            if dt >= 10.0 or count >= 5:
                break
        cpu = {
            "value": round(count / dt, 5),
            "unit": "proofs/s",
            "cores": oracle_ref.lib().oracle_num_threads(),
            "kind": "port",
            "host": host_info(),
            "sample": f"{count} full proof(s) of the same workload ({wl['workload']}) by the C oracle restating the "
                      f"winterfell 0.12 CPU path (OpenMP threads = cores = every CPU of this job's host share: "
                      f"cgroup quota / affinity, of {os.cpu_count()} on the machine), {dt * 1e3:.0f} ms in all; "
                      f"proof bytes identical to GPU: {same}",
        }

    metric = (f"STARK proofs/sec + prove-time ms, MiMC AIR 2^{wl['log_n']}-step trace" if args.air == "mimc"
              else f"STARK proofs/sec + prove-time ms, aggregation AIR 2^{wl['log_n']}-step trace")
    if sharded:
        metric += ", one proof domain-sharded over all GPUs"
    out = {
        "metric": metric,
        "value": round(aggregate_rate(1 if sharded else world, args.steps, elapsed), 3),
        "unit": "proofs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong" if sharded else "weak",
        "vs_baseline": None,
        "dtype": "f128 (u128 mod 2^128-45*2^40+1)",
        "data": "synthetic (MiMC trace x0=42e6+rank)" if args.air == "mimc" else "synthetic (seeded u64 model entries)",
        "config": {"workload": wl["workload"],
                   "trace_length": n, "trace_width": width, "blowup": B, "num_queries": 40, "grinding": 21,
                   "fri_folding": 16, "fri_remainder_max_degree": 7,
                   "parallelism": f"coset-sharded{world} (RCCL)" if sharded else f"replicas{world}",
                   "env": zkp_env(),
                   "step": ("GlobalUpdate trace built on each rank's device from the updates + zkp_prove_sharded"
                            if sharded and args.air == "agg" else
                            "zkp_prove_sharded from the host trace: each rank uploads its row slice" if sharded else
                            "zkp_prove: host trace (pageable numpy) -> proof bytes, PCIe upload included "
                            "(SURVEY.md §8(d) 'prove')")},
        "step_ms": step_summary(m["times"]),
        "trace_resident": {
            "ms_per_proof": round(el_in / args.steps * 1e3, 3),
            "proofs_per_s": round(aggregate_rate(1 if sharded else world, args.steps, el_in), 3),
            "step": ("zkp_prove_sharded on a trace already in every rank's HBM" if sharded else
                     "zkp_prove_device: trace resident in HBM -> proof bytes on the host")},
        "first_proof_ms": round(m["first_ms"], 3),
        "sustained": {"proofs": sus_n, "seconds": round(sus_s, 3), "proofs_per_s": round(sus_n / sus_s, 3)},
        "concurrent": concurrent,
        "tampered": tampered,
        "fresh_host_buffer": fresh,
        "session": ({**session, "over_zkp_prove": round(session["session_ms"] / ms, 3)} if session else None),
        "roofline": roofline,
        # every launch of the two profiled proofs (HIP events per launch, side stream included)
        "launches": launches_of(kernels),
        "cpu_baseline": cpu,
        "c1": c1,
        "c3": c3,
        "reference_flow": ref_flow,
        "rank_emulation": rank_emu,
        "proof_bytes": len(proof),
        "verified_by_oracle": verified,
        "parity": "bit-exact vs the C oracle; parity vs winterfell 0.12 bytes unpinned (DESIGN.md §2)",
    }
    if run_sharded:
        def headline_on_timeout():
            print(json.dumps({**out, "sharded": {"error": "timed out (watchdog)"}}), flush=True)
        try:
            out["sharded"] = sharded_leg(ctx, rank, world, dist, local_rank, on_timeout=headline_on_timeout)
        except Exception as e:  # noqa: BLE001 — reported in the line, the headline stands
            out["sharded"] = {"error": f"{type(e).__name__}: {e}"}
    print(json.dumps(out), flush=True)
    if args.stats:
        for k, v in sorted(host_stages.items()):
            print(f"{k:26s} calls={v['launches']:6d} wall_ms={v['ms']:9.3f}", file=sys.stderr)
        for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["ms"]):
            print(f"{k:20s} launches={v['launches']:6d} ms={v['ms']:9.3f} "
                  f"GB/s={v['bytes'] / (v['ms'] * 1e-3) / 1e9 if v['ms'] else 0:9.1f}", file=sys.stderr)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    main()
