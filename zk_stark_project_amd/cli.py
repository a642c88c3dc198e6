"""`zk_stark_project --step {setup,witness,proof} --data-dir D --bs B [--verbose]`.

The reference binary's CLI (/root/reference/src/main.rs:55-74, flow :79-493)
driven by the MI355X prover: per-device TrainingUpdate proofs, then the
GlobalUpdate aggregation proof, each verified like the reference does. The
stdout lines the reference prints are kept verbatim because the Python
harness parses them (/root/reference/verification/time_memory_analytics/
analyze.py:416-506, regexes :476-482): "Training proof size: N bytes",
"proof: Tms, N bytes", "Proof size: N bytes", "Total training proof size",
"Aggregation proof size", "Total proof size".

Launch it as `bin/zk_stark_project ...` (or `python -m zk_stark_project_amd.cli`);
INTEGRATION.md shows where the harness expects the executable.
"""
from __future__ import annotations

import argparse
import os
import random
import sys
import time

SAMPLE_SIZE = 50  # main.rs:77


def _parse(argv):
    ap = argparse.ArgumentParser(prog="zk_stark_project", description="STARK Aggregator with built-in training")
    ap.add_argument("--step", default="setup", type=str.lower, choices=["setup", "witness", "proof"],
                    help="step to run: setup, witness, or proof")
    ap.add_argument("--data-dir", default="devices/edge_device/data",
                    help="path to folder containing Device_*/data files")
    ap.add_argument("--bs", type=int, default=1, help="batch size for the ZK circuit")
    ap.add_argument("--verbose", action="store_true", help="Enable verbose output for benchmarking")
    # not in the reference: the reference draws masks/models/batches from thread_rng
    ap.add_argument("--seed", type=int, default=None, help="seed every random draw (reproducible runs)")
    ap.add_argument("--device", type=int, default=int(os.environ.get("ZKP_DEVICE", "0")),
                    help="HIP device ordinal")
    return ap.parse_args(argv)


def _ms(t0):
    return int((time.perf_counter() - t0) * 1000)


def _load_devices(data_dir, verbose, rng):
    from .helper import EdgeDevice, read_dataset
    devices = []
    for name in sorted(os.listdir(data_dir)):  # main.rs:112-141
        path = os.path.join(data_dir, name)
        if not os.path.isdir(path) or not name.startswith("Device_"):
            continue
        ds = os.path.join(path, "train.txt")
        if not os.path.exists(ds):
            ds = os.path.join(path, "device_data.txt")
        if not os.path.exists(ds):
            if verbose:
                print(f"Warning: no data file in {path}, skipping", file=sys.stderr)
            continue
        if verbose:
            print(f"Loading {ds}")
        feats, labs = read_dataset(ds)
        devices.append(EdgeDevice(feats, labs, random.Random(rng.getrandbits(64))))
    return devices


def _zk_batch(dev, bs):
    """main.rs:164-192: first `bs` of SAMPLE_SIZE sampled rows -> felts, one-hot labels, zero signs."""
    from .helper import AC, FE, f64_to_felt, label_to_one_hot
    host_feats, host_labs = dev.next_batch(SAMPLE_SIZE)
    if len(host_feats) < bs:
        return None
    feats = [[f64_to_felt(v) for v in row] for row in host_feats[:bs]]
    labs = [label_to_one_hot(lab, AC, 1e6)[0] for lab in host_labs[:bs]]
    return feats, [[0] * FE for _ in feats], labs


def _training_prover(opts, batch, bs, rng, ctx):
    from .helper import AC, FE, f64_to_felt, generate_initial_model
    from .prover import TrainingUpdateProver
    feats, feats_sign, labs = batch
    init_w, init_w_sign, init_b, init_b_sign = generate_initial_model(FE, AC, 1.0, rng)
    return TrainingUpdateProver(opts, init_w, init_b, init_w_sign, init_b_sign, feats, feats_sign, labs,
                                f64_to_felt(0.0001), f64_to_felt(1e6), bs, mask_seed=rng.getrandbits(63), ctx=ctx)


def _aggregator(opts, client_reps, rng, ctx):
    """main.rs:241-269: local models from the clients' last-row values, N(0, 1e4) global model."""
    from .helper import AC, FE, f64_to_felt, generate_initial_model
    from .prover import GlobalUpdateProver
    local_w, local_b = [], []
    for rep in client_reps:
        v = float(rep) / 1e6  # rep.as_int() as f64 / 1e6
        local_w.append([[f64_to_felt(v)] * FE for _ in range(AC)])
        local_b.append([f64_to_felt(v)] * AC)
    g_w, _, g_b, _ = generate_initial_model(FE, AC, 10_000.0, rng)
    k = f64_to_felt(float(len(client_reps)))
    return GlobalUpdateProver(opts, g_w, g_b, local_w, local_b, k,
                              blinding=[rng.getrandbits(64) for _ in range(60)], ctx=ctx)


def main(argv=None) -> int:
    args = _parse(argv)
    overall = time.perf_counter()
    if args.bs == 0:
        print("Error: ZK circuit batch size must be positive", file=sys.stderr)
        return 1
    if args.bs > SAMPLE_SIZE:
        print(f"Error: ZK circuit batch size ({args.bs}) cannot exceed sample size ({SAMPLE_SIZE})", file=sys.stderr)
        return 1
    print(f"DEBUG: Starting with batch size = {args.bs}")
    print(f"DEBUG: Step = {args.step.capitalize()}")

    from . import _native
    from .air import GlobalUpdateAir, TrainingUpdateAir
    from .options import ProofOptions
    from .prover import verify

    opts = ProofOptions.reference()  # main.rs:98-107
    rng = random.Random(args.seed)
    try:
        devices = _load_devices(args.data_dir, args.verbose, rng)
    except OSError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    if not devices:
        print("Error: No Device_* data found!", file=sys.stderr)
        return 1
    if args.verbose:
        print(f"→ Found {len(devices)} devices\n")

    ctx = _native.Context(args.device) if args.step != "witness" else None
    step_start = time.perf_counter()
    client_reps, total_training = [], 0

    if args.step in ("setup", "proof") and args.verbose and args.step == "setup":
        print("--- Client Training Updates ---")
    for i, dev in enumerate(devices):
        batch = _zk_batch(dev, args.bs)
        if batch is None:
            if args.verbose and args.step == "setup":
                print(f"Warning: Device {i + 1} has fewer samples than ZK batch size", file=sys.stderr)
            continue
        tp = _training_prover(opts, batch, args.bs, rng, ctx)
        if args.step == "witness":
            print(f"DEBUG: Witness step - Device {i + 1}, batch size {args.bs}")
            trace = tp.build_trace()
            print(f"DEBUG: Witness trace - length: {trace.length()}, width: {trace.width()}")
            client_reps.append(trace.get(0, trace.length() - 1))
            continue
        print(f"DEBUG: {'Device' if args.step == 'setup' else 'Proof step - Device'} {i + 1}, "
              f"batch size {args.bs}")
        t0 = time.perf_counter()
        trace = tp.build_trace()
        print(f"DEBUG: Trace dimensions - length: {trace.length()}, width: {trace.width()}")
        proof = tp.prove(trace)
        size = len(proof.to_bytes())
        total_training += size
        if args.verbose and args.step == "setup":
            print(f"Device {i + 1:>2}: ZK proof for {args.bs} samples: gen = {_ms(t0):>4}ms, size = {size} bytes")
            print(f"Training proof size: {size} bytes")
        try:
            verify(TrainingUpdateAir, proof, tp.get_pub_inputs(trace), opts)
        except _native.VerifierError as e:
            print(f"training proof failed!: {e}", file=sys.stderr)
            return 101
        client_reps.append(trace.get(0, trace.length() - 1))

    if args.step == "setup":
        t0 = time.perf_counter()
        _aggregator(opts, client_reps, rng, ctx)
        if args.verbose:
            print(f"Aggregator ready in {_ms(t0)}ms\n")
            print(f"STEP=setup: Generated {len(client_reps)} ZK proofs (bs={args.bs})")
            print(f"Total training proof size: {total_training} bytes")
    elif args.step == "witness":
        agg = _aggregator(opts, client_reps, rng, ctx)
        t0 = time.perf_counter()
        tr = agg.build_trace()
        if args.verbose:
            print(f"witness: {tr.length()} rows in {_ms(t0)}ms")
    else:
        agg = _aggregator(opts, client_reps, rng, ctx)
        t1 = time.perf_counter()
        tr = agg.build_trace()
        if args.verbose:
            print(f"trace: {tr.length()} rows in {_ms(t1)}ms")
        t2 = time.perf_counter()
        pf = agg.prove(tr)
        agg_size = len(pf.to_bytes())
        if args.verbose:
            print(f"proof: {_ms(t2)}ms, {agg_size} bytes")
            print(f"Proof size: {agg_size} bytes")
            print("verifying… ", end="")
        try:
            verify(GlobalUpdateAir, pf, agg.get_pub_inputs(tr), opts)
        except _native.VerifierError as e:
            print(f"aggregation failed!: {e}", file=sys.stderr)
            return 101
        if args.verbose:
            print("OK")
            print(f"Total training proof size: {total_training} bytes")
            print(f"Aggregation proof size: {agg_size} bytes")
            print(f"Total proof size: {total_training + agg_size} bytes")

    if args.verbose:
        print(f"\nStep '{args.step}' completed in: {_ms(step_start)}ms")
        print(f"Overall runtime: {_ms(overall)}ms")
    if ctx is not None:
        ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
