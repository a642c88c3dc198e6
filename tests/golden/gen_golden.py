"""Generate the golden fixtures in tests/golden/*.json from the pure-Python
spec restatements in spec.py (TEST INFRASTRUCTURE).

Provenance of each pin:
  * blake3.json   — "" / "abc" digests are the published BLAKE3 values
                    (SURVEY.md Appendix D); the 1025-byte vector (bytes i % 251)
                    is the published BLAKE3 test vector; other lengths come from
                    spec.py, which reproduces those published values.
  * f128.json     — Python big-int arithmetic mod p (winter-math f128 constants,
                    SURVEY.md F1: p, generator 3, two-adicity 40, root).
  * mimc.json     — src/helper.rs:25-27 (f64_to_felt), :213-233 (mimc_cipher,
                    mimc_hash_matrix), :404-406 (round constants); the bench
                    inputs of benches/bench_mimc.rs:41-45 and
                    :22-27 (StdRng = ChaCha12, restated in spec.py and pinned by
                    the RFC 8439 §2.3.2 ChaCha20 block vector);
                    the builder-defined MiMC AIR trace.
  * ntt.json      — naive O(n^2) interpolation + coset evaluation (DFT definition).
  * merkle.json   — naive MerkleTree::new over hash_elements(row) leaves.
The reference itself (Rust + un-vendored winterfell 0.12) cannot be built or
imported here, so no fixture is an output of the reference.

Run:  python tests/golden/gen_golden.py
"""
import json
import os
import random

import spec

HERE = os.path.dirname(os.path.abspath(__file__))


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1)


def main():
    rnd = random.Random(20250614)
    P = spec.P

    # ---------------------------------------------------------------- f128
    special = [0, 1, 2, P - 1, P - 2, 2**64 - 1, 2**64, 2**127, P - 2**64, 45 * 2**40, 2**128 - 1 - P]
    vals = special + [rnd.randrange(P) for _ in range(64)]
    ops = []
    for i, a in enumerate(vals):
        b = vals[(7 * i + 3) % len(vals)]
        ops.append({"a": str(a), "b": str(b), "add": str((a + b) % P), "sub": str((a - b) % P),
                    "mul": str(a * b % P), "inv_a": str(spec.inv(a)), "a_pow_b64": str(pow(a, b % 2**64, P))})
    dump("f128.json", {
        "modulus": str(P), "generator": spec.G, "two_adicity": spec.TWO_ADICITY,
        "two_adic_root": str(spec.TWO_ADIC_ROOT),
        "felt_new_u128_max": str(spec.felt_new(2**128 - 1)),
        "roots_of_unity": {str(k): str(spec.root_of_unity(k)) for k in (1, 2, 4, 8, 16, 20, 23, 40)},
        "ops": ops,
    })

    # ---------------------------------------------------------------- blake3
    vec = []
    for n in (0, 1, 2, 3, 16, 40, 63, 64, 65, 127, 128, 1023, 1024, 1025, 1920, 2048, 2049, 3072, 4080, 4096, 5000):
        d = bytes(i % 251 for i in range(n))
        vec.append({"len": n, "pattern": "i%251", "digest": spec.blake3(d).hex()})
    felt_rows = []
    for nf in (1, 4, 5, 16, 64, 65, 120, 128, 129, 192, 193, 255):
        els = [rnd.randrange(P) for _ in range(nf)]
        felt_rows.append({"felts": [str(e) for e in els], "hash_elements": spec.hash_elements(els).hex()})
    dump("blake3.json", {
        "published": {"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
                      "abc": "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85",
                      "1025_i%251_prefix": "d00278ae47eb27b34faecf67b4fe263f82d5412916c1ffd97c8cb7fb814b8444"},
        "vectors": vec, "hash_elements": felt_rows,
        "merge": {"a": bytes(range(32)).hex(), "b": bytes(range(32, 64)).hex(),
                  "out": spec.merge(bytes(range(32)), bytes(range(32, 64))).hex()},
        "merge_with_int": {"seed": bytes(range(32)).hex(), "v": 1234567,
                           "out": spec.merge_with_int(bytes(range(32)), 1234567).hex()},
    })

    # ---------------------------------------------------------------- mimc / helper
    f64 = [0.0, 1.0, 42.0, 0.5, 0.0000005, 0.0000015, 3.5, 2.1, 1e-6, -1.0, -0.5, 123456.789, 64.0]
    rcs = spec.get_round_constants()
    trace = [42 * 10**6]
    for i in range(63):
        trace.append(pow((trace[-1] + rcs[i % 64]) % P, 7, P))
    dump("mimc.json", {
        "f64_to_felt": [{"x": x, "felt": str(spec.f64_to_felt(x))} for x in f64],
        "round_constants": [str(r) for r in rcs],
        "mimc_cipher": [
            {"x": str(42 * 10**6), "rc": str(10**6), "z": "0",
             "out": str(spec.mimc_cipher(42 * 10**6, 10**6, 0))},
            {"x": "7", "rc": "11", "z": "13", "out": str(spec.mimc_cipher(7, 11, 13))},
        ],
        "mimc_hash_matrix_bench": str(spec.mimc_hash_matrix([[42 * 10**6] * 9] * 6, [10**6] * 6, rcs)),
        # benches/bench_mimc.rs:17-34: x, rc = the first two next_u64 of StdRng::from_seed([24; 32])
        # (ChaCha12 restated in spec.py, its core pinned by the RFC 8439 block vector)
        "bench_mimc_cipher": (lambda xr: {"seed_byte": 24, "x": str(xr[0]), "rc": str(xr[1]), "z": "0",
                                          "out": str(spec.mimc_cipher(xr[0], xr[1], 0))})(
            spec.stdrng_next_u64(bytes([24] * 32), 2)),
        "mimc_air_trace_x0_42e6_n64": [str(v) for v in trace],
    })

    # ---------------------------------------------------------------- ntt / lde
    cases = []
    for n, b in ((8, 2), (8, 4), (16, 4), (32, 8)):
        values = [rnd.randrange(P) for _ in range(n)]
        coeffs, lde = spec.naive_lde(values, b)
        cases.append({"n": n, "blowup": b, "values": [str(v) for v in values],
                      "coeffs": [str(c) for c in coeffs], "lde": [str(v) for v in lde]})
    dump("ntt.json", {"offset": 3, "cases": cases})

    # ---------------------------------------------------------------- merkle
    mcases = []
    for w, rows in ((1, 8), (3, 16), (120, 4)):
        cols = [[rnd.randrange(P) for _ in range(rows)] for _ in range(w)]
        leaves = [spec.hash_elements([cols[c][r] for c in range(w)]) for r in range(rows)]
        mcases.append({"w": w, "rows": rows, "cols": [[str(v) for v in c] for c in cols],
                       "root": spec.merkle_root(leaves).hex()})
    dump("merkle.json", {"cases": mcases})


if __name__ == "__main__":
    main()
