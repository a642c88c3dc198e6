"""Proofs/s on one GPU with P proofs in flight: P host threads, each with its own
zkp_ctx (own streams and buffers) proving the C2 trace from HBM back to back
(ctypes releases the GIL inside zkp_prove_device). Probe for DESIGN.md §5."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zk_stark_project_amd import _native  # noqa: E402


def main():
    air = sys.argv[1] if len(sys.argv) > 1 else "mimc"
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    ctxs = [_native.Context(0) for _ in range(4)]
    wl = bench.make_workload(air, False, None, 8, 0, ctxs[0])
    pub = wl["prover"].get_pub_inputs(wl["trace"]).to_elements()
    host = wl["trace"].data
    dts = []
    for c in ctxs:
        d = c.alloc(host.nbytes)
        c.to_device(d, host)
        dts.append(d)
    ref = None
    for c, d in zip(ctxs, dts):
        for _ in range(3):
            p, _ = c.prove_device(wl["air_id"], d, wl["width"], wl["n"], pub, wl["opts"])
        ref = ref or p
        assert p == ref
    for P in (1, 2, 3, 4, 1):
        counts = [0] * P
        stop = threading.Event()
        bad = []

        def worker(i):
            while not stop.is_set():
                p, _ = ctxs[i].prove_device(wl["air_id"], dts[i], wl["width"], wl["n"], pub, wl["opts"])
                if p != ref:
                    bad.append(i)
                counts[i] += 1
        th = [threading.Thread(target=worker, args=(i,)) for i in range(P)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        time.sleep(secs)
        stop.set()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        n = sum(counts)
        print(f"{air} in_flight={P} proofs={n} s={dt:.3f} proofs/s={n / dt:.1f} ms/proof={dt / n * 1e3:.3f} "
              f"identical={not bad}", flush=True)


if __name__ == "__main__":
    main()
