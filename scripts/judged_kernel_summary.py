#!/usr/bin/env python3
"""Summary of a `rocprofv3 --kernel-trace` run of the judged bench command (profiles/):
the dominant kernel's dispatches of the headline workload, picked by shape from the
trace (the same command also runs the C3 leg, the reference flow, the session and
concurrent legs) on the headline context's stream (the stream of the first such
dispatch: the concurrent leg's three contexts overlap each other's kernels on their
own streams), and their average duration, to set beside the bench line's live
`roofline.avg_launch_ms`.
  python scripts/judged_kernel_summary.py <run_kernel_trace.csv> [bench json line file]
C2 ntt_dit = its two passes: k_ntt8<true, 256, 11, ...> dispatches with 512 position blocks
(2^20 / 2048) and k_ntt8<true, 512, 9, ...> with 256 (2^20 / 4096);
C3 ntt_dit (round 6: 11 + 7 passes at 2^18) = k_ntt8<true, 256, 11, ...> dispatches with 128 position
blocks (2^18 / 2048) and k_ntt8<true, 256, 7, ...> with 128 (2^18 / (16 groups x 128))."""
import csv
import json
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = "void (anonymous namespace)::k_ntt8<"
    fam = {"c2_ntt_dit": lambda r: (r["Kernel_Name"].startswith(k + "true, 256, 11,") and int(r["Grid_Size_Y"]) == 512)
           or (r["Kernel_Name"].startswith(k + "true, 512, 9,") and int(r["Grid_Size_Y"]) == 256),
           "c3_ntt_dit": lambda r: (r["Kernel_Name"].startswith(k + "true, 256, 11,")
                                    or r["Kernel_Name"].startswith(k + "true, 256, 7,")) and int(r["Grid_Size_Y"]) == 128}
    out = {}
    for name, pred in fam.items():
        sel = sorted((r for r in rows if pred(r)), key=lambda r: int(r["Start_Timestamp"]))
        if not sel:
            continue
        every = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
        head = sel[0]["Stream_Id"]
        sel = [r for r in sel if r["Stream_Id"] == head]
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
        by = defaultdict(list)
        for r in sel:
            if True:
                by[r["Kernel_Name"].split("::k_ntt8")[1].split("(")[0]].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        out[name] = {"stream": head, "dispatches": len(ds), "avg_ms": round(sum(ds) / len(ds), 5) if ds else None,
                     "all_streams": {"dispatches": len(every), "avg_ms": round(sum(every) / len(every), 5)},
                     "by_instance": {k: {"n": len(v), "avg_ms": round(sum(v) / len(v), 5)} for k, v in by.items()}}
    if len(sys.argv) > 2:
        line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
        c3 = line.get("c3") or {}
        lpp = (c3.get("roofline") or {}).get("launches_per_proof")
        if lpp and "c3_ntt_dit" in out:
            # the C3 leg's timed proofs alone: bench.measure() runs 1 + 2 + (W - 1) proofs
            # before its K timed ones, each with lpp ntt_dit launches; the leg's
            # trace-resident and tampered-trace proofs (larger column groups) come after
            sel = sorted((r for r in rows if fam["c3_ntt_dit"](r)), key=lambda r: int(r["Start_Timestamp"]))
            k, w, lpp = int(c3["steps"]), int(line["warmup"]), int(lpp)
            t = sel[(2 + w) * lpp:(2 + w + k) * lpp]
            ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in t]
            if ds:
                out["c3_ntt_dit"]["timed_region"] = {"dispatches": len(ds), "avg_ms": round(sum(ds) / len(ds), 5)}
        out["bench_live_avg_launch_ms"] = {"c2": line["roofline"]["avg_launch_ms"],
                                           "c3": (line.get("c3") or {}).get("roofline", {}).get("avg_launch_ms")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
