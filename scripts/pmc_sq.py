"""Per-kernel SQ counter summary from scripts/pmc_profile.sh passes (gfx950).

For each kernel family: average duration (from the counter rows' timestamps),
VALU instructions per launch, VALU issue utilisation = SQ_INSTS_VALU * 4 cycles /
(duration * 2.4 GHz * 1024 SIMDs), LDS instructions, bank conflicts, waves.
Usage: python3 scripts/pmc_sq.py gpurun_out/pmc
"""
import csv
import glob
import os
import sys
from collections import defaultdict

CLOCK_GHZ = 2.4
SIMDS = 256 * 4


def fam(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    return name


def main(d):
    acc = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = fam(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            acc[k]["#" + r["Counter_Name"]] += 1
            dur[(k, r["Counter_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':44s} {'launch':>6s} {'us':>8s} {'VALU/launch':>12s} {'VALUutil':>8s} {'LDS/launch':>10s} "
          f"{'bankconf':>9s} {'waves':>8s}")
    rows = []
    for k, c in acc.items():
        n = c.get("#SQ_INSTS_VALU", 0)
        if not n:
            continue
        ds = dur[(k, "SQ_INSTS_VALU")]
        us = sum(ds) / len(ds) / 1e3
        valu = c["SQ_INSTS_VALU"] / n
        util = valu * 4 / (us * 1e3 * CLOCK_GHZ * SIMDS) if us else 0
        lds = c.get("SQ_INSTS_LDS", 0) / n
        nb = c.get("#SQ_LDS_BANK_CONFLICT", 0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0) / nb if nb else float("nan")
        waves = c.get("SQ_WAVES", 0) / n
        rows.append((us * n, k, n, us, valu, util, lds, bc, waves))
    out = {}
    for _, k, n, us, valu, util, lds, bc, waves in sorted(rows, reverse=True):
        print(f"{k[:44]:44s} {int(n):6d} {us:8.1f} {valu:12.4g} {util:8.3f} {lds:10.4g} {bc:9.4g} {waves:8.0f}")
        out[k] = {"launches": int(n), "avg_us": us, "valu_insts_per_launch": valu, "valu_issue_util": util,
                  "lds_insts_per_launch": lds, "lds_bank_conflicts_per_launch": bc, "waves_per_launch": waves}
    import json
    with open(os.path.join(d, "sq.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
