#!/bin/bash
# One default bench line (the driver's command) on the GPU box -> gpurun_out/b_last.json.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/b_last.json 2> gpurun_out/b_last.err || { tail -20 gpurun_out/b_last.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b_last.json").read().strip().splitlines()[-1])
rf = d["reference_flow"]
print(d["value"], d["ms_per_step"], d["step_ms"]["median"], d["roofline"]["avg_launch_ms"],
      d["c3"]["ms_per_step"], d["c3"]["step_ms"]["median"], rf["warm"]["prove_ms_total"],
      rf["training_proof_profile"]["warm_ms_per_proof"])
PY
