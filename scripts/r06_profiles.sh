#!/bin/bash
# Round-6 profiles (GPU box): PMC traffic + SQ passes for C2 and C3 (scripts/profile_round.sh),
# then the kernel trace (--stats) of the judged bench command itself.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/profile_round.sh r06_c2 > gpurun_out/prof_c2.out 2>&1 || { tail -5 gpurun_out/prof_c2.out; exit 1; }
bash scripts/profile_round.sh r06_c3 --air agg > gpurun_out/prof_c3.out 2>&1 || { tail -5 gpurun_out/prof_c3.out; exit 1; }
if [ "${1:-}" = "judged" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_judged -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_judged.json 2> gpurun_out/prof_judged.err || { tail -5 gpurun_out/prof_judged.err; exit 1; }
fi
echo PROFOK
