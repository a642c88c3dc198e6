#!/bin/bash
# GPU-box check used during development (run via gpurun from the repo root):
# the -m gpu suite, then the C2 bench line, then the C3 bench line; each step
# time-limited, stopping at the first failure. Output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
grep -E "passed|failed|PASSED.*c5|slowest" gpurun_out/t1.log | tail -5
timeout -k 10 240 python bench.py --steps 20 --stats > gpurun_out/b1.json 2> gpurun_out/b1.err || { tail -20 gpurun_out/b1.err; exit 1; }
timeout -k 10 200 python bench.py --air agg --steps 10 --no-cpu-baseline --stats > gpurun_out/b1agg.json 2> gpurun_out/b1agg.err || { tail -20 gpurun_out/b1agg.err; exit 1; }
timeout -k 10 120 python3 scripts/timeline.py > gpurun_out/timeline.txt 2>&1 || { tail -5 gpurun_out/timeline.txt; exit 1; }
echo ALLOK
