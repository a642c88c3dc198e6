#!/bin/bash
# The whole -m gpu suite (incl. the C5 oracle-bytes test) and smoke(), each time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 \
  > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
grep -E "passed|failed|skipped" gpurun_out/full_tests.log | tail -3
grep -E "oracle_bytes" gpurun_out/full_tests.log | head -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKEOK')" > gpurun_out/smoke.log 2>&1 \
  || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
