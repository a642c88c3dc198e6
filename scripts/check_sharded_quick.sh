#!/bin/bash
# Sharded-path regression check + one-rank device work (C4, C5) after a change.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py \
  tests/test_gpu_sharded_gloo.py tests/test_gpu_comm.py -k "not oracle_bytes" > gpurun_out/shq_tests.log 2>&1 \
  || { tail -30 gpurun_out/shq_tests.log; exit 1; }
tail -2 gpurun_out/shq_tests.log
bash scripts/rank_emulate.sh
