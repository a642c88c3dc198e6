#!/bin/bash
# Sharded-path check on one GPU: the sharded -m gpu tests (in-process group and
# two-process gloo), then the per-rank work measurement (scripts/sharded_rank_work.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py \
  tests/test_gpu_sharded_gloo.py -k "not oracle_bytes" > gpurun_out/sh_tests.log 2>&1 \
  || { tail -30 gpurun_out/sh_tests.log; exit 1; }
tail -3 gpurun_out/sh_tests.log
timeout -k 10 400 python -u scripts/sharded_rank_work.py --host > gpurun_out/rank_work.log 2>&1 \
  || { tail -30 gpurun_out/rank_work.log; exit 1; }
cat gpurun_out/rank_work.log
