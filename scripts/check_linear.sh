#!/bin/bash
# Coefficient-form linear evaluation: the GlobalUpdate/TrainingUpdate parity,
# stage and sharded GPU tests, then a C3 A/B against ZKP_EVAL_POINTWISE=1.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_stages.py tests/test_gpu_sharded.py tests/test_gpu_sharded_gloo.py -k "not oracle_bytes" \
  > gpurun_out/lin_tests.log 2>&1 || { tail -30 gpurun_out/lin_tests.log; exit 1; }
tail -2 gpurun_out/lin_tests.log
timeout -k 10 400 bash scripts/ab_env.sh ZKP_EVAL_POINTWISE=1 --air agg > gpurun_out/ab_lin.txt 2>&1 || { cat gpurun_out/ab_lin.txt; exit 1; }
cat gpurun_out/ab_lin.txt
