#!/bin/bash
# A/B of build_exp/b (the last commit) against the tree, 3 alternations, + quick parity.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mimc" \
  > gpurun_out/ab2_tests.log 2>&1 || { tail -30 gpurun_out/ab2_tests.log; exit 1; }
tail -1 gpurun_out/ab2_tests.log
bash scripts/ab_libs.sh build_exp/b/x/libzkp.so zk_stark_project_amd/libzkp.so
