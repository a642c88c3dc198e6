#!/bin/bash
# 2^18 pass-shape A/B: 11 + 7 (256-thread 7-stage pass, adopted) vs 11 + 7 (512) vs 9 + 9, tuning only.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in kbench_ntt kbench_ntt_k7_512 kbench_ntt_t9; do
    echo "== $v round $r"
    timeout -k 10 90 ./tests/native/$v 18 || exit 1
  done
done > gpurun_out/kbench_k7.txt 2>&1
cat gpurun_out/kbench_k7.txt
