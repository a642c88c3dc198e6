#!/bin/bash
# Rows-of-16 LDS swizzle A/B (the 7-stage 256-thread passes), tuning only:
# kbench_ntt_prev16 = x ^ (q & 7), kbench_ntt_sw16 = x ^ ((q & 7) | (q2 ^ q4) << 3).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in kbench_ntt_prev16 kbench_ntt_sw16; do
    echo "== $v round $r"
    timeout -k 10 90 ./tests/native/$v 18 || exit 1
    timeout -k 10 60 ./tests/native/$v 13 tu || exit 1
    timeout -k 10 90 ./tests/native/$v 21 || exit 1
  done
done > gpurun_out/kbench_sw16.txt 2>&1
grep -E "==|DIT lde [0-9]+ cols|DIF|TU|tu" gpurun_out/kbench_sw16.txt
