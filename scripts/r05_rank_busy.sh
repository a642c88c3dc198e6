#!/bin/bash
# Union-of-intervals device time of one emulated C4 rank, one-stream vs alternating composition LDEs
# (scripts/rank_busy.py): bash scripts/r05_rank_busy.sh <lib A> <lib B>
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in "$1" "$2"; do
  T=gpurun_out/rank_busy_$(basename $L .so)
  rm -rf $T
  ZKP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $T -o run -- \
    python3 scripts/rank_emulate.py --air mimc --world 8 --steps 4 > $T.json 2>/dev/null || exit 1
  echo "$L $(python3 scripts/rank_busy.py $T/run_kernel_trace.csv 78 4)"
done
