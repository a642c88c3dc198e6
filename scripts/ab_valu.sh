#!/bin/bash
# SQ_INSTS_VALU per kernel for two libzkp builds (tuning only): scripts/ab_valu.sh <lib A> <lib B> <tag> [bench args]
set -u
export TMPDIR=/tmp
A=$1; B=$2; TAG=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-verify --sustain-s 0 $*"
i=0
for L in "$A" "$B"; do
  OUT=$ROOT/gpurun_out/abv_${TAG}_$i
  mkdir -p $OUT
  ZKP_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU \
    --output-format csv -d $OUT/sq1 -o run -- python3 $ROOT/bench.py $ARGS > $OUT/sq1.log 2>&1 || { echo "SQ pass failed"; exit 1; }
  mkdir -p $OUT/sq && cp -r $OUT/sq1 $OUT/sq/ && python3 $ROOT/scripts/pmc_sq.py $OUT/sq > $OUT/sq.txt || exit 1
  echo "== $L"; head -12 $OUT/sq.txt
  i=$((i+1))
done
