#!/bin/bash
# Round profile for the judged bench line (run on the GPU box, from the repo root):
#   1. rocprofv3 --kernel-trace --stats        -> per-kernel average duration
#   2. rocprofv3 --pmc FETCH_SIZE (own pass)    -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE (own pass)    -> HBM write bytes per dispatch
#   4-5. two SQ counter passes                   -> VALU issue utilisation, LDS bank conflicts
# then scripts/pmc_traffic.py folds them into gpurun_out/prof_<tag>/traffic.json.
# Usage: scripts/profile_round.sh <tag> [bench args...]
set -u
export TMPDIR=/tmp
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-verify --sustain-s 0 --no-concurrent --no-c3 --no-reference-flow --no-rank-emulation --no-tampered $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "FETCH_SIZE pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $ROOT/bench.py $ARGS > $OUT/write.log 2>&1 || { echo "WRITE_SIZE pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU \
  --output-format csv -d $OUT/sq1 -o run -- python3 $ROOT/bench.py $ARGS > $OUT/sq1.log 2>&1 || { echo "SQ pass 1 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY \
  SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq2 -o run -- python3 $ROOT/bench.py $ARGS > $OUT/sq2.log 2>&1 || { echo "SQ pass 2 failed"; exit 1; }
python3 $ROOT/scripts/pmc_traffic.py $OUT > $OUT/traffic.txt || { echo "post-processing failed"; exit 1; }
mkdir -p $OUT/sq && cp -r $OUT/sq1 $OUT/sq2 $OUT/sq/ && python3 $ROOT/scripts/pmc_sq.py $OUT/sq > $OUT/sq.txt || { echo "SQ post-processing failed"; exit 1; }
echo done
