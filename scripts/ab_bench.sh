# A/B device-resident timing of two libzkp builds on one box (tuning only):
#   scripts/ab_bench.sh <lib A> <lib B> [bench args]
# alternates A and B three times; prints ms_per_step / pcie_inclusive ms.
set -e
A=$1; B=$2; shift 2
for r in 1 2 3; do
  for L in "$A" "$B"; do
    out=$(ZKP_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-verify --sustain-s 0 --steps 40 "$@")
    echo "$L $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["ms_per_step"], d["pcie_inclusive"]["ms_per_proof"])')"
  done
done
