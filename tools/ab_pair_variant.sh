#!/bin/bash
# GPU: same-box A/B of the bench chain over pair-kernel variants (PO2Q_PAIR_VARIANT):
# 123 (default at C = 16: prio + nt loads + nt stores), 122 (nt loads only), 120 (plain).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
for r in 1 2; do
  for v in 123 122 120; do
    PO2Q_PAIR_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abv_${v}_$r.log 2>&1
  done
done
