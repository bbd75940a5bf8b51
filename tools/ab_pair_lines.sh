#!/bin/bash
# GPU: pair parity, then a same-box A/B of the bench chain: full-line pair stores (default,
# variant 123) against 64-byte half-line stores (1123).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pairtests.log 2>&1
for r in 1 2; do
  for v in 123 1123; do
    PO2Q_PAIR_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/abl_${v}_$r.log 2>&1
  done
done
