#!/bin/bash
# GPU: pair parity, pair timing, then a same-box A/B of the bench chain: the wave-uniform inf
# check (default) against the per-value isinf guard in the pair's splits (variant 2123).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_s2ds.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pairtests.log 2>&1
timeout -k 10 300 python tools/pair_bench.py > gpurun_out/pairb.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/abg_default_$r.log 2>&1
  PO2Q_PAIR_VARIANT=2123 timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/abg_guard_$r.log 2>&1
done
