#!/bin/bash
# GPU: parity of the fused stride-2 + shortcut kernel and the pair kernel, then a same-box A/B
# of the bench chain with and without the fused transition (each step under its own limit).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_s2ds.py tests/test_gpu_pair.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2ds_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_s2ds_$r.log 2>&1
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-s2ds > gpurun_out/ab_nos2ds_$r.log 2>&1
done
