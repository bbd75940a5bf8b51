#!/bin/bash
# GPU: parity of the fused stride-2 kernel and the batched weight pack, then a same-box A/B of
# the bench chain: batched packs vs one pack launch per layer, and stage-2 pairs on top.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_s2ds.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pack_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_pack_$r.log 2>&1
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pack-batch > gpurun_out/ab_nopack_$r.log 2>&1
  PO2Q_PAIR_C32=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_packc32_$r.log 2>&1
done
