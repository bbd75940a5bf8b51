#!/bin/bash
# GPU: same-box A/B of the fused stride-2 transition at CIFAR size (ResNet56 @32 fused eval
# forward, tools/model_bench.py) and at 224: PO2Q_S2DS=0 runs conv1 and the shortcut separately.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python tools/model_bench.py --model resnet56 --image 32 --classes 10 --graph > gpurun_out/abs_32_on_$r.log 2>&1
  PO2Q_S2DS=0 timeout -k 10 300 python tools/model_bench.py --model resnet56 --image 32 --classes 10 --graph > gpurun_out/abs_32_off_$r.log 2>&1
done
