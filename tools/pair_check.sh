#!/bin/bash
# GPU: pair parity tests, pair timing, HBM traffic of the default pair, and a bench run.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PO2Q_TUNE_FILE=$PWD/gpurun_out/tune.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_s2ds.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pairtests.log 2>&1
timeout -k 10 300 python tools/pair_bench.py > gpurun_out/pairb.log 2>&1
cp profiles/traffic.json gpurun_out/traffic.json
bash tools/pmc.sh "--pair --shape 16,224,16,3,1,1" tpair "conv_pair" hbm > gpurun_out/pmc_tpair.log 2>&1
python3 tools/traffic.py gpurun_out/pmc_tpair --algorithmic 1644274688 --out gpurun_out/traffic.json > gpurun_out/traffic.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
