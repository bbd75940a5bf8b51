#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel-trace only,
# never combined with sys/runtime traces) over tools/prof_layer.py.
# Usage: tools/pmc.sh "<prof_layer args>" [tag] [kernel regex] [all|hbm]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${1:-}
TAG=${2:-layer}
KRE=${3:-conv_x3p|conv_bf16x3}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
if [ "${4:-all}" = hbm ]; then GROUPS_=("FETCH_SIZE" "WRITE_SIZE"); fi
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "$KRE" --pmc $g --output-format csv -d "$OUT/g$i" -o run \
      -- python3 "${PMC_DRIVER:-tools/prof_layer.py}" $ARGS > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "pmc group $i rc=$rc: $g" | tee -a "$OUT/status.txt"
  if [ $rc -ge 124 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
exit 0
