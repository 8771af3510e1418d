#!/bin/bash
# SQ counter passes (counters only + kernel names; no trace domains combined with --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 3 --warmup 1 --cpu-steps 0 --no-profile --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  timeout -k 10 600 rocprofv3 --pmc $set -d gpurun_out/pmc_sq$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq$i.log 2>&1 || exit $?
  echo "pass $i ok"
  i=$((i+1))
done
