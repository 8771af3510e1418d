#!/bin/bash
# SQ counter passes (3 runs) over a short bench, then the per-kernel summary for a regex:
#   tools/sq_quick.sh [regex]      (GPU box; writes gpurun_out/pmc_sq*/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sq*
ARGS="--steps 6 --warmup 2 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0 --train-steps 0 --no-e2e --sharded-T 0 --no-profile"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  timeout -k 10 200 rocprofv3 --pmc $set -d gpurun_out/pmc_sq$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq$i.log 2>&1 || exit 1
  i=$((i+1))
done
python3 tools/pmc_sq.py "${1:-wino|halo}"
