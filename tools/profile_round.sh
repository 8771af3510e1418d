#!/bin/bash
# Round evidence for bench.py (small files), written to gpurun_out/profiles/ on the GPU box (the
# directory gpurun copies back); copy them into profiles/ afterwards:
#   ${TAG}_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (graph-replayed steps)
#   ${TAG}_pmc_traffic.json   FETCH_SIZE / WRITE_SIZE passes -> HBM bytes per launch
#   ${TAG}_sq_counters.txt    SQ counter passes (MFMA busy, waits, LDS) per kernel
# Counter passes never combine --pmc with trace domains (one pass per counter group).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/profiles
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0 --train-steps 0 --no-e2e --sharded-T 0"
PMC_ARGS="$ARGS --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_trace.log 2>&1
cp "$(find gpurun_out/prof_trace -name '*kernel_stats.csv' | head -1)" $OUT/${TAG}_kernel_stats.csv
# one graph-replayed step, dispatch by dispatch (device timestamps)
python3 tools/trace_step.py gpurun_out/prof_trace $OUT/${TAG}_trace_step.json > $OUT/${TAG}_trace_step.txt
rm -f gpurun_out/prof_trace/*kernel_trace.csv
# eager HIP-event breakdown of one step (bench.py DMX_BENCH_BREAKDOWN) and the bench line of this build
DMX_BENCH_BREAKDOWN=$OUT/${TAG}_breakdown.json timeout -k 10 300 python3 bench.py --cpu-steps 0 --train-steps 0 --png-steps 0 > $OUT/${TAG}_bench_noprof.jsonl 2> gpurun_out/bench_noprof.err
echo "[profile] trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py $PMC_ARGS > gpurun_out/prof_write.log 2>&1
python3 tools/pmc_traffic.py gpurun_out/prof_fetch gpurun_out/prof_write $OUT/${TAG}_pmc_traffic.json > gpurun_out/pmc_traffic.txt
cp $OUT/${TAG}_pmc_traffic.json $OUT/pmc_traffic.json  # bench.py reads this one (lib_sha256-stamped)
echo "[profile] traffic ok"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"; do
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmc_sq$i -o run --output-format csv -- python3 bench.py $PMC_ARGS > gpurun_out/pmc_sq$i.log 2>&1
  i=$((i+1))
done
python3 tools/pmc_sq.py "igemm|wino|conv_in|attention|norm|tok_|prep|step_tail|embed" > $OUT/${TAG}_sq_counters.txt
echo "[profile] sq ok"
