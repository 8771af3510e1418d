#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats + PMC HBM traffic (separate passes,
# counters never combined with trace domains).  Outputs under gpurun_out/prof_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 10 --warmup 2 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0"}
# counter passes serialise every dispatch: few steps, no config-4/5 side runs (per-launch averages)
PMC_ARGS=${PMC_ARGS:-"--steps 3 --warmup 1 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0 --no-profile"}
if [ -z "$SKIP_TRACE" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof_trace.log 2>&1 || exit $?
echo "[prof] trace ok"
fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS > gpurun_out/prof_fetch.log 2>&1 || exit $?
echo "[prof] fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py $PMC_ARGS > gpurun_out/prof_write.log 2>&1 || exit $?
echo "[prof] write ok"
find gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write -name "*.csv" | head -20
