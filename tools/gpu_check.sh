#!/bin/bash
# One GPU-box pass: smoke -> pytest -m gpu -> bench (+ optional rocprof).  Stops at the
# first fault / abort / timeout (exit codes other than 0 and pytest's 1 = "tests failed").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "[gpu_check] $(date) host=$(hostname)"; rocm-smi --showproductname 2>/dev/null | grep -i -E "card|series" | head -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "[gpu_check] smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf --timeout=600 ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "[gpu_check] pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
if [ -n "$BENCH" ]; then
  DMX_BENCH_BREAKDOWN=gpurun_out/breakdown.json timeout -k 10 600 python bench.py $BENCH > gpurun_out/bench.log 2>&1; rc=$?
  echo "[gpu_check] bench rc=$rc"; tail -3 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py $PROF > gpurun_out/prof.log 2>&1; rc=$?
  echo "[gpu_check] rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  [ $rc -eq 0 ] || exit $rc
fi
echo "[gpu_check] done"
