#!/bin/bash
# A/B the x3 GEMM pipeline variants on the full step (one process each, same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2}; do
  DMX_X3_PIPE=$v DMX_BENCH_BREAKDOWN=gpurun_out/bd_pipe$v.json timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-steps 0 > gpurun_out/bench_pipe$v.log 2>&1 || exit $?
  echo "variant $v: $(python -c "import json;d=json.load(open('gpurun_out/bench_pipe$v.log'.replace('.log','.log')) if False else None" 2>/dev/null)$(grep -o '"value": [0-9.]*' gpurun_out/bench_pipe$v.log)"
done
