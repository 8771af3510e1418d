#!/bin/bash
# Same-box A/B of runtime toggles: AB="VAR=a VAR=b,VAR2=c ..." runs bench once per setting
# (a setting is a comma-separated list of VAR=value), ROUNDS (default 2) times interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for kv in $AB; do
    env $(echo "$kv" | tr ',' ' ') DMX_BENCH_BREAKDOWN=gpurun_out/bd_ab$i.json timeout -k 10 300 \
      python bench.py --steps 40 --warmup 3 --cpu-steps 0 > gpurun_out/bench_ab$i.log 2>&1 || exit $?
    echo "round $round $kv: $(grep -o '"value": [0-9.]*' gpurun_out/bench_ab$i.log)"
    i=$((i+1))
  done
done
