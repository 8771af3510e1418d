#!/bin/bash
# Same-box interleaved A/B of any number of arms, each an env string (library builds via DMX_LIB):
#   [ROUNDS=2] tools/ab_arms.sh "DMX_HALO_MS=1" "DMX_HALO_MS=2" "DMX_LIB=libhead.so" ...
# Prints steps/s per arm and round; the last round also writes a per-launch breakdown of arm i to
# gpurun_out/bd_arm<i>.json (tools/ab_cmp.py compares two of them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=${ROUNDS:-2}
ARGS="--steps 60 --warmup 5 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0 --train-steps 0 --no-e2e --sharded-T 0"
for r in $(seq 1 $R); do
  i=0
  for arm in "$@"; do
    bd=""
    [ $r -eq $R ] && bd="gpurun_out/bd_arm$i.json"
    out=$(env $arm DMX_BENCH_BREAKDOWN=$bd timeout -k 10 300 python bench.py $ARGS $([ -z "$bd" ] && echo --no-profile) 2>gpurun_out/ab_err.log) || { echo "arm $arm failed"; tail -5 gpurun_out/ab_err.log; exit 1; }
    v=$(echo "$out" | python -c "import json,sys;print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
    echo "round $r arm$i ($arm): $v"
    i=$((i+1))
  done
done
