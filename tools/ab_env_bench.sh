#!/bin/bash
# Same-box interleaved A/B of environment settings on the graph-replayed config-2 step:
#   bash tools/ab_env_bench.sh ROUNDS "ENV_A" "ENV_B" ...   (each ENV_x: space-separated VAR=val, or "-")
# prints value / ms_per_step per arm and round; writes gpurun_out/ab_<arm>_<round>.json breakdowns.
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs DMX_BENCH_BREAKDOWN=gpurun_out/ab_${i}_${r}.json timeout -k 10 120 python bench.py --cpu-steps 0 --train-steps 0 --png-steps 0 --config4-steps 0 --legs-steps 0 --config5-steps 0 --no-e2e --sharded-T 0 > gpurun_out/ab_${i}_${r}.log 2>&1 || { echo "arm $i failed"; tail -3 gpurun_out/ab_${i}_${r}.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_${i}_${r}.log').read().strip().splitlines()[-1]); print('round $r arm $i [$e]', d['value'], d['ms_per_step'])"
    i=$((i+1))
  done
done
