#!/bin/bash
# Same-box interleaved A/B of the config-4 (fp16) leg: tools/ab_cfg4.sh "A_ENV" "B_ENV" [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="$1"; B="$2"; R=${3:-2}
for r in $(seq 1 $R); do
  for arm in A B; do
    envs=$([ $arm = A ] && echo "$A" || echo "$B")
    v=$(env $envs timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-steps 0 --config4-steps 100 --config5-steps 0 --legs-steps 0 --png-steps 0 --train-steps 0 --no-e2e --sharded-T 0 --no-profile 2>/dev/null | python -c "import json,sys;print(json.loads(sys.stdin.read().strip().splitlines()[-1])['config4']['value'])") || exit 1
    echo "round $r arm $arm ($envs): $v"
  done
done
