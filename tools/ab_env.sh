#!/bin/bash
# Same-box interleaved A/B of env knobs: tools/ab_env.sh "A_ENV" "B_ENV" [rounds]
# e.g. tools/ab_env.sh "DMX_PP=1" "DMX_PP=0" 2 ; prints steps/s per arm and round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="$1"; B="$2"; R=${3:-2}
for r in $(seq 1 $R); do
  for arm in A B; do
    envs=$([ $arm = A ] && echo "$A" || echo "$B")
    v=$(env $envs timeout -k 10 300 python bench.py --steps 60 --warmup 5 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --no-profile 2>/dev/null | python -c "import json,sys;print(json.loads(sys.stdin.read())['value'])") || exit 1
    echo "round $r arm $arm ($envs): $v"
  done
done
