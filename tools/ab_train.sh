#!/bin/bash
# Same-box interleaved A/B of env knobs on the training step (bench.py train leg):
#   tools/ab_train.sh "A_ENV" "B_ENV" ... ; ROUNDS=2 by default; prints forward / backward ms per arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUNDS:-2}
for r in $(seq 1 $R); do
  for envs in "$@"; do
    out=$(env $envs timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-steps 0 --config4-steps 0 \
          --config5-steps 0 --legs-steps 0 --png-steps 0 --no-e2e --sharded-T 0 --no-profile --train-steps 10 2>/dev/null) || exit 1
    echo "$out" | python -c "import json,sys;t=json.loads(sys.stdin.read().strip().splitlines()[-1])['train_step'];print('round $r ($envs):', t['value'], 'img/s fwd', t['native_forward_ms'], 'bwd', t['native_backward_ms'])"
  done
done
