#!/bin/bash
# Same-box interleaved A/B of in-tree library builds: [ROUNDS=2] tools/ab_lib.sh libA.so libB.so [libC.so ...]
# (build the arms with `python diffusion-model_amd/dmx/build.py --out libX.so -- -DKNOB=...`).
# Prints steps/s per arm and round; the last round of each arm also writes a per-launch
# breakdown to gpurun_out/bd_<lib>.json (tools/bd_compare.py compares two of them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS="$@"; R=${ROUNDS:-2}
ARGS="--steps 60 --warmup 5 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 --png-steps 0 --train-steps 0"
for r in $(seq 1 $R); do
  for lib in $LIBS; do
    bd=""
    [ $r -eq $R ] && bd="gpurun_out/bd_${lib%.so}.json"
    out=$(DMX_LIB=$lib DMX_BENCH_BREAKDOWN=$bd timeout -k 10 300 python bench.py $ARGS $([ -z "$bd" ] && echo --no-profile) 2>gpurun_out/ab_err.log) || { echo "arm $lib failed"; tail -5 gpurun_out/ab_err.log; exit 1; }
    v=$(echo "$out" | python -c "import json,sys;print(json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
    echo "round $r $lib: $v"
  done
done
