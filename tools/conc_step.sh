#!/bin/bash
# Step determinism under a concurrent second process (GPU box): per arm (env string) two
# step_det.py runs at once.  tools/conc_step.sh S HW R "ARM" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=$1; HW=$2; R=$3; shift 3
for v in "$@"; do
  env $v timeout -k 10 200 python tools/step_det.py $S $HW $R > gpurun_out/sA.log 2>&1 &
  pa=$!
  env $v timeout -k 10 200 python tools/step_det.py $S $HW $R > gpurun_out/sB.log 2>&1
  rb=$?
  wait $pa
  ra=$?
  echo "== $v"
  grep -ah "runs\|cksum" gpurun_out/sA.log gpurun_out/sB.log
  [ $ra -ne 0 -o $rb -ne 0 ] && { echo "arm $v failed ($ra/$rb)"; tail -3 gpurun_out/sA.log gpurun_out/sB.log; exit 1; }
done
exit 0
