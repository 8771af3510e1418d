#!/bin/bash
# Determinism under a concurrent second process on the same GPU (GPU box): for each arm (an env
# string) two det_check.py runs at once; prints both summaries.  tools/conc_det.sh N HW R "ARM" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=$1; HW=$2; R=$3; shift 3
for v in "$@"; do
  env $v timeout -k 10 200 python tools/det_check.py $N $HW $R > gpurun_out/dA.log 2>&1 &
  pa=$!
  env $v timeout -k 10 200 python tools/det_check.py $N $HW $R > gpurun_out/dB.log 2>&1
  rb=$?
  wait $pa
  ra=$?
  grep -ah "N=" gpurun_out/dA.log gpurun_out/dB.log
  [ $ra -ne 0 -o $rb -ne 0 ] && { echo "arm $v failed ($ra/$rb)"; tail -3 gpurun_out/dA.log gpurun_out/dB.log; exit 1; }
done
exit 0
