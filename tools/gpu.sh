#!/bin/bash
# gpurun with waits for infrastructure-side unavailability only (status "transient": no box / backoff;
# the command did not run).  Any run that started — pass or fail — is reported once, never repeated.
#   tools/gpu.sh TIMEOUT 'command'
T=$1
shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  [ "$st" != "transient" ] && exit $rc
  echo "[gpu.sh] transient (attempt $i), waiting"
  sleep 75
done
exit $rc
