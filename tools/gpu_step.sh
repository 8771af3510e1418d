#!/bin/bash
# One GPU call = a sequence of steps, each under its own time limit; stops at the first step that
# faulted, aborted or timed out (exit 124 / 134 / 137 / 139 / >128), continues past plain test
# failures (exit 1) so the later steps still report.  Usage (on the GPU box, from the repo root):
#   tools/gpu_step.sh SECONDS LOG -- command ...   (appends "step rc=N" to gpurun_out/steps.txt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=$1; LOG=$2; shift 3
[ -f gpurun_out/.stop ] && { echo "skipped after an earlier fault: $*" >> gpurun_out/steps.txt; exit 0; }
timeout -k 10 "$T" "$@" > "gpurun_out/$LOG" 2>&1
rc=$?
echo "$LOG rc=$rc" >> gpurun_out/steps.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then touch gpurun_out/.stop; fi
exit 0
