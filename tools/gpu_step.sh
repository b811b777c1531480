#!/bin/bash
# gpu_step.sh NAME TIMEOUT CMD... : run one GPU step under its own time limit, log to
# gpurun_out/NAME.log, print its status and tail; exit non-zero (stopping the
# caller's && chain) on a crash / fault / timeout -- test failures (rc 1) too.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
name=$1 t=$2; shift 2
timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
exit $rc
