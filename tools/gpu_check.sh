#!/bin/bash
# One gpurun call: GPU parity tests, smoke, a short bench.  Stops at the first
# crash/fault/timeout (exit status other than 0 or 1); test failures (1) continue.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?; echo "$name rc=$rc"; tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 5 --warmup 2
