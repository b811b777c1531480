#!/bin/bash
# One gpurun call: the per-golden error report in both precisions, then the GPU tests.
# Stops at the first crash/fault/timeout (exit status other than 0 or 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/parity_report.py --precision both > gpurun_out/parity_both.jsonl 2> gpurun_out/parity_both.err
rc=$?; echo "parity_report rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/parity_both.err; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
exit $rc
