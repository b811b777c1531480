#!/bin/bash
# A/B of the encoder halves on uniform fused batches whose workgroup count is not
# a whole number of rounds (tools/forward_ab.py; PDSC_ENC_HALVES 1 = halves on
# uniform batches too, 0 = never).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for h in 0 1; do
    PDSC_ENC_HALVES=$h AB_TAG="halves=$h r$r" AB_SHAPES="${SHAPES:-40x1000,48x1000,80x1000,96x1000,112x1000,128x1000,160x1000,192x1000}" \
      timeout -k 10 300 python tools/forward_ab.py 10 > gpurun_out/uh_${h}_$r.log 2>&1 || exit 3
    tail -1 gpurun_out/uh_${h}_$r.log
  done
done
