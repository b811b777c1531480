#!/bin/bash
# A/B of the ragged forward's encoder parts (PDSC_ENC_PARTS) on one box: ms per
# ragged / uniform forward (tools/ragged_ab.py), then the ragged GPU tests at
# the chosen count.  Usage: bash tools/parts_ab.sh "0 2 3 4" [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 "${2:-2}"); do
  for p in $1; do
    if [ "$p" = 0 ]; then env=PDSC_ENC_HALVES=0; else env=PDSC_ENC_PARTS=$p; fi
    env $env RAGGED_LEGS=ragged timeout -k 10 300 python tools/ragged_ab.py 20 > gpurun_out/parts_ab_${p}_$r.log 2>&1 || exit 3
    echo "parts=$p r$r: $(tail -1 gpurun_out/parts_ab_${p}_$r.log)"
  done
done
