#!/bin/bash
# Kernel traces of tools/ragged_ab.py's three legs, one rocprofv3 run per leg
# (GPU box): bash tools/prof_ragged.sh; then python tools/trace_by_grid.py gpurun_out/prag_<leg>/run_kernel_trace.csv
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
for leg in uniform padded ragged; do
  RAGGED_LEGS=$leg timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prag_$leg -o run -- python3 $R/tools/ragged_ab.py 5 > $R/gpurun_out/prag_$leg.log 2>&1 || exit 1
done
