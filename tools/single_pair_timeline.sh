#!/bin/bash
# single_pair_timeline.sh TAG N : rocprofv3 kernel trace of tools/single_pair_run.py (one
# N-correspondence pair per forward, 20 forwards) -> gpurun_out/spt_TAG/ and the last
# forward's timeline in gpurun_out/spt_TAG/timeline.md.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1 N=${2:-1000}
OUT="$R/gpurun_out/spt_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/single_pair_run.py" "$N" 20 > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/single_pair_timeline.py" "$f" "single pair N=$N" > "$OUT/timeline.md" && head -5 "$OUT/timeline.md"
