#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (HBM bytes) of a short bench.
# Usage (on the GPU box): bash tools/profile.sh <tag> [bench args...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline "$@")
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${BENCH[@]}" \
    > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -20 "$OUT/trace.log"; exit 1; }
echo "trace ok"
[ -n "$NO_PMC" ] && exit 0
for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc "$ctr" --output-format csv -d "$OUT/pmc_$ctr" -o run -- "${BENCH[@]}" \
        > "$OUT/pmc_$ctr.log" 2>&1 || { echo "pmc $ctr rc=$?"; tail -20 "$OUT/pmc_$ctr.log"; exit 1; }
    echo "pmc $ctr ok"
done
find "$OUT" -name "*.csv" | head -20
