#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes of a short bench.
# Usage (on the GPU box): [NO_PMC=1] [PMC="ctrA ctrB;ctrC"] bash tools/profile.sh <tag> [bench args...]
# Each ';'-separated group of PMC is its own rocprofv3 pass (default: HBM bytes).
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
IFS=';' read -ra PGROUPS <<< "${PMC:-FETCH_SIZE;WRITE_SIZE}"
i=0
for grp in "${PGROUPS[@]}"; do
    i=$((i+1))
    timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_$i" -o run -- "${BENCH[@]}" \
        > "$OUT/pmc_$i.log" 2>&1 || { echo "pmc [$grp] rc=$?"; tail -20 "$OUT/pmc_$i.log"; exit 1; }
    echo "pmc [$grp] ok"
done
