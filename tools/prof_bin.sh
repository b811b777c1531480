#!/bin/bash
# prof_bin.sh TAG "PMC group;PMC group" CMD... : rocprofv3 kernel trace + one pass per
# PMC group of a standalone binary (diagnostics: tools/att_w64_bench etc.), into
# gpurun_out/pb_TAG/.  Each pass under its own time limit; stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1 PM=$2; shift 2
BIN=$1; shift
case "$BIN" in /*) ;; *) BIN="$R/$BIN" ;; esac
set -- "$BIN" "$@"
OUT="$R/gpurun_out/pb_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$@" > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
IFS=';' read -ra G <<< "$PM"
i=0
for g in "${G[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/pmc_$i" -o run -- "$@" > "$OUT/pmc_$i.log" 2>&1 || { echo "pmc [$g] rc=$?"; tail -5 "$OUT/pmc_$i.log"; exit 1; }
done
echo "prof $TAG ok"
