#!/bin/bash
# Per-kernel A/B of whole forwards: rocprofv3 kernel-trace stats of tools/forward_ab.py per
# library variant ("-" = the product, else PDSC_LIB_VARIANT=<it>), one pass each, and with
# PMC="..." a counter pass of each.  Usage (GPU box): [AB_SHAPES=8x5000] [PMC=FETCH_SIZE] bash tools/prof_fwd_ab.sh V...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  lv=""; [ "$v" != - ] && lv=$v
  tag=${lv:-product}
  PDSC_LIB_VARIANT=$lv timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pf_$tag -o run -- python3 $R/tools/forward_ab.py ${AB_REPS:-10} > $R/gpurun_out/pf_$tag.log 2>&1 || exit 1
  if [ -n "$PMC" ]; then
    PDSC_LIB_VARIANT=$lv timeout -k 10 180 rocprofv3 --pmc $PMC --output-format csv -d $R/gpurun_out/pfm_$tag -o run -- python3 $R/tools/forward_ab.py ${AB_REPS:-10} > $R/gpurun_out/pfm_$tag.log 2>&1 || exit 1
  fi
done
