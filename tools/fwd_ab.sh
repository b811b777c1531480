#!/bin/bash
# A/B of whole forwards (tools/forward_ab.py) over variants, alternating, on one box:
# fwd_ab.sh ROUNDS VARIANT...  (variant "-" = the product; "KNOB=value" = an environment
# knob, several joined by '+'; anything else = PDSC_LIB_VARIANT=<it>).  AB_SHAPES / reps as forward_ab.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    knob=PDSC_AB_NONE=1; lv=""
    case "$v" in -) ;; *=*) knob=${v//+/ };; *) lv=$v;; esac
    env $knob PDSC_LIB_VARIANT=$lv AB_TAG="$v r$r" timeout -k 10 240 python tools/forward_ab.py ${AB_REPS:-20} || exit $?
  done
done
