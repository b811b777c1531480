#!/bin/bash
# A/B of library variants on one box: ab.sh NAME ROUNDS VARIANT... (variant "-" = the product libpdsc.so,
# "KNOB=value" = the product library with that environment knob)
# Each run is a short bench (headline shape only); prints per-variant ms/step and attention launch ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
name=$1 rounds=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    lv=$v; knob=PDSC_AB_NONE=1; [ "$v" = "-" ] && lv=""
    case "$v" in *=*) knob=$v; lv="";; esac
    out=gpurun_out/${name}_${v}_$r.log
    env "$knob" PDSC_LIB_VARIANT=$lv timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --f32-steps 0 \
        --path-n ${PATH_N:-0} ${BENCH_ARGS} > "$out" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 "$out"; exit $rc; fi
    python3 - "$out" "$v" "$r" <<'PY'
import json, sys
t = open(sys.argv[1]).read().strip().splitlines()[-1]
d = json.loads(t)
print(f"{sys.argv[2]:>8} r{sys.argv[3]} ms/step {d['ms_per_step']:.4f} attn_launch {d['roofline']['launch_ms']*1e3:.1f} us "
      f"frac {d['roofline']['frac']:.4f} stages {json.dumps(d.get('stages_ms'))}")
PY
  done
done
