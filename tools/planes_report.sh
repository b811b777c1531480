#!/bin/bash
# two-plane (product) vs three-plane (-DPDSC_W_PLANES=3,
# libpdsc_w3.so) 1x1-conv weights -- per golden the h3 error against the
# reference and against the exact-fp32 mode (tools/parity_report.py), and the
# bench pairs' parity block (bench.py's cpu leg runs the oracle on all 128 pairs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in w2 w3; do
  lv=""; [ "$v" = w3 ] && lv=w3
  PDSC_LIB_VARIANT=$lv timeout -k 10 300 python -u tools/parity_report.py --precision h3 > gpurun_out/planes_$v.jsonl 2> gpurun_out/planes_$v.err || { tail -20 gpurun_out/planes_$v.err; exit 1; }
  PDSC_LIB_VARIANT=$lv timeout -k 10 300 python bench.py --steps 5 --warmup 2 --f32-steps 0 --path-n 0 > gpurun_out/planes_bench_$v.log 2>&1 || { tail -20 gpurun_out/planes_bench_$v.log; exit 1; }
  echo "== $v"; tail -1 gpurun_out/planes_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'parity', json.dumps(d['parity']['h3']))"
done
