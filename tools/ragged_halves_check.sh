set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ragged_eq.py > gpurun_out/req_default.log 2>&1 || exit 3
grep B= gpurun_out/req_default.log
PDSC_ENC_HALVES=1 timeout -k 10 300 python tools/ragged_eq.py > gpurun_out/req_all.log 2>&1 || exit 3
grep B= gpurun_out/req_all.log
timeout -k 10 600 python -m pytest tests -q -m gpu -k "ragged or forward_list or bench_parity" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ragged_tests.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/ragged_tests.log
for r in 1 2; do
  for v in PDSC_ENC_HALVES=0 PDSC_ENC_BAL=0 PDSC_ENC_BAL=1; do
    env $v RAGGED_LEGS=ragged timeout -k 10 300 python tools/ragged_ab.py 20 > gpurun_out/bal_${v}_$r.log 2>&1 || exit 3
    echo "$v r$r: $(tail -1 gpurun_out/bal_${v}_$r.log)"
  done
done
