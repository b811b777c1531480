set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python tools/variant_bits.py dump gpurun_out/halves0.npz > gpurun_out/halves_bits.log 2>&1 && \
PDSC_ENC_HALVES=1 timeout -k 10 240 python tools/variant_bits.py cmp gpurun_out/halves0.npz >> gpurun_out/halves_bits.log 2>&1; echo bits rc=$?; tail -2 gpurun_out/halves_bits.log
for r in 1 2; do
  for h in 0 1; do
    PDSC_ENC_HALVES=$h RAGGED_LEGS=uniform,ragged timeout -k 10 300 python tools/ragged_ab.py 20 > gpurun_out/halves_ab_${h}_$r.log 2>&1 || exit 3
    echo "halves=$h r$r: $(tail -3 gpurun_out/halves_ab_${h}_$r.log | tr '\n' ' ')"
  done
done
PDSC_ENC_HALVES=1 timeout -k 10 600 python -m pytest tests -q -m gpu -k "ragged or bench_parity or graph" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/halves_tests.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/halves_tests.log
