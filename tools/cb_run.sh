set -o pipefail
timeout -k 10 120 ./tools/mfma_shape_probe > gpurun_out/mfma_shape.log 2>&1 || exit 1
for r in 1 2; do for v in old rp1 rp2 rp4; do
  for sh in "8 5000 3" "128 1000 3"; do timeout -k 10 60 ./tools/compat_bench_$v $sh | grep compat_packed | sed "s/^/$v r$r /" >> gpurun_out/cb.log || exit 1; done
done; done
