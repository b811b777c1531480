set -o pipefail
for a in "5000 7000 1" "5000 7500 1" "1000 7000 1" "5000 5000 8" "1000 7 128"; do
  PDSC_LIB_VARIANT=knndiag timeout -k 10 120 python tools/knn_paths.py $a 2>&1 | grep -v amdgpu.ids || exit $?
done
