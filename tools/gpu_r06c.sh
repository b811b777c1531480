set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" knnold; do
  PDSC_LIB_VARIANT=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/knn5k_$v -o run -- python3 tools/single_pair_run.py 5000 20 > gpurun_out/knn5k_$v.log 2>&1 || exit 1
done; echo ok
for a in "5000 7000 1" "5000 7000 8"; do
  PDSC_LIB_VARIANT=knndiag timeout -k 10 120 python tools/knn_paths.py $a 2>&1 | grep -v amdgpu.ids || exit $?
done > gpurun_out/knn_paths.log
AB_SHAPES="8x5000,1x5000" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 2 - knnold > gpurun_out/ab_knn2.log 2>&1; echo ab rc=$?
