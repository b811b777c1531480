set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" knnold; do
  PDSC_LIB_VARIANT=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/knn5k_$v -o run -- python3 tools/single_pair_run.py 5000 20 > gpurun_out/knn5k_$v.log 2>&1 || exit 1
done; echo ok
AB_SHAPES="8x5000,128x1000,1x5000" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 2 - knnold > gpurun_out/ab_knnfb.log 2>&1; echo ab rc=$?
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
