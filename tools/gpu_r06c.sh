set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
AB_SHAPES="1x1000,1x2000,1x5000,4x1000,16x1000,8x5000,128x1000" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 2 - c16old > gpurun_out/ab_c16.log 2>&1; echo ab rc=$?
