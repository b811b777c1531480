set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SHAPES="1x1000,1x1500,2x1000,4x500,1x2000,8x250" AB_REPS=40 timeout -k 10 600 bash tools/fwd_ab.sh 1 - PDSC_ATT_TINY=8 > gpurun_out/ab_tiny_rule.log 2>&1; echo ab rc=$?
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
