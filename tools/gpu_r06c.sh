set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SHAPES="1x1000,1x2000,1x5000,2x1000,4x1000" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 2 - PDSC_PW_PREFETCH=0 > gpurun_out/ab_pf.log 2>&1; echo ab rc=$?
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
