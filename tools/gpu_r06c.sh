set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_parity.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit 1
AB_SHAPES="1x1000,1x700,2x500,1x300" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 2 - PDSC_ATT_WS=1 PDSC_ATT_WS=2 > gpurun_out/ab_ws.log 2>&1; echo ab rc=$?
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
