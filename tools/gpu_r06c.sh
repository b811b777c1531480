set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SHAPES="128x1000" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 3 - nobar > gpurun_out/ab_nobar.log 2>&1; echo ab rc=$?
