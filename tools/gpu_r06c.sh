set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SHAPES="1x1000,1x1024,2x500,1x700,1x300" AB_REPS=40 timeout -k 10 600 bash tools/fwd_ab.sh 2 PDSC_ATT_TINY_SLOTS=128 PDSC_ATT_TINY_SLOTS=96 PDSC_ATT_TINY_SLOTS=64 PDSC_ATT_TINY_SLOTS=32 > gpurun_out/ab_tslots2.log 2>&1; echo ab rc=$?
