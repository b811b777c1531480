set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_SHAPES="1x1000,1x5000,128x1000,8x5000" AB_REPS=30 timeout -k 10 600 bash tools/fwd_ab.sh 2 - PDSC_TAIL_FUSED=0 > gpurun_out/ab_tail.log 2>&1; echo ab rc=$?
PDSC_LIB_VARIANT=stamps timeout -k 10 120 python tools/pw_stamps.py > gpurun_out/pw_stamps_tiny.log 2>&1; echo pws rc=$?
PDSC_ATT_TINY=0 PDSC_LIB_VARIANT=stamps timeout -k 10 120 python tools/pw_stamps.py > gpurun_out/pw_stamps_r06b.log 2>&1; echo pws rc=$?
