#!/bin/bash
# r06d: GPU tests, smoke, bench and the rocprofv3 profile (kernel trace + HBM bytes + SQ counters) of the tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
PMC="FETCH_SIZE;WRITE_SIZE;SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" bash tools/profile.sh ${TAG:-r06d}
