#!/bin/bash
# One box, several steps (the box acquisition is charged): the dev loop (tests, field variants,
# bench + kernel stats), then the training-kernel PMC passes.   tools/gpu_combo.sh <tag>
R=$GRAFT_REPO_ROOT
TAG=${1:-combo}
cd $R
bash tools/gpu_dev.sh $TAG; rc=$?
[ $rc -ne 0 ] && exit $rc
cd $R
PMC_PASSES=${PMC_PASSES:-"SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_BRANCH"} \
  bash tools/gpu_train_pmc.sh ${TAG}_pmc f32
